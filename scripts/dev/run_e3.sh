set -u
O=gpurun_out/e5; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r=$?; tail -3 $O/pytest.log
[ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 500 bash scripts/dev/enc_ab.sh $O/framing_ab.log "lib/e4.so lib/e5.so" 3 encode > /dev/null 2>&1 || exit $?
timeout -k 10 300 bash scripts/dev/leg_ab.sh $O/c5_ab.log "lib/e4.so lib/e5.so" 3 c5 > /dev/null 2>&1 || exit $?
python3 - <<'PY'
import json,re
for f in ["gpurun_out/e5/framing_ab.log","gpurun_out/e5/c5_ab.log"]:
    cur=None
    for line in open(f):
        if line.startswith("=="): cur=" ".join(line.split()[1:3])
        elif line.startswith("{"):
            d=json.loads(line); d=d if "encode_ms" in d else list(d.values())[0]
            print(f.split("/")[-1], cur, {k:d[k] for k in d if k.endswith("_ms")})
PY
