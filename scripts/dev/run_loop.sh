set -u
O=gpurun_out/loop; mkdir -p $O
CPK_LIB=capnp-zig_amd/lib/loop4.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_stress.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r=$?; tail -2 $O/pytest.log
[ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 400 bash scripts/dev/enc_ab.sh $O/enc_ab.log "lib/e4.so lib/loop4.so lib/loop16.so" 2 encode > /dev/null 2>&1 || exit $?
timeout -k 10 400 bash scripts/dev/leg_ab.sh $O/c5_ab.log "lib/e4.so lib/loop4.so lib/loop16.so" 2 c5 > /dev/null 2>&1 || exit $?
python3 - <<'PY'
import json
for f in ["gpurun_out/loop/enc_ab.log","gpurun_out/loop/c5_ab.log"]:
    cur=None; res={}
    for line in open(f):
        if line.startswith("=="): p=line.split(); cur=(p[1],p[3] if "thr" in line else "c5")
        elif line.startswith("{"):
            d=json.loads(line); d=d if "encode_ms" in d else list(d.values())[0]
            res.setdefault(cur,[]).append((d["encode_ms"], d.get("decode_ms")))
    for k,v in sorted(res.items()): print(f.split("/")[-1],k,v)
PY
