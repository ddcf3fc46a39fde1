set -u
O=gpurun_out/ekw2; mkdir -p $O

timeout -k 10 400 bash scripts/dev/leg_ab.sh $O/c5_ab.log "lib/e4.so lib/early16k.so lib/cap16k.so" 3 c5 > /dev/null 2>&1 || exit $?
python3 - <<'PY'
import json
for f in ["gpurun_out/ekw2/c5_ab.log"]:
    cur=None; res={}
    for line in open(f):
        if line.startswith("=="): p=line.split(); cur=(p[1],p[3] if "thr" in line else "c5")
        elif line.startswith("{"):
            d=json.loads(line); d=d if "encode_ms" in d else list(d.values())[0]
            res.setdefault(cur,[]).append((d["encode_ms"], d.get("decode_ms")))
    for k,v in sorted(res.items()): print(f.split("/")[-1],k,v)
PY
