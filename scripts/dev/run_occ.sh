set -u
O=gpurun_out/occ; mkdir -p $O
timeout -k 10 600 bash scripts/dev/enc_ab.sh $O/ab.log "lib/e4.so lib/e4_pad4096.so lib/e4_pad9984.so" 2 encode > /dev/null 2>&1 || exit $?
python3 - <<'PY'
import json
cur=None; res={}
for line in open("gpurun_out/occ/ab.log"):
    if line.startswith("=="): cur=tuple(line.split()[1:4:2])
    elif line.startswith("{"): res.setdefault(cur,[]).append(json.loads(line)["encode_ms"])
for k,v in sorted(res.items()): print(k,v)
PY
