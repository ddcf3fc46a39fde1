set -u
O=gpurun_out/li; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_words_adversarial.py tests/test_gpu_parity.py tests/test_gpu_read_message.py tests/test_gpu_stress.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r=$?; tail -2 $O/pytest.log
[ $r -ne 0 ] && exit $r
DECS=words,auto timeout -k 10 600 bash scripts/dev/lib_ab.sh $O/ab.log "lib/prev.so lib/li.so" 3 --thr 128,26,230 > /dev/null 2>&1 || exit $?
python3 - <<'PY'
import json
cur=None
for line in open("gpurun_out/li/ab.log"):
    if line.startswith("=="): cur=line.split()[1]
    elif line.startswith("{"):
        d=json.loads(line); print(cur, {k:(v["ms"],v["bit_exact"]) for k,v in d.items()})
PY
timeout -k 10 200 python3 -u scripts/dev/fuzz_batches.py --seconds 60 --units 400000 --seed 41 > $O/fuzz.log 2>&1 || exit $?
tail -1 $O/fuzz.log | cut -c1-300
