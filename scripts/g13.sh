#!/bin/bash
# C1/C5 parity tests, then the bench with the skewed (C5) leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r01f
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error|assert" "$OUT/pytest_gpu.log" | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-path --no-read-message \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['c5_skewed'])"
exit $rc
