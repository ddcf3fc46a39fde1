#!/bin/bash
# Full GPU parity suite, encode timing at p = .5/.1/.9, bench with the C5 leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r01g
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error|assert" "$OUT/pytest_gpu.log" | tail -15
[ $rc -gt 1 ] && exit $rc
for t in 128 26 230; do
  timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t --only encode,encoded_size 2>/dev/null \
      | sed "s/^/t$t /" || exit 1
done
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-path --no-read-message \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['encode_ms'], d['decode_ms'], d['c5_skewed'])"
exit $rc
