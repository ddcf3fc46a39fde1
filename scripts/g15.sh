#!/bin/bash
# GPU parity suite, then decode timing at p = .5/.1/.9 (default decoder).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r01h}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error|assert" "$OUT/pytest_gpu.log" | tail -15
[ $rc -gt 1 ] && exit $rc
for t in 128 26 230; do
  timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t --only decode 2>/dev/null | sed "s/^/t$t /" || exit 1
done
