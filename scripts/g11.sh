#!/bin/bash
# GPU parity suite, then decoder timing: indexed (6) vs stream (4) decoders at p = .5/.1/.9.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r01e
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" "$OUT/pytest_gpu.log" | tail -15
[ $rc -gt 1 ] && exit $rc
for v in 6 7; do
  for t in 128 26 230; do
    CPK_DECODE_VARIANT=$v timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t \
        --only decode 2>/dev/null | sed "s/^/v$v t$t /" || exit 1
  done
done
