#!/bin/bash
# Dev loop for the decoder: decode parity tests, then decode timings at p = .5/.1/.9.
# Usage: bash scripts/dev/dev_decode.sh TAG [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=${1:-dev}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_side_stream.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
for t in 128 26 230; do
  timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t --only decode,copy_U --reps 7 > "$OUT/mb_t$t.json" 2> "$OUT/mb_t$t.err"
  rc=$?; echo "t$t rc=$rc $(cat $OUT/mb_t$t.json)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
