#!/bin/bash
# GPU dev loop: parity tests, then the wave-decoder phase probe at 3 densities.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dev
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/dev/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/dev/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for t in ${THRS:-26 128 230}; do
  timeout -k 10 120 ./tools/wv_probe ${UNITS:-262144} $t || exit $?
done 2>&1 | tee gpurun_out/dev/probe.log
for t in ${MB_THRS:-26 128 230}; do
  timeout -k 10 200 python3 scripts/microbench.py --only decode --zero-thresh $t --reps 5 2>/dev/null || exit $?
done | tee gpurun_out/dev/mb.log
