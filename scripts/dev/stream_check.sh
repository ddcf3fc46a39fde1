#!/bin/bash
# Dev-only: parity tests of the streaming mid decoder (-k stream), then decode timings of
# the streaming and two-pass decoders at p = 0.5 / 0.1 / 0.9 (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/stream
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_contract.py -x -q \
  --timeout 120 --timeout-method thread -k "stream" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_framer.py -x -q --timeout 600 --timeout-method thread \
  > $O/pytest_framer.log 2>&1 || { tail -40 $O/pytest_framer.log; exit 1; }
tail -2 $O/pytest_framer.log
for t in ${THRS:-128 26 230}; do
  for d in stream twopass stream twopass; do
    timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only decode --decoder $d > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
    echo "t=$t dec=$d $(tail -1 $O/x.json)"
  done
done
