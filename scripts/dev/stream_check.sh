#!/bin/bash
# Dev-only: parity tests of the streaming decoder (-k stream), decode timings of the streaming
# and two-pass decoders at p = 0.5 / 0.1 / 0.9 and on C5 (same box), then the resumable framer
# tests and the rpc_framer_split leg. A test failure is reported and the next step runs; a
# crash, abort or time limit (rc > 128 or 124) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
# the streaming decoder exists in dev builds only (scripts/dev/build_all_variants.sh)
export CPK_LIB=${CPK_LIB:-capnp-zig_amd/lib_exp/dev_decoders.so}
O=gpurun_out/stream
mkdir -p $O
step() {  # name, then the command; stops the script on a crash / time limit
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
last() { grep '^{' "$1" | tail -1; }  # the step's JSON line (its rc line follows it)
[ -n "${SKIP_PARITY:-}" ] || step parity timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_contract.py tests/test_gpu_configs.py -x -q \
  --timeout 120 --timeout-method thread -k "stream or encode_message" > $O/pytest.log 2>&1
[ -n "${SKIP_PARITY:-}" ] || tail -3 $O/pytest.log
for t in ${THRS:-128 26 230}; do
  for d in stream twopass stream twopass; do
    step mb timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only decode --decoder $d > $O/x.json 2>&1
    echo "t=$t dec=$d $(last $O/x.json)"
  done
done
for d in stream twopass stream twopass; do
  step c5 timeout -k 10 200 python3 bench.py --only c5 --decoder $d > $O/c5.json 2>&1
  echo "c5 dec=$d $(last $O/c5.json)"
done
step framer timeout -k 10 600 python3 -u -m pytest tests/test_gpu_framer.py -x -q --timeout 600 --timeout-method thread \
  > $O/pytest_framer.log 2>&1
tail -3 $O/pytest_framer.log
step split timeout -k 10 300 python3 bench.py --only rpc_framer_split > $O/split.json 2>&1
last $O/split.json
