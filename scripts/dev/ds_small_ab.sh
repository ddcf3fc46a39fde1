#!/bin/bash
# Dev-only: the streaming decoder on the small units only (lib_exp/ds_small.so: CPK_DEV_DECODERS=1
# CPK_DS_SMALL=1; mid units two-pass): stream-decoder tests under it, then C5 alternating with
# the shipped two-pass path (decode_small_kernel for the small units), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ds_small
mkdir -p $O
CPK_LIB=capnp-zig_amd/lib_exp/ds_small.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_decode_contract.py tests/test_gpu_configs.py tests/test_gpu_stress.py tests/test_gpu_small_units.py \
  -x -q --timeout 300 --timeout-method thread -k "stream" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  CPK_LIB=capnp-zig_amd/lib_exp/ds_small.so timeout -k 10 200 python3 bench.py --only c5 --decoder stream > $O/c5.json 2>&1 || exit 1
  echo "ds_small $(grep '^{' $O/c5.json | cut -c1-300)"
  timeout -k 10 200 python3 bench.py --only c5 > $O/c5.json 2>&1 || exit 1
  echo "shipped  $(grep '^{' $O/c5.json | cut -c1-300)"
done
