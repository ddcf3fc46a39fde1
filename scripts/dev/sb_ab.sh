#!/bin/bash
# Dev-only: single-buffer calls through one kernel (launch_decode_one / launch_encode_one): the
# single-buffer, C1 and single-unit parity tests, then the crossover table at p = 0.5 for the
# shipped build and the previous commit's (lib_exp/sb_old.so), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/sb_ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_single_buffer.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -x -q --timeout 280 --timeout-method thread -k "single or c1 or kats or golden or fixture" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for lib in capnp-zig_amd/lib/libcapnp_packed.so capnp-zig_amd/lib_exp/sb_old.so; do
  CPK_LIB=$lib timeout -k 10 300 python3 scripts/crossover.py 128 > $O/x_$(basename $lib .so).json 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -3 $O/x_$(basename $lib .so).json; exit $rc; }
  echo "done $lib"
done
