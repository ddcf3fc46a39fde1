#!/bin/bash
# Dev-only: the persistent prefetching one-tile message pass (CPK_EM_PF2): message tests under a
# one-block grid (every wave loops over ~55 messages) and under the resident grid, then the
# framing leg alternating with the shipped build. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/em_pf2
mkdir -p $O
for v in em_pf2_g1 em_pf2; do
  CPK_LIB=capnp-zig_amd/lib_exp/$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_configs.py -x -q \
    --timeout 180 --timeout-method thread -k "message" > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2 3; do
  for lib in capnp-zig_amd/lib_exp/em_pf2.so capnp-zig_amd/lib/libcapnp_packed.so; do
    CPK_LIB=$lib timeout -k 10 300 python3 bench.py --only framing > $O/f.json 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/f.json; exit $rc; }
    echo "lib=$(basename $lib) $(grep '^{' $O/f.json | tail -1 | cut -c1-200)"
  done
done
