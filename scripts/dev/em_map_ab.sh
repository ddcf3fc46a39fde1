#!/bin/bash
# Dev-only: the one-tile message gather through a per-word segment map (lib_exp/em_map.so,
# CPK_EM_MAP=1) against the shipped search-based pair gather: message tests under the map
# build, then the framing leg alternating the two builds, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/em_map
mkdir -p $O
CPK_LIB=capnp-zig_amd/lib_exp/em_map.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -x -q \
  --timeout 280 --timeout-method thread -k "message" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for lib in capnp-zig_amd/lib_exp/em_map.so capnp-zig_amd/lib/libcapnp_packed.so; do
    CPK_LIB=$lib timeout -k 10 300 python3 bench.py --only framing > $O/f.json 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/f.json; exit $rc; }
    echo "lib=$(basename $lib) $(grep '^{' $O/f.json | tail -1 | cut -c1-200)"
  done
done
