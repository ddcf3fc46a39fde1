#!/bin/bash
# Dev-only: the framer walk with window tables (spec lookups for windows a message only passes
# through) against the previous commit's walk (lib_exp/fw_old.so): framer GPU tests, then the
# rpc_framer_split and rpc_framer legs alternating the two builds, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/fw_ab
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_framer.py tests/test_gpu_read_message.py -x -q --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in capnp-zig_amd/lib/libcapnp_packed.so capnp-zig_amd/lib_exp/fw_old.so; do
    for leg in rpc_framer_split rpc_framer; do
      CPK_LIB=$lib timeout -k 10 300 python3 bench.py --only $leg > $O/x.json 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -5 $O/x.json; exit $rc; }
      echo "lib=$(basename $lib) $(grep '^{' $O/x.json | tail -1 | cut -c1-700)"
    done
  done
done
