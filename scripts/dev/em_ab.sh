#!/bin/bash
# Dev-only: the one-tile message encoder (encode_message_tile1, pair gather) against the previous
# commit's (lib_exp/em_old.so): its tests, phase stamps (lib_exp/em_prof.so), then the framing
# bench leg alternating the two builds, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/em_ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -x -q --timeout 280 \
  --timeout-method thread -k "message" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
CPK_LIB=capnp-zig_amd/lib_exp/em_prof.so timeout -k 10 180 python3 scripts/dev/em_prof.py > $O/em_prof.json 2>&1
rc=$?; tail -1 $O/em_prof.json; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for lib in capnp-zig_amd/lib/libcapnp_packed.so capnp-zig_amd/lib_exp/em_old.so; do
    CPK_LIB=$lib timeout -k 10 300 python3 bench.py --only framing > $O/f.json 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/f.json; exit $rc; }
    echo "lib=$(basename $lib) $(grep '^{' $O/f.json | tail -1)"
  done
done
