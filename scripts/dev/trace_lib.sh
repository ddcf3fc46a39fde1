#!/bin/bash
# Dev-only: C5 kernel timeline (rocprofv3 kernel trace) for each lib_exp/NAME.so and the shipped library.
# usage: bash scripts/dev/trace_lib.sh NAME...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for n in "$@" shipped; do
  lib=capnp-zig_amd/lib_exp/$n.so; [ $n = shipped ] && lib=capnp-zig_amd/lib/libcapnp_packed.so
  O=gpurun_out/tr_$n; mkdir -p $O
  CPK_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
      python3 bench.py --only c5 --steps 5 --warmup 1 > $O/log 2>&1 || { echo "$n rc=$?"; tail -5 $O/log; exit 1; }
  echo "== $n"; python3 scripts/dev/timeline.py $O/run_kernel_trace.csv | tail -12
done
