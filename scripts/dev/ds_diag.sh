#!/bin/bash
# Dev-only: why decode_stream_kernel is slow. Same-box decode timings of the shipped build and
# the temporal-store variant (lib_exp/ds_tst.so) with the streaming decoder at p = 0.5, then the
# PMC passes of scripts/pmc.sh on the streaming decode (stream kernel counters and HBM bytes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ds_diag
mkdir -p $O
for r in 1 2; do
  for lib in capnp-zig_amd/lib_exp/dev_decoders.so capnp-zig_amd/lib_exp/ds_tst.so; do
    CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh 128 --only decode --decoder stream > $O/x.json 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
    echo "lib=$(basename $lib) $(grep '^{' $O/x.json | tail -1)"
  done
done
CPK_LIB=capnp-zig_amd/lib_exp/dev_decoders.so bash scripts/pmc.sh ds_diag/pmc --zero-thresh 128 --only decode --decoder stream
