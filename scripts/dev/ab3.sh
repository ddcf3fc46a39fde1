#!/bin/bash
# Dev-only same-box A/B/C: microbench for lib_exp/{A,B}.so and the shipped library, alternating.
# usage: bash scripts/dev/ab3.sh A B [only]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
only=${3:-encode,decode}
O=gpurun_out/ab
mkdir -p $O
for t in ${THRS:-128}; do
  for r in 1 2; do
    for lib in "capnp-zig_amd/lib_exp/$1.so" "capnp-zig_amd/lib_exp/$2.so" "capnp-zig_amd/lib/libcapnp_packed.so"; do
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only $only > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
      echo "t=$t lib=$(basename $lib) $(tail -1 $O/x.json)"
    done
  done
done
