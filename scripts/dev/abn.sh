#!/bin/bash
# Dev-only same-box A/B/…: microbench for lib_exp/{NAME…}.so and the shipped library,
# alternating, at zero-byte thresholds $THRS (default 128), $REPS rounds (default 2).
# usage: ONLY=decode THRS="26 128 230" bash scripts/dev/abn.sh NAME...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
only=${ONLY:-encode,decode}
O=gpurun_out/ab
mkdir -p $O
libs=()
for n in "$@"; do libs+=("capnp-zig_amd/lib_exp/$n.so"); done
libs+=("capnp-zig_amd/lib/libcapnp_packed.so")
for t in ${THRS:-128}; do
  for r in $(seq ${REPS:-2}); do
    for lib in "${libs[@]}"; do
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only $only ${MB_ARGS:-} > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
      echo "t=$t lib=$(basename $lib) $(tail -1 $O/x.json)"
    done
  done
done
