#!/bin/bash
# Dev-only: C5 leg time and per-kernel FETCH/WRITE for several library builds (same box).
# usage: bash scripts/dev/c5_fetch_ab.sh TAG "lib_exp/a.so lib_exp/b.so"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=$1; LIBS=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for L in $LIBS; do
  N=$(basename "$L" .so)
  export CPK_LIB=capnp-zig_amd/$L
  mkdir -p "$OUT/$N"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/$N/pmc_$c" -o run -- python3 bench.py --only c5 > "$OUT/$N/pmc_$c.log" 2>&1 || exit 1
  done
done
bash scripts/dev/lib_legs.sh "$OUT/legs.log" "$LIBS" c5 2 > /dev/null || exit 1
python3 scripts/dev/c5_fetch_summary.py "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
