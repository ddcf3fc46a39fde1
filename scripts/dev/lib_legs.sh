#!/bin/bash
# Dev-only: bench.py side legs (--only LEG) over several library builds, alternating, same box.
# usage: bash scripts/dev/lib_legs.sh OUT "lib_exp/a.so lib_exp/b.so" "c5 dense" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$1; LIBS=$2; LEGS=$3; R=${4:-2}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for r in $(seq 1 "$R"); do
  for L in $LIBS; do
    for G in $LEGS; do
      echo "== $L $G round $r" >> "$OUT"
      CPK_LIB=capnp-zig_amd/$L timeout -k 10 240 python3 bench.py --only "$G" 2>/dev/null | tail -1 >> "$OUT" || exit 1
    done
  done
done
cat "$OUT"
