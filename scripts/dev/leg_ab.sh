#!/bin/bash
# Dev-only: one bench.py side leg (--only LEG) over several library builds, ABBA order, same box.
# usage: bash scripts/dev/leg_ab.sh OUT "lib/a.so lib/b.so" ROUNDS LEG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$1; LIBS=$2; R=${3:-2}; LEG=${4:-framing}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in $(seq 1 "$R"); do
  ORDER=$LIBS; [ $((r % 2)) -eq 0 ] && ORDER=$REV
  for L in $ORDER; do
    echo "== $L $LEG round $r" >> "$OUT"
    CPK_LIB=capnp-zig_amd/$L timeout -k 10 180 python3 bench.py --only "$LEG" 2>/dev/null | tail -1 >> "$OUT" || exit 1
  done
done
cat "$OUT"
