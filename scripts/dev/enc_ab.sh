#!/bin/bash
# Dev-only: microbench encode (and anything else in CASES) over several library builds,
# alternating, same box, at three densities. usage: bash scripts/dev/enc_ab.sh OUT "lib_exp/a.so lib_exp/b.so" [rounds] [cases]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$1; LIBS=$2; R=${3:-2}; CASES=${4:-encode}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in $(seq 1 "$R"); do
  ORDER=$LIBS; [ $((r % 2)) -eq 0 ] && ORDER=$REV  # ABBA: no build always runs first
  for L in $ORDER; do
    for T in 128 25 230; do
      echo "== $L thr $T round $r" >> "$OUT"
      CPK_LIB=capnp-zig_amd/$L timeout -k 10 120 python3 scripts/microbench.py --reps 15 --only "$CASES" --zero-thresh $T 2>/dev/null | tail -1 >> "$OUT" || exit 1
    done
  done
done
cat "$OUT"
