#!/bin/bash
# Dev-only: alternate dec_ab.py (words decoder) over several library builds, same box.
# usage: bash scripts/dev/lib_ab.sh OUT "lib_exp/a.so lib_exp/b.so ..." [rounds] [dec_ab args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$1; LIBS=$2; R=${3:-2}; shift 3 || shift $#
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for r in $(seq 1 "$R"); do
  for L in $LIBS; do
    echo "== $L round $r" >> "$OUT"
    CPK_LIB=capnp-zig_amd/$L timeout -k 10 240 python3 scripts/dev/dec_ab.py --decoders ${DECS:-words} --reps 5 "$@" 2>/dev/null | tail -1 >> "$OUT" || exit 1
  done
done
cat "$OUT"
