#!/bin/bash
# A/B decode timings: default lib and each lib_exp/*.so given, p = .5/.1/.9. Usage: bash scripts/dev/ab.sh TAG lib1.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for lib in default "$@"; do
  for t in 128 26 230; do
    if [ "$lib" = default ]; then L=""; else L="$lib"; fi
    CPK_LIB=$L timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t --only decode --reps 7 > "$OUT/x.json" 2>/dev/null
    rc=$?; echo "$lib t$t rc=$rc $(cat $OUT/x.json)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
