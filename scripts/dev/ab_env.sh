#!/bin/bash
# A/B decode timings under environment settings, p = .5/.1/.9, plus decoded_size.
# Usage: bash scripts/dev/ab_env.sh TAG "ENV=1" ...   ("-" = no setting)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for e in "$@"; do
  for t in 128 26 230; do
    if [ "$e" = "-" ]; then E=""; else E="$e"; fi
    env $E timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t --only decode,decoded_size --reps 7 > "$OUT/x.json" 2>/dev/null
    rc=$?; echo "[$e] t$t rc=$rc $(cat $OUT/x.json)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
