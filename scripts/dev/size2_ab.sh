#!/bin/bash
# Dev A/B: size-only walk, decode_index_kernel<true> vs size_walk_kernel<1|2> (CPK_SIZE2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-size2}
mkdir -p "$OUT"
for rep in 1 2; do
for thr in 128 26 230; do
  for v in 0 1 2; do
    CPK_SIZE2=$v timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $thr --only decoded_size --reps 9 \
        > "$OUT/mb_${v}_${thr}.json" 2> "$OUT/mb_${v}_${thr}.err"
    rc=$?; echo "size2=$v thr=$thr rc=$rc $(cat $OUT/mb_${v}_${thr}.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["decoded_size_ms"], d["size_ok"])')"
    [ $rc -ne 0 ] && exit $rc
  done
done
done
exit 0
