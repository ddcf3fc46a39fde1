#!/bin/bash
# Decoder development loop on the GPU box: parity tests, then decode timings per
# variant and density. Every GPU step has its own limit; a crash stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/dev
mkdir -p "$OUT"
fatal() { case "$1" in 124|137|134|139) return 0 ;; *) return 1 ;; esac; }

echo "[dev] $(date -u +%T) pytest -m gpu"
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then exit $rc; fi

for v in ${VARIANTS:-0 2}; do
  for thr in ${THRS:-26 128 230}; do
    echo "[dev] variant=$v thr=$thr"
    CPK_DECODE_VARIANT=$v timeout -k 10 300 python3 scripts/microbench.py --zero-thresh $thr --only decode${EXTRA_ONLY:-} --reps 7 \
        > "$OUT/mb_v${v}_t${thr}.json" 2> "$OUT/mb_v${v}_t${thr}.err"
    rc=$?; cat "$OUT/mb_v${v}_t${thr}.json"; tail -3 "$OUT/mb_v${v}_t${thr}.err"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
