#!/bin/bash
# Fused single-pass decoder vs the indexed two-pass decoder on one box:
# decode parity tests first (fused = library default), then decode-only timings
# (scripts/microbench.py) at p = 0.5 / 0.1 / 0.9 under both CPK_DECODE settings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fused_ab}
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
      tests/test_gpu_decode_contract.py tests/test_gpu_small_units.py tests/test_gpu_side_stream.py \
      tests/test_gpu_long_windows.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
for thr in 128 26 230; do
  for mode in twopass fused; do
    CPK_DECODE=$mode timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $thr --only decode --reps 9 \
        > "$OUT/mb_${mode}_${thr}.json" 2> "$OUT/mb_${mode}_${thr}.err"
    rc=$?; echo "$mode thr=$thr rc=$rc $(cat $OUT/mb_${mode}_${thr}.json)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
