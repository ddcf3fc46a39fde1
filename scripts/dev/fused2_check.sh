#!/bin/bash
# Fused decoder (CPK_DECODE=fused) parity on the decode tests, then decode-only timings
# (scripts/microbench.py) at p = 0.5 / 0.1 / 0.9 for both decoders on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fused2}
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  CPK_DECODE=fused timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_decode_contract.py tests/test_gpu_stress.py tests/test_gpu_zig_fuzz.py tests/test_gpu_configs.py} \
      -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
for thr in ${THRS:-128 26 230}; do
  for mode in twopass fused; do
    CPK_DECODE=$mode timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $thr --only decode --reps 9 \
        > "$OUT/mb_${mode}_${thr}.json" 2> "$OUT/mb_${mode}_${thr}.err"
    rc=$?; echo "$mode thr=$thr rc=$rc $(cat $OUT/mb_${mode}_${thr}.json)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
