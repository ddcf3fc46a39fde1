#!/bin/bash
# Dev loop for the two-pass decoder: parity tests, timings, per-kernel split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dev
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/dev/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/dev/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for t in ${THRS:-26 128 230}; do
  CPK_DECODE_VARIANT=${V:-5} timeout -k 10 200 python3 scripts/microbench.py --only decode --zero-thresh $t --reps 5 2>/dev/null || exit $?
done | cut -c1-110
CPK_DECODE_VARIANT=${V:-5} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dev/prof -o run -- \
    python3 scripts/microbench.py --only decode --reps 3 > gpurun_out/dev/prof.log 2>&1 || exit $?
f=$(find gpurun_out/dev/prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'cpk::' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
"
