#!/bin/bash
# Dev: GPU tests (selected files first), then the C5 leg and headline microbench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dev}; shift
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
NOHEAD=${NOHEAD:-} bash scripts/dev/ab_c5.sh ${AB:-}
