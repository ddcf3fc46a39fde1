#!/bin/bash
# Fill-pass grid sweep, alone (variant 6) and overlapped with the index passes (variant 7).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in 6 7; do
  for b in 2 3 4 5; do
    CPK_FILL_BLOCKS_PER_CU=$b CPK_DECODE_VARIANT=$v timeout -k 10 120 python3 scripts/microbench.py \
        --zero-thresh 128 --only decode 2>/dev/null | sed "s/^/v$v b$b /" || exit 1
  done
done
