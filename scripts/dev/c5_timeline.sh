#!/bin/bash
# Dev-only: kernel timeline of one C5 encode + decode (bench --only c5 under a kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c5tl}
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --only c5 > "$OUT/run.log" 2>&1 || exit 1
python3 scripts/dev/timeline.py "$OUT/trace/run_kernel_trace.csv" 40 > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"
