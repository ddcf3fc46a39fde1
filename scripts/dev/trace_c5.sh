#!/bin/bash
# Dev: kernel trace of the C5 leg (bench.py --only c5), for the per-call timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-trace_c5}
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --only c5 --steps 5 --warmup 1 > "$OUT/trace.log" 2>&1
echo "trace rc=$?"; tail -2 "$OUT/trace.log"
