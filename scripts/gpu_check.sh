#!/bin/bash
# One GPU session: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout/abort stops the script
# (test FAILURES, exit 1, still let the bench run so a number is recorded).
# Usage (from the repo root, on the GPU box): bash scripts/gpu_check.sh [tag] [pytest-args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

fatal() {  # exit codes that mean the GPU step crashed or hung
    case "$1" in 124|137|134|139|-6|-11) return 0 ;; *) return 1 ;; esac
}

echo "[gpu_check] $(date -u +%T) smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if fatal $rc; then echo "smoke crashed/hung: stopping"; exit $rc; fi

echo "[gpu_check] $(date -u +%T) pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed/hung: stopping"; exit $rc; fi

echo "[gpu_check] $(date -u +%T) bench"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
if [ $rc -ne 0 ]; then exit $rc; fi

echo "[gpu_check] $(date -u +%T) rocprofv3 kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.err"
find "$OUT/prof" -name '*stats*' | head
exit $rc
