#!/bin/bash
# Bench + profiles for one round, in this order: FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (kernel trace only) -> per-launch HBM traffic JSON -> the
# bench JSON line (which reports that traffic) -> rocprofv3 kernel-trace stats of
# the bench command. Usage: bash scripts/gpu_bench.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o bench -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-read-message --no-skewed --no-sweep --no-dense --no-c1 --no-validate --no-ceilings > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/pmc_traffic.py "$OUT" 1048576x4096_t128 profiles/pmc_traffic.json > "$OUT/pmc_traffic.json" || exit 1
export CPK_TRAFFIC_JSON="$OUT/pmc_traffic.json"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path --no-read-message --no-skewed --no-sweep --no-dense --no-c1 --no-validate --no-ceilings > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
rc=$?; echo "trace rc=$rc"
exit $rc
