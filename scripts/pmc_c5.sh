#!/bin/bash
# C5 PMC for the shipped library (verdict r4 item 2): FETCH_SIZE and WRITE_SIZE of one C5 encode +
# decode step per kernel, in separate passes, plus the C5 leg's times. Usage: bash scripts/pmc_c5.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_pmc_c5}
mkdir -p "$OUT/ship"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/ship/pmc_$c" -o run -- python3 bench.py --only c5 > "$OUT/ship/pmc_$c.log" 2>&1 || exit 1
done
timeout -k 10 200 python3 bench.py --only c5 > "$OUT/c5.json" 2>/dev/null || exit 1
python3 scripts/dev/c5_fetch_summary.py "$OUT" > "$OUT/traffic.txt"
cat "$OUT/traffic.txt" "$OUT/c5.json"
