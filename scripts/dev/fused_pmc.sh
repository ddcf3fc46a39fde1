#!/bin/bash
# Dev-only: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and kernel stats of
# decode-only microbench runs under both decoders. Usage: bash scripts/dev/fused_pmc.sh TAG [thr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fused_pmc}; THR=${2:-128}
mkdir -p "$OUT"
for mode in twopass fused; do
  mkdir -p "$OUT/$mode"
  for c in FETCH_SIZE WRITE_SIZE; do
    CPK_DECODE=$mode timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/$mode/pmc_$c" -o run -- \
        python3 scripts/microbench.py --reps 2 --only decode --zero-thresh $THR > "$OUT/$mode/$c.log" 2>&1
    rc=$?; echo "$mode $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  CPK_DECODE=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$mode/trace" -o run -- \
      python3 scripts/microbench.py --reps 5 --only decode --zero-thresh $THR > "$OUT/$mode/trace.log" 2>&1
  rc=$?; echo "$mode trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/pmc_traffic.py "$OUT/$mode" "decode_$mode" /dev/null > "$OUT/$mode/traffic.json"
done
exit 0
