#!/bin/bash
# Dev-only: PMC passes over the C5 skewed leg (bench.py --only c5); kernels run
# serialised under --pmc. Usage: bash scripts/dev/pmc_c5.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_c5}
mkdir -p "$OUT"
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py --only c5 --steps 2 --warmup 1 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) echo "stopping"; exit $rc ;; esac
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --only c5 --steps 5 --warmup 1 > "$OUT/trace.log" 2>&1
echo "trace rc=$?"
