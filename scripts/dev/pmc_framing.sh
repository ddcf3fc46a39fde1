#!/bin/bash
# Dev-only: SQ counters and HBM bytes of the framing leg (bench.py --only framing): the fused
# message encoder beside encode_kernel on the same framed bytes (toBytes copy + encode_batch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_framing
mkdir -p "$OUT"
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py --only framing > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
