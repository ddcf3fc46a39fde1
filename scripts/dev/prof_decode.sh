#!/bin/bash
# Diagnostic: decode/encode kernel timings + SQ PMC passes (kernel trace only, one
# counter set per pass). Usage: bash scripts/dev/prof_decode.sh TAG [microbench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=${1:-prof}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for t in ${DENS:-128 26 230}; do
  timeout -k 10 120 python3 scripts/microbench.py --zero-thresh $t "$@" > "$OUT/mb_t$t.json" 2> "$OUT/mb_t$t.err"
  rc=$?; echo "microbench t$t rc=$rc"; cat "$OUT/mb_t$t.json"
  [ $rc -ne 0 ] && exit $rc
done
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAVES" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
      python3 scripts/microbench.py --reps 2 --only ${ONLY:-decode,encode,decoded_size} "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 scripts/pmc_summary.py "$OUT"
exit 0
