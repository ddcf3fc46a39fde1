#!/bin/bash
# DEV (round 6): PMC of the words decoder, shipped tree vs the round-5 library (lib/r5_ref.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for tag in new r5; do
  OUT=gpurun_out/pmcw_$tag; mkdir -p $OUT
  [ $tag = r5 ] && export CPK_LIB=$PWD/capnp-zig_amd/lib/r5_ref.so || unset CPK_LIB
  i=0
  for set in \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
    "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
    "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
        python3 scripts/dev/dec_ab.py --decoders words --reps 1 --thr 128 > "$OUT/p$i.log" 2>&1
    rc=$?; echo "$tag pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
python3 scripts/pmc_summary.py gpurun_out/pmcw_new gpurun_out/pmcw_r5 2>&1 | grep -A1 "words\|==" 
