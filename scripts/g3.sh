set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-g3}; mkdir -p $O
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  CPK_DECODE_VARIANT=${VAR:-6} timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 scripts/microbench.py --reps 2 --units 262144 --only decode > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
