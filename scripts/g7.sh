set -u
export TMPDIR=/tmp
O=gpurun_out/g7; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "indexed" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for b in ${BLKS:-64 128}; do
for t in 128 26 230; do
  CPK_IX_BLK=$b timeout -k 10 100 python3 scripts/microbench.py --only decoded_size,decode --reps 5 --zero-thresh $t > $O/x.json 2>/dev/null || exit $?
  echo "blk=$b t=$t $(cat $O/x.json)"
done
done
