set -u
export TMPDIR=/tmp
O=gpurun_out/g4; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -25 $O/pytest.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for t in 128 26 230; do
  timeout -k 10 150 python3 scripts/microbench.py --only decode,decoded_size --reps 5 --zero-thresh $t > $O/mb_t$t.json 2>$O/mb_t$t.err || exit $?
  echo "t=$t $(cat $O/mb_t$t.json)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/microbench.py --only decode --reps 5 > $O/prof.log 2>&1 || exit $?
python3 scripts/kstats.py $O/prof/run_kernel_stats.csv
bash scripts/g9.sh
