set -u
export TMPDIR=/tmp
O=gpurun_out/u5
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for t in 128 26 230; do
timeout -k 10 120 python3 scripts/microbench.py --reps 7 --zero-thresh $t --only encode,decode,decoded_size > $O/mb_$t.json 2>&1 || exit $?
tail -1 $O/mb_$t.json
done
