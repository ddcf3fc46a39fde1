set -u
O=gpurun_out/soft; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r=$?; tail -2 $O/pytest.log
[ $r -ne 0 ] && exit $r
DECS=words,auto timeout -k 10 600 bash scripts/dev/lib_ab.sh $O/ab.log "lib/e4.so lib/soft.so" 3 > /dev/null 2>&1 || exit $?
cat $O/ab.log | cut -c1-400
timeout -k 10 200 python3 -u scripts/dev/fuzz_batches.py --seconds 90 --units 400000 --seed 11 > $O/fuzz.log 2>&1 || exit $?
tail -1 $O/fuzz.log | cut -c1-300
