set -u
O=gpurun_out/e2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r=$?; tail -3 $O/pytest.log
[ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 600 bash scripts/dev/enc_ab.sh $O/ab.log "lib/base.so lib/e2.so" 3 encode > /dev/null 2>&1; r2=$?
cat $O/ab.log | grep -v "^$" | head -60
exit $r2
