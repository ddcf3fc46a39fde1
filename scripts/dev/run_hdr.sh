set -u
O=gpurun_out/hdr; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r=$?; tail -2 $O/pytest.log
[ $r -ne 0 ] && exit $r
timeout -k 10 500 bash scripts/dev/leg_ab.sh $O/rm_ab.log "lib/prev.so lib/hdr.so" 4 read_message > /dev/null 2>&1 || exit $?
grep -o '"ms": [0-9.]*\|"bit_exact": [a-z]*\|== lib/[a-z]*.so' $O/rm_ab.log | paste - - - 
