set -u
O=gpurun_out/probe2; mkdir -p $O
timeout -k 10 400 bash scripts/dev/leg_ab.sh $O/c5_ab.log "lib/e4.so lib/cap16k.so" 3 c5 > /dev/null 2>&1 || exit $?
grep -o '"encode_ms": [0-9.]*, "decode_ms": [0-9.]*' $O/c5_ab.log | paste - - - - - - ; grep "==" $O/c5_ab.log | tr '\n' ' '
