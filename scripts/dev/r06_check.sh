#!/bin/bash
# DEV (round 6): diag, words/auto decode A/B against the round-5 library (lib/r5_ref.so, built
# from 8da5d9d by hand), the whole GPU suite and the reader leg, in one GPU call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_check; mkdir -p $O
timeout -k 10 200 python3 scripts/dev/words_diag.py 2>&1 | grep -v amdgpu.ids | head -4
timeout -k 10 300 python3 scripts/dev/dec_ab.py --decoders words,auto --reps 5 > $O/dab.log 2>&1 || exit $?
CPK_LIB=$PWD/capnp-zig_amd/lib/r5_ref.so timeout -k 10 300 python3 scripts/dev/dec_ab.py --decoders words,auto --reps 5 > $O/dab5.log 2>&1 || exit $?
tail -1 $O/dab.log; tail -1 $O/dab5.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/all.log 2>&1
r=$?; tail -6 $O/all.log
timeout -k 10 300 python3 bench.py --only read_message > $O/rm.json 2> $O/rm.err; cat $O/rm.json
exit $r
