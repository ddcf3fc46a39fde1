# DEV (round 6): C5 kernel timeline, and the words decoder's last-generation tail (1M units
# = 5.33 resident grids of decode_words_kernel vs 983,040 = exactly 5)
set -u
O=gpurun_out/probe; mkdir -p $O
timeout -k 10 240 bash scripts/dev/c5_timeline.sh probe/c5tl > $O/c5tl.log 2>&1 || exit $?
for u in 983040 1048576 786432 819200; do
  timeout -k 10 200 python3 scripts/dev/dec_ab.py --decoders words --units $u --thr 128 --reps 7 2>/dev/null | tail -1 > $O/tail_$u.json || exit $?
  echo "$u $(cat $O/tail_$u.json)"
done
tail -45 $O/c5tl/timeline.txt
DECS=auto timeout -k 10 600 bash scripts/dev/lib_ab.sh $O/noside_ab.log "lib/e4.so lib/noside.so" 3 --thr 128,230 > /dev/null 2>&1 || exit $?
cat $O/noside_ab.log
