set -u
export TMPDIR=/tmp
O=gpurun_out/g1; mkdir -p $O
for t in 128 26 230; do
 for v in 4 5 0; do
  CPK_DECODE_VARIANT=$v timeout -k 10 150 python3 scripts/microbench.py --only decode,decoded_size,encode,copy_U --reps 5 --zero-thresh $t > $O/mb_v${v}_t$t.json 2>$O/mb_v${v}_t$t.err || exit $?
  echo "v=$v t=$t $(cat $O/mb_v${v}_t$t.json)"
 done
done
