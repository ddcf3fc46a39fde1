set -u
export TMPDIR=/tmp
O=gpurun_out/g2; mkdir -p $O
for t in 128 26; do
CPK_DECODE_VARIANT=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v5_t$t -o run -- python3 scripts/microbench.py --only decode --reps 5 --zero-thresh $t > $O/v5_t$t.log 2>&1 || exit $?
done
find $O -name '*kernel_stats*' -exec sh -c 'echo == $1; cut -d, -f1-8 $1' _ {} \;
