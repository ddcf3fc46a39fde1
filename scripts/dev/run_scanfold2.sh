# Round 6 dev: the fused class scan, second form (loads beside the unit metadata, one scan per
# class). GPU suite, short fuzz, then kernel traces of the microbench with both libraries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/scanfold2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u scripts/dev/fuzz_batches.py --seconds 60 --seed 71 > $O/fuzz.log 2>&1
rc=$?; tail -1 $O/fuzz.log; [ $rc -ne 0 ] && exit $rc
for lib in prev libcapnp_packed prev libcapnp_packed; do
  p=capnp-zig_amd/lib_ab/prev.so; [ $lib = libcapnp_packed ] && p=capnp-zig_amd/lib/libcapnp_packed.so
  CPK_LIB=$p timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${lib}_$RANDOM -o mb -- \
      python3 scripts/microbench.py --reps 9 --zero-thresh 128 --only encode,decode >> $O/$lib.json 2>> $O/$lib.err
  rc=$?; echo "$lib rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
