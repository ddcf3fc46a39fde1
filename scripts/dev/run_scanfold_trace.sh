# Round 6 dev: kernel traces of the microbench (p = 0.5) with the previous and the new library,
# to measure the class pass's span (class_count start -> class_scatter end) per batch call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/scanfold_trace
mkdir -p $O
for lib in prev libcapnp_packed; do
  p=capnp-zig_amd/lib_ab/prev.so; [ $lib = libcapnp_packed ] && p=capnp-zig_amd/lib/libcapnp_packed.so
  CPK_LIB=$p timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$lib -o mb -- \
      python3 scripts/microbench.py --reps 9 --zero-thresh 128 --only encode,decode > $O/$lib.json 2> $O/$lib.err
  rc=$?; echo "$lib rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
