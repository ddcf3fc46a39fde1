# Round 6 dev: the workspace-head memset folded into class_scan_kernel. GPU suite on the new
# library, then an alternating microbench A/B against lib_ab/prev.so (the previous build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/memfold
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for t in 128 230; do
  for r in 1 2 3; do
    for lib in capnp-zig_amd/lib_ab/prev.so capnp-zig_amd/lib/libcapnp_packed.so; do
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only encode,decode > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
      echo "t=$t lib=$(basename $lib) $(tail -1 $O/x.json)" | tee -a $O/ab.txt
    done
  done
done
