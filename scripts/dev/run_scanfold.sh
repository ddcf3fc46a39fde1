# Round 6 dev: class_scan folded into class_scatter for batches of <= 1M units. GPU suite and
# fuzz on the new library, then an alternating microbench A/B against lib_ab/prev.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/scanfold
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python3 -u scripts/dev/fuzz_batches.py --seconds 90 --seed 61 > $O/fuzz.log 2>&1
rc=$?; tail -1 $O/fuzz.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python3 -u scripts/dev/fuzz_batches.py --seconds 90 --seed 62 --big --units 5000 > $O/fuzz_big.log 2>&1
rc=$?; tail -1 $O/fuzz_big.log; [ $rc -ne 0 ] && exit $rc
for t in 128 230; do
  for r in 1 2 3; do
    for lib in capnp-zig_amd/lib_ab/prev.so capnp-zig_amd/lib/libcapnp_packed.so; do
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only encode,decode > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
      echo "t=$t lib=$(basename $lib) $(tail -1 $O/x.json)" | tee -a $O/ab.txt
    done
  done
done
