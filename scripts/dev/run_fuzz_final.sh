# Round 6: randomized batch fuzzing of the final tree (fused class scan), normal and big units.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fuzz_r06g
mkdir -p $O
timeout -k 10 480 python3 -u scripts/dev/fuzz_batches.py --seconds 420 --seed 81 > $O/fuzz.log 2>&1
rc=$?; tail -1 $O/fuzz.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 360 python3 -u scripts/dev/fuzz_batches.py --seconds 300 --seed 82 --big --units 5000 > $O/fuzz_big.log 2>&1
rc=$?; tail -1 $O/fuzz_big.log; exit $rc
