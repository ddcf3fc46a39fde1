set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5p
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c5p/calib -o run -- ./scripts/dev/fetch_calib > gpurun_out/c5p/calib.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5p/trace -o run -- python3 bench.py --only c5 > gpurun_out/c5p/trace.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d gpurun_out/c5p/pmc_$c -o run -- python3 bench.py --only c5 > gpurun_out/c5p/pmc_$c.log 2>&1 || exit 1
done
