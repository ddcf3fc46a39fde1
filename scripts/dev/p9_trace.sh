set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/dev/dec_ab.py --decoders twopass,words --thr 230 --reps 5 > gpurun_out/p9_ab.json 2>/dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p9tr -o run -- python3 scripts/dev/dec_ab.py --decoders twopass --thr 230 --reps 3 > gpurun_out/p9tr.log 2>&1 || exit 1
