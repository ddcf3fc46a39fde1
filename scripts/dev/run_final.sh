# Round 6 final-tree validation: smoke + GPU suite + bench + full trace (gpu_check), then the PMC +
# bench + headline-only trace (gpu_bench), then C5 PMC. One GPU call; stops at the first crash.
set -u
T=${1:-r06c}
bash scripts/gpu_check.sh $T || exit $?
bash scripts/gpu_bench.sh ${T}_pmc || exit $?
timeout -k 10 600 bash scripts/pmc_c5.sh ${T}_pmc_c5 > /dev/null 2>&1 || exit $?
tail -30 gpurun_out/${T}_pmc_c5/traffic.txt
