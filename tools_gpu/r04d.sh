# PMC traffic of the C3 kernel, parent order vs pair order (separate passes).
set -o pipefail
export PMC_SETS="FETCH_SIZE WRITE_SIZE TCC_HIT_sum@TCC_MISS_sum"
bash tools_gpu/profile.sh r04d_ord --steps 5 --warmup 1 --no-cpu-baseline || exit 1
DM_PIPE_NOORDER=1 bash tools_gpu/profile.sh r04d_pair --steps 5 --warmup 1 --no-cpu-baseline || exit 1
python3 tools_gpu/pmc_summary.py gpurun_out/prof_r04d_ord gen_pipe pair_plan plan_order
python3 tools_gpu/pmc_summary.py gpurun_out/prof_r04d_pair gen_pipe pair_plan plan_order
