# C3 parent order by index array: parity, in-process A/B, kernel trace.
set -o pipefail
mkdir -p gpurun_out/r04h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "benched_kernel or hot_kernel or c4_migration or ea_generation or trajectory" > gpurun_out/r04h/pytest.out 2>&1; rc=$?
tail -2 gpurun_out/r04h/pytest.out
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=4 AB_GENS=8 timeout -k 10 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_NOORDER unset 1 > gpurun_out/r04h/ab_order.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04h/ab_order.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04h/kt -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04h/kt.log 2>&1 || exit 1
python3 tools_gpu/pmc_summary.py gpurun_out/r04h gen_pipe pair_plan plan_order scan_ fillBuffer
