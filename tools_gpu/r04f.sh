# C3 plan order A/B in one process: pair order, parent order with a run per
# wave, parent order with a run per workgroup (waves interleaved).
set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "benched_kernel" > gpurun_out/r04f/pytest.out 2>&1; rc=$?
tail -2 gpurun_out/r04f/pytest.out
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=4 AB_GENS=8 timeout -k 10 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_ORDER_MODE 0 1 > gpurun_out/r04f/ab_mode.txt 2>&1 || exit 1
cat gpurun_out/r04f/ab_mode.txt | grep -v amdgpu.ids
AB_ROUNDS=4 AB_GENS=8 timeout -k 10 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_NOORDER unset 1 > gpurun_out/r04f/ab_order.txt 2>&1 || exit 1
cat gpurun_out/r04f/ab_order.txt | grep -v amdgpu.ids
