set -o pipefail
mkdir -p gpurun_out/r04i
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "benched_kernel" > gpurun_out/r04i/pytest.out 2>&1; rc=$?
tail -2 gpurun_out/r04i/pytest.out
[ $rc -eq 0 ] || exit $rc
DM_PIPE_PLAN_SCATTER=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "benched_kernel" > gpurun_out/r04i/pytest2.out 2>&1; rc=$?
tail -2 gpurun_out/r04i/pytest2.out
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=5 AB_GENS=8 timeout -k 10 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_PLAN_SCATTER unset 1 > gpurun_out/r04i/ab_scatter.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04i/ab_scatter.txt
AB_ROUNDS=5 AB_GENS=8 timeout -k 10 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_NOORDER unset 1 > gpurun_out/r04i/ab_order.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04i/ab_order.txt
