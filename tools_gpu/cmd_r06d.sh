# C3 prelude A/B (this build vs libdeapmi_old.so) + the generation parity tests
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_knobs.py -x -q --timeout 300 --timeout-method thread -k "native_hot_kernel or short_rows or benched_kernel_at_full_size or plan_orders or knobs or generation" > gpurun_out/r06d/pytest.txt 2>&1 || { tail -30 gpurun_out/r06d/pytest.txt; exit 1; }
tail -2 gpurun_out/r06d/pytest.txt
bash tools_gpu/ab_lib.sh r06d/ab_c3 "--steps 30 --warmup 5" old || exit 1
bash tools_gpu/ab_lib.sh r06d/ab_c3b "--steps 30 --warmup 5" old || exit 1
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
timeout -k 10 200 $KT -d gpurun_out/r06d/kt_c3 -- python3 bench.py --steps 10 --warmup 2 --warmup-secs 0 --no-cpu-baseline > gpurun_out/r06d/kt_c3.out 2>&1 || exit 1
