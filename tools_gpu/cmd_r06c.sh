set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "native_hot_kernel or short_rows or benched_kernel_at_full_size" > gpurun_out/r06c/pytest.txt 2>&1 || { tail -30 gpurun_out/r06c/pytest.txt; exit 1; }
tail -2 gpurun_out/r06c/pytest.txt
for c in c3d30 zdt1; do bash tools_gpu/ab_lib.sh r06c/ab_$c "--config $c --steps 20 --warmup 3" pd1 pd2 || exit 1; done
for c in c2b8192 c3f32 c3d2000; do timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06c/shape_$c.out 2>&1 || exit 1; done
cat gpurun_out/r06c/ab_*/summary.txt
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
for v in "DM_PIPE_NOORDER=1" "DM_PIPE_LABEL_ROUNDS=0" "DM_PIPE_LABEL_ROUNDS=1" "DM_PIPE_LABEL_ROUNDS=2"; do
  n=${v//=/_}
  env $v timeout -k 10 200 $KT -d gpurun_out/r06c/kt_$n -- python3 bench.py --steps 10 --warmup 2 --warmup-secs 0 --no-cpu-baseline > gpurun_out/r06c/kt_$n.out 2>&1 || exit 1
done
