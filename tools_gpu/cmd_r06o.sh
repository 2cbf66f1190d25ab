set -o pipefail
mkdir -p gpurun_out/r06o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_support.py -x -q --timeout 300 --timeout-method thread -k "dcd or statistics or stats" > gpurun_out/r06o/pytest.txt 2>&1 || { tail -30 gpurun_out/r06o/pytest.txt; exit 1; }
tail -2 gpurun_out/r06o/pytest.txt
for r in 1 2; do timeout -k 10 300 python bench.py --config c5x --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06o/c5x_$r.out 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06o/c5x_$r.out; done
