set -o pipefail
mkdir -p gpurun_out/r06v
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "short_rows_multiobjective" > gpurun_out/r06v/pytest.txt 2>&1 || { tail -40 gpurun_out/r06v/pytest.txt; exit 1; }
tail -12 gpurun_out/r06v/pytest.txt
