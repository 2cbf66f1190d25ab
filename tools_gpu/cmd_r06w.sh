set -o pipefail
mkdir -p gpurun_out/r06w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "nsga2 or nondominated or dominance or crowd or front or short_rows" > gpurun_out/r06w/pytest.txt 2>&1 || { tail -40 gpurun_out/r06w/pytest.txt; exit 1; }
tail -2 gpurun_out/r06w/pytest.txt
bash tools_gpu/ab_lib.sh r06w/ab_c5 "--config c5 --steps 5 --warmup 2 --warmup-secs 0" old || exit 1
bash tools_gpu/ab_lib.sh r06w/ab_c5b "--config c5 --steps 5 --warmup 2 --warmup-secs 0" old || exit 1
