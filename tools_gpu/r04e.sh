set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_islands_mp.py tests/test_gpu_islands.py > gpurun_out/r04e/pytest.out 2>&1; rc=$?
tail -3 gpurun_out/r04e/pytest.out
[ $rc -eq 0 ] || exit $rc
bash tools_gpu/r04d.sh
