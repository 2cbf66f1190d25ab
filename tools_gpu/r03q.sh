# Full GPU suite, then the C2 split A/B (tools_gpu/c2_split.sh), then C5 bench + trace.
T=${TAG:-r03q}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/$T/pytest.out 2>&1 || { tail -30 gpurun_out/$T/pytest.out; exit 1; }
tail -1 gpurun_out/$T/pytest.out
TAG=$T bash tools_gpu/c2_split.sh || exit 1
timeout -k 10 200 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5.out 2>&1 || exit 1
echo "c5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/c5.out)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -o run -d gpurun_out/$T/kt_c5 -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/kt_c5.out 2>&1 || exit 1
