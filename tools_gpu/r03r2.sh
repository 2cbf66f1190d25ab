# NSGA-II / dominance GPU subset, the full-size NSGA-II tests, C5 bench + trace.
T=${TAG:-r03r2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "nsga2 or dominance or bitset or nondominated or front or near_clone or crowding or dcd or full_size" tests > gpurun_out/$T/pytest.out 2>&1 || { tail -30 gpurun_out/$T/pytest.out; exit 1; }
tail -1 gpurun_out/$T/pytest.out
timeout -k 10 200 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5.out 2>&1 || exit 1
echo "c5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/c5.out)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -o run -d gpurun_out/$T/kt_c5 -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/kt_c5.out 2>&1 || exit 1
