set -o pipefail
T=${TAG:-r03l}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "nsga2 or dominance or bitset or nondominated or front or near_clone or lexicographic" tests > gpurun_out/$T/pytest.out 2>&1 || { tail -30 gpurun_out/$T/pytest.out; exit 1; }
tail -1 gpurun_out/$T/pytest.out
timeout -k 10 200 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/c5.out 2>&1 || exit 1
cut -c1-400 gpurun_out/$T/c5.out | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -o run -d gpurun_out/$T/kt_c5 -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/kt_c5.out 2>&1 || exit 1
