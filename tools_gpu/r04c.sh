# C3 parent-ordered plans: parity of the benched kernel, then an in-process
# A/B against pair order, then the bench line.
set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "benched_kernel or hot_kernel or c4_migration or ea_generation or trajectory" > gpurun_out/r04c/pytest.out 2>&1; rc=$?
tail -3 gpurun_out/r04c/pytest.out
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=4 AB_GENS=8 timeout -k 10 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_NOORDER unset 1 > gpurun_out/r04c/ab.txt 2>&1 || exit 1
cat gpurun_out/r04c/ab.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04c/bench_c3.json 2> gpurun_out/r04c/bench_c3.err || exit 1
cat gpurun_out/r04c/bench_c3.json
