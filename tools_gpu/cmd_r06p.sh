set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "short_rows or native_hot_kernel or eamupluslambda or mu_plus or nsga2_example or var_or" > gpurun_out/r06p/pytest.txt 2>&1 || { tail -30 gpurun_out/r06p/pytest.txt; exit 1; }
tail -2 gpurun_out/r06p/pytest.txt
for c in zdt1 c3d30; do timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06p/shape_$c.out 2>&1 || exit 1; python3 -c "
import json
d=json.loads(open('gpurun_out/r06p/shape_$c.out').read().strip().splitlines()[-1])
print('$c', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
