# C3 prelude: gather jump instead of the label kernel (A/B against libdeapmi_old.so) + tests
set -o pipefail
mkdir -p gpurun_out/r06h
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_knobs.py -x -q --timeout 300 --timeout-method thread -k "plan_orders or knobs or benched_kernel_at_full_size" > gpurun_out/r06h/pytest.txt 2>&1 || { tail -30 gpurun_out/r06h/pytest.txt; exit 1; }
tail -2 gpurun_out/r06h/pytest.txt
bash tools_gpu/ab_lib.sh r06h/ab_c3 "--steps 30 --warmup 5" old || exit 1
bash tools_gpu/ab_lib.sh r06h/ab_c3b "--steps 30 --warmup 5" old || exit 1
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
timeout -k 10 200 $KT -d gpurun_out/r06h/kt_c3 -- python3 bench.py --steps 10 --warmup 2 --warmup-secs 0 --no-cpu-baseline > gpurun_out/r06h/kt_c3.out 2>&1 || exit 1
python3 - gpurun_out/r06h/kt_c3/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("dm::pair_plan", "dm::plan_", "void dm::gen_pipe", "void dm::scan")):
        print(r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 1))
PY
bash tools_gpu/cmd_r06g.sh
