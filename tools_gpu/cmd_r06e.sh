# plan-kernel ablations (profiling builds): kernel traces of C3
set -o pipefail
mkdir -p gpurun_out/r06e
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
for v in base pa1 pa2 pa3; do
  lib=$PWD/deap_amd/libdeapmi.so; [ $v != base ] && lib=$PWD/deap_amd/libdeapmi_$v.so
  env DEAPMI_LIB=$lib timeout -k 10 200 $KT -d gpurun_out/r06e/kt_$v -- python3 bench.py --steps 10 --warmup 2 --warmup-secs 0 --no-cpu-baseline > gpurun_out/r06e/kt_$v.out 2>&1 || exit 1
  python3 - gpurun_out/r06e/kt_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("dm::pair_plan", "dm::plan_", "void dm::gen_pipe", "void dm::scan")):
        print(sys.argv[2], r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
