set -o pipefail
mkdir -p gpurun_out/r06f
cd /tmp && export TMPDIR=/tmp && (timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r06f/counters.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r06f/counters.txt 2>&1); cd $GRAFT_REPO_ROOT
grep -c . gpurun_out/r06f/counters.txt
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
timeout -k 10 200 $KT -d gpurun_out/r06f/kt_c3 -- python3 bench.py --steps 10 --warmup 2 --warmup-secs 0 --no-cpu-baseline > gpurun_out/r06f/kt_c3.out 2>&1 || exit 1
python3 - gpurun_out/r06f/kt_c3/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("dm::pair_plan", "dm::plan_", "void dm::gen_pipe", "void dm::scan")):
        print(r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 1))
PY
timeout -k 10 300 python3 tools_gpu/deme_gap_probe.py 4 10 > gpurun_out/r06f/gap4.txt 2>&1 || exit 1
cat gpurun_out/r06f/gap4.txt | cut -c1-300
