# C5: PMC pass for the peel's VALU instructions per selection, then the bench line.
set -o pipefail
mkdir -p gpurun_out/r04g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/r04g/pmc -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04g/pmc.log 2>&1 || { tail -5 gpurun_out/r04g/pmc.log; exit 1; }
python3 tools_gpu/c5_peel_pmc.py gpurun_out/r04g/pmc gpurun_out/r04g/c5_peel_pmc.json "rocprofv3 --pmc, bench.py --config c5, round 4 (gpurun_out/r04g)" || exit 1
mkdir -p profiles && cp gpurun_out/r04g/c5_peel_pmc.json profiles/c5_peel_pmc.json
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04g/bench_c5.json 2> gpurun_out/r04g/bench_c5.err || exit 1
cat gpurun_out/r04g/bench_c5.json
