set -o pipefail
mkdir -p gpurun_out/r06y
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/r06y/pmc_lds -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --warmup-secs 0 --no-cpu-baseline > gpurun_out/r06y/pmc.out 2>&1 || { tail -20 gpurun_out/r06y/pmc.out; exit 1; }
echo done
