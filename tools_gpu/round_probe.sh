#!/bin/bash
# GPU-box helper: HBM ceiling probe, C2 (packed-bit) kernel trace + traffic
# PMC passes, C3 SQ issue counters.  Every GPU step has its own limit; the
# first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r01d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 tools_gpu/bwtest3 > $OUT/bwtest3.txt 2>&1 || { echo "probe failed"; exit 1; }
cat $OUT/bwtest3.txt
ARGS="--config c2 --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2/kt -o run --output-format csv -- python3 bench.py $ARGS > $OUT/c2_kt.log 2>&1 || { echo "c2 kernel-trace failed"; tail -5 $OUT/c2_kt.log; exit 1; }
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/c2/pmc_$pmc -o run --output-format csv -- python3 bench.py $ARGS > $OUT/c2_pmc_$pmc.log 2>&1 || { echo "c2 pmc $pmc failed"; exit 1; }
done
python3 tools_gpu/pmc_summary.py $OUT/c2 gen_ pair_plan > $OUT/c2_pmc_summary.txt && cat $OUT/c2_pmc_summary.txt
ARGS="--config c3 --steps 10 --warmup 2 --no-cpu-baseline"
mkdir -p $OUT/c3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/c3/pmc_sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/c3_pmc_sq.log 2>&1 || { echo "c3 sq pmc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS GRBM_COUNT -d $OUT/c3/pmc_sq2 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/c3_pmc_sq2.log 2>&1 || { echo "c3 sq2 pmc failed"; exit 1; }
python3 tools_gpu/pmc_summary.py $OUT/c3 gen_ > $OUT/c3_pmc_summary.txt && cat $OUT/c3_pmc_summary.txt
