#!/bin/bash
# GPU-box helper: rocprofv3 kernel trace + stats, then separate PMC passes
# (counters never combined with tracing domains).  Usage: profile.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS=${@:-"--steps 10 --warmup 2 --no-cpu-baseline"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || { echo "kernel-trace failed rc=$?"; tail -20 $OUT/kt.log; exit 1; }
for pmc in ${PMC_SETS:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"}; do
  pmc=${pmc//@/ }
  name=$(echo $pmc | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $pmc -d $OUT/pmc_$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$name.log 2>&1 || { echo "pmc $pmc failed rc=$?"; tail -5 $OUT/pmc_$name.log; exit 1; }
done
echo "profile done"; find $OUT -name "*.csv" | head -20
