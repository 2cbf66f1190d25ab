#!/bin/bash
# PMC passes (one counter set per run, no tracing domains) over a short C5 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_c5}
mkdir -p $OUT
ARGS=${ARGS:-"--config c5 --steps 1 --warmup 1"}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
done
python3 tools_gpu/pmc_summary.py $OUT ${KFILTER:-sym_dom} > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
