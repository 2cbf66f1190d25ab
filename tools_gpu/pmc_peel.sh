#!/bin/bash
# PMC passes over the C5 selection's peel kernel (one counter set per run, no
# tracing domains): issue mix, wait states, LDS activity and HBM bytes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_peel}
mkdir -p $OUT
ARGS=${ARGS:-"--config c5 --steps 1 --warmup 1 --no-cpu-baseline"}
K=${KREGEX:-peel_owned}
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$K" -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
done
python3 tools_gpu/pmc_summary.py $OUT $K > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
