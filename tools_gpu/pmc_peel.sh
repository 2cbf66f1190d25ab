# PMC passes over the fixed-input selNSGA2 probe (one pass per counter group).
T=${1:-r03r}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
           "TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/$T/pmc_$i -o run --output-format csv -- python3 tools_gpu/c5_dom_probe.py 2 > gpurun_out/$T/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/$T/pmc_$i.log; }
done
echo done
