#!/bin/bash
# Kernel-trace A/B of library variants: ab_kt.sh TAG "BENCH ARGS" VARIANT...
# (a variant is deap_amd/libdeapmi_VARIANT.so; "base" = the product build);
# per run the bench line and the rocprofv3 kernel statistics, interleaved.
T=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$T
run() {  # run NAME LIB
  local name=$1 lib=$2
  DEAPMI_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/$name -o run -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/$T/$name.out 2>&1 || return 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/$name.out)" | tee -a gpurun_out/$T/summary.txt
}
B=$PWD/deap_amd/libdeapmi.so
for r in 1 2; do
  run base$r $B || exit 1
  for v in "$@"; do run $v$r $PWD/deap_amd/libdeapmi_$v.so || exit 1; done
done
