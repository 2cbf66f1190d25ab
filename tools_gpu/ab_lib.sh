# bench.py per library variant, interleaved: ab_lib.sh TAG "BENCH ARGS" VARIANT...
# (a variant is deap_amd/libdeapmi_VARIANT.so; "base" = the product build)
T=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$T
run() {  # run NAME LIB
  local name=$1 lib=$2
  env DEAPMI_LIB=$lib timeout -k 10 180 python bench.py $ARGS --no-cpu-baseline > gpurun_out/$T/$name.out 2>&1 || return 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/$name.out) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/$T/$name.out | head -1)" | tee -a gpurun_out/$T/summary.txt
}
B=$PWD/deap_amd/libdeapmi.so
for r in 1 2; do
  run base$r $B || exit 1
  for v in "$@"; do run $v$r $PWD/deap_amd/libdeapmi_$v.so || exit 1; done
done
