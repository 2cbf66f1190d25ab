# C2 bench per library variant / env: ab_c2.sh TAG VARIANT...
# (a variant is a library deap_amd/libdeapmi_VARIANT.so; "base" = the product build)
T=$1; shift
mkdir -p gpurun_out/$T
run() {  # run NAME LIB [ENV=VAL]
  local name=$1 lib=$2; shift 2
  env DEAPMI_LIB=$lib "$@" timeout -k 10 120 python bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/$T/$name.out 2>&1 || return 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/$name.out) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/$T/$name.out)" | tee -a gpurun_out/$T/summary.txt
}
B=$PWD/deap_amd/libdeapmi.so
run base $B || exit 1
for v in "$@"; do run $v $PWD/deap_amd/libdeapmi_$v.so || exit 1; done
run base2 $B || exit 1
for v in "$@"; do run ${v}2 $PWD/deap_amd/libdeapmi_$v.so || exit 1; done
