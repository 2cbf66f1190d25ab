# C2 bench per library variant / env: ab_c2.sh TAG
T=$1
mkdir -p gpurun_out/$T
run() {  # run NAME LIB [ENV=VAL]
  local name=$1 lib=$2; shift 2
  env DEAPMI_LIB=$lib "$@" timeout -k 10 120 python bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/$T/$name.out 2>&1 || return 1
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/$name.out) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/$T/$name.out)"
}
B=$PWD/deap_amd/libdeapmi.so
run base $B && run w7 $PWD/deap_amd/libdeapmi_w7.so && run w8 $PWD/deap_amd/libdeapmi_w8.so && run pp4 $B DM_BITS_PP4=1 && run base2 $B
