# C5 bench (no profiler) per library variant, interleaved: ab_c5b.sh TAG variant...
T=$1; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do
for v in "$@"; do
  lib=$PWD/deap_amd/libdeapmi_$v.so; [ $v = base ] && lib=$PWD/deap_amd/libdeapmi.so
  DEAPMI_LIB=$lib timeout -k 10 150 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/${v}_$rep.out 2>&1 || exit 1
  echo "$v $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/${v}_$rep.out) $(grep -o '"selection": {"ms": [0-9.]*' gpurun_out/$T/${v}_$rep.out)"
done; done
