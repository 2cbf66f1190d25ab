# C5 bench + kernel trace per library variant: ab_c5.sh TAG variant...
T=$1; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for v in "$@"; do
  lib=$PWD/deap_amd/libdeapmi_$v.so; [ $v = base ] && lib=$PWD/deap_amd/libdeapmi.so
  DEAPMI_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -o run -d gpurun_out/$T/kt_$v -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/$v.out 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/$v.out)"
done
