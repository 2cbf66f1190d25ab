# C2 A/B of library variants with HBM counters: c2_ab_pmc.sh TAG VARIANT...
# timing (ab_c2.sh), then one FETCH_SIZE and one WRITE_SIZE pass per library
T=$1; shift
bash tools_gpu/ab_c2.sh $T "$@" || exit 1
for v in base "$@"; do
  lib=$PWD/deap_amd/libdeapmi_$v.so
  [ $v = base ] && lib=$PWD/deap_amd/libdeapmi.so
  for pmc in FETCH_SIZE WRITE_SIZE; do
    DEAPMI_LIB=$lib timeout -k 10 180 rocprofv3 --pmc $pmc -d gpurun_out/$T/$v/pmc_$pmc -o run --output-format csv -- python3 bench.py --config c2 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/$T/$v.pmc_$pmc.log 2>&1 || exit 1
  done
  python3 tools_gpu/pmc_summary.py gpurun_out/$T/$v gen_bits fit_key > gpurun_out/$T/pmc_$v.txt 2>&1
done
