#!/bin/bash
# GPU-box runner.  STEPS (space separated) picks the steps, e.g.
#   STEPS="pytest smoke bench_c3" TAG=r05k tools_gpu/run.sh
# Every GPU step runs under its own timeout; the script stops at the first
# failing step (fault / abort / timeout / test failure) and starts nothing
# more on the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -15 $OUT/$name.err; tail -15 $OUT/$name.out; exit $rc; fi
  tail -2 $OUT/$name.out | cut -c1-700
}
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
for s in ${STEPS:-pytest smoke bench_c3}; do
  case $s in
    pytest) step pytest 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_c3) step bench_c3 400 python bench.py --steps 20 --warmup 5 ;;
    bench_c3q) step bench_c3q 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench_c2) step bench_c2 200 python bench.py --config c2 --steps 100 --warmup 5 ;;
    bench_c4) step bench_c4 400 python bench.py --islands 8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench_c5) step bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2 ;;
    bench_c5q) step bench_c5q 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    bench_c5x) step bench_c5x 600 python bench.py --config c5x --steps 5 --warmup 2 ;;
    bench_c5m4) step bench_c5m4 400 python bench.py --config c5 --nobj 4 --steps 3 --warmup 2 --no-cpu-baseline ;;
    kt_c5m4) step kt_c5m4 400 $KT -d $OUT/kt_c5m4 -- python3 bench.py --config c5 --nobj 4 --steps 3 --warmup 1 --no-cpu-baseline ;;
    gap1) step gap1 200 python tools_gpu/deme_gap_probe.py 1 20 ;;
    digests)  # the one-GPU reference of the scaling runs' deme digests (profiles/deme_digests.json)
      for sw in "20 5" "50 3"; do
        set -- $sw
        for per in 1 2 4 8; do
          step digests_${per}_$1 300 python bench.py --gpus 1 --islands-per-gpu $per --steps $1 --warmup $2 --no-cpu-baseline --digests-out $OUT/deme_digests.json
        done
      done ;;
    native)  # the product loops launch library kernels only (no at::native after the marker)
      for ph in easimple c5 c5x; do
        step native_$ph 300 $KT -d $OUT/native_$ph -- python3 tools_gpu/native_free_probe.py $ph
        step native_${ph}_names 60 python3 tools_gpu/trace_names.py $OUT/native_$ph/run_kernel_trace.csv $OUT/native_$ph.json
      done ;;
    migab)  # placement cost at k = 4,096 with heavy duplicates: this library vs libdeapmi_migold.so
      for v in new old; do
        lib=$PWD/deap_amd/libdeapmi.so; [ $v = old ] && lib=$PWD/deap_amd/libdeapmi_migold.so
        export DEAPMI_LIB=$lib
        step migab_$v 300 $KT -d $OUT/migab_$v -- python3 -m pytest tests/test_gpu_islands.py -q -x -k "heavy_duplicates"
        unset DEAPMI_LIB
      done ;;
    alloc)
      for m in base mid:8 mid:16 mid:24 mid:32 mid:16 post:16 base; do
        step alloc_${m/:/_} 120 python tools_gpu/alloc_order_probe.py $m 20
        cat $OUT/alloc_${m/:/_}.out >> $OUT/alloc.jsonl
      done ;;
    gap8) step gap8 400 python tools_gpu/deme_gap_probe.py 8 20 ;;
    kt_c3) step kt_c3 300 $KT -d $OUT/kt_c3 -- python3 bench.py --steps 12 --warmup 2 --no-cpu-baseline ;;
    kt_c2) step kt_c2 300 $KT -d $OUT/kt_c2 -- python3 bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline ;;
    kt_c4) step kt_c4 400 $KT -d $OUT/kt_c4 -- python3 bench.py --islands 8 --steps 10 --warmup 0 --no-cpu-baseline ;;
    kt_c5) step kt_c5 400 $KT -d $OUT/kt_c5 -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_c3|pmc_c2)
      cfg=${s#pmc_}
      for pmc in FETCH_SIZE WRITE_SIZE; do
        step pmc_${cfg}_$pmc 180 rocprofv3 --pmc $pmc -d $OUT/pmc_${cfg}_$pmc -o run --output-format csv -- python3 bench.py --config $cfg --steps 6 --warmup 1 --no-cpu-baseline
      done ;;
    pmc_c5peel)
      step pmc_c5peel 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d $OUT/pmc_c5peel -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline
      step c5peel_json 60 python3 tools_gpu/c5_peel_pmc.py $OUT/pmc_c5peel $OUT/c5_peel_pmc.json "rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU, bench.py --config c5 (gpurun_out/$(basename $OUT))"
      mkdir -p profiles && cp $OUT/c5_peel_pmc.json profiles/c5_peel_pmc.json ;;
    shapes)  # genome shapes beside the benched ones
      for c in ${SHAPES:-c3d30 c3d2000 c3f32 c2b8192 zdt1}; do
        step shape_$c 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline
      done ;;
    kt_shapes)
      for c in ${SHAPES:-c3d30 c3d2000 c3f32 c2b8192 zdt1}; do
        step kt_$c 300 $KT -d $OUT/kt_$c -- python3 bench.py --config $c --steps 10 --warmup 2 --warmup-secs 0 --no-cpu-baseline
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
