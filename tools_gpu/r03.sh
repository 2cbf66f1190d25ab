#!/bin/bash
# Round-3 GPU-box runner.  STEPS (space separated) picks the steps, e.g.
#   STEPS="pytest smoke bench_c3" TAG=r03a tools_gpu/r03.sh
# Every GPU step runs under its own timeout; the script stops at the first
# failing step (fault / abort / timeout / test failure) and starts nothing
# more on the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -15 $OUT/$name.err; tail -15 $OUT/$name.out; exit $rc; fi
  tail -2 $OUT/$name.out | cut -c1-600
}
KT="rocprofv3 --kernel-trace --stats --output-format csv -o run"
for s in ${STEPS:-pytest smoke bench_c3}; do
  case $s in
    pytest) step pytest 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_c3) step bench_c3 400 python bench.py --steps 20 --warmup 5 ;;
    bench_c3q) step bench_c3q 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench_c2) step bench_c2 200 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline ;;
    bench_c4) step bench_c4 400 python bench.py --islands 8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench_c5) step bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2 ;;
    bench_c5q) step bench_c5q 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    bench_c5x) step bench_c5x 600 python bench.py --config c5x --steps 5 --warmup 2 ;;
    kt_c3) step kt_c3 300 $KT -d $OUT/kt_c3 -- python3 bench.py --steps 12 --warmup 2 --no-cpu-baseline ;;
    kt_c2) step kt_c2 300 $KT -d $OUT/kt_c2 -- python3 bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline ;;
    kt_c4) step kt_c4 400 $KT -d $OUT/kt_c4 -- python3 bench.py --islands 8 --steps 10 --warmup 0 --no-cpu-baseline ;;
    kt_c5) step kt_c5 400 $KT -d $OUT/kt_c5 -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_c3|pmc_c2)
      cfg=${s#pmc_}
      for pmc in FETCH_SIZE WRITE_SIZE; do
        step pmc_${cfg}_$pmc 180 rocprofv3 --pmc $pmc -d $OUT/pmc_${cfg}_$pmc -o run --output-format csv -- python3 bench.py --config $cfg --steps 6 --warmup 1 --no-cpu-baseline
      done ;;
    alloc)
      for m in torch raw contig arena; do step alloc_${m}1 240 python tools_gpu/alloc_probe.py $m 1; done
      step alloc_torch4 300 python tools_gpu/alloc_probe.py torch 4
      step alloc_arena4 300 python tools_gpu/alloc_probe.py arena 4 ;;
    counters) step counters 120 rocprofv3 -L ;;
    abnt) step ab_nt 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_NTLOAD 0 1 ;;
    abdepth) step ab_depth 300 python tools_gpu/ab_inproc.py c3 DM_PIPE_DEPTH 2 4 ;;
    c5ilp)
      step c5_ilp1 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_ilp0 300 env DEAPMI_LIB=$PWD/deap_amd/libdeapmi_ilp0.so python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    c5pb)
      step c5_pb_base 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_pb1 300 env DEAPMI_LIB=$PWD/deap_amd/libdeapmi_pb1.so python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_pb_base2 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    c5srows)
      step c5_s1 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_s0 300 env DEAPMI_LIB=$PWD/deap_amd/libdeapmi_s0.so python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_s1b 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_lexfull 300 env DM_LEX_FULL=1 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_wq0 300 env DEAPMI_LIB=$PWD/deap_amd/libdeapmi_wq0.so python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    c5ab2)
      step c5_persist 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_multi 300 env DM_PEEL_MULTI=1 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_multi_fp 300 env DM_PEEL_MULTI=1 DM_CROWD_FP=1 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    c5ab)
      step c5_t1 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_t0 300 env DEAPMI_LIB=$PWD/deap_amd/libdeapmi_t0.so python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
      step c5_multi 300 env DM_PEEL_MULTI=1 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    alloc_pair)
      for d in 0 4096 65536 262144 1048576 3145728 16777216 1073741824; do
        step alloc_pair_$d 200 python tools_gpu/alloc_probe.py pair 1 12 $d
      done
      step alloc_torch1b 200 python tools_gpu/alloc_probe.py torch 1 12
      step alloc_pair4 300 python tools_gpu/alloc_probe.py pair 4 12 0 ;;
    pmc_alloc)
      i=0
      for pmc in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_TCC_READ_REQ_LATENCY_sum" \
                 "TCP_TCC_READ_REQ_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
                 "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum"; do
        i=$((i+1))
        step pmc_alloc_$i 240 rocprofv3 --pmc $pmc -d $OUT/pmc_alloc_$i -o run --output-format csv -- python3 tools_gpu/alloc_probe.py torch 4 6
      done ;;
    c2ab)
      step c2_keys 200 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline
      step c2_nokeys 200 env DM_BITS_NOKEYS=1 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline ;;
    pmc_c2sq)
      step pmc_c2sq1 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_BUSY_CYCLES -d $OUT/pmc_c2sq1 -o run --output-format csv -- python3 bench.py --config c2 --steps 4 --warmup 1 --no-cpu-baseline
      step pmc_c2sq2 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_SMEM -d $OUT/pmc_c2sq2 -o run --output-format csv -- python3 bench.py --config c2 --steps 4 --warmup 1 --no-cpu-baseline ;;
    pmc_c5sq) step pmc_c5sq 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS -d $OUT/pmc_c5sq -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all done"
