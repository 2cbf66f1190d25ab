# C2 plan + stream form (DM_BITS_SPLIT): the packed-bit parity tests with it
# on, then interleaved C2 benches, fused vs split.
T=${TAG:-c2split}
mkdir -p gpurun_out/$T
DM_BITS_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "hot_kernel or benched_kernel or bits_tournament or onemax or bits" tests > gpurun_out/$T/pytest_split.out 2>&1 || { tail -30 gpurun_out/$T/pytest_split.out; exit 1; }
tail -1 gpurun_out/$T/pytest_split.out
for rep in 1 2 3; do
  for v in fused split; do
    if [ $v = split ]; then export DM_BITS_SPLIT=1; else unset DM_BITS_SPLIT; fi
    timeout -k 10 120 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/$T/${v}_$rep.out 2>&1 || exit 1
    echo "$v $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/${v}_$rep.out) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/$T/${v}_$rep.out) $(grep -o '"frac": [0-9.]*' gpurun_out/$T/${v}_$rep.out | head -1)"
  done
done
unset DM_BITS_SPLIT
