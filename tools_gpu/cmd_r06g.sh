# rocprofv3 per-instance counter syntax probe (short program, each pass under its own kill timer)
mkdir -p gpurun_out/r06g
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for spec in 'TCC_EA0_RDREQ[0]' 'TCC_EA0_RDREQ[0,0]'; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc "$spec" -d $R/gpurun_out/r06g/p$i -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --warmup-secs 0 --no-cpu-baseline > $R/gpurun_out/r06g/p$i.log 2>&1
  echo "spec $spec rc=$?"; tail -3 $R/gpurun_out/r06g/p$i.log | cut -c1-300
  ls $R/gpurun_out/r06g/p$i 2>/dev/null | head
done
