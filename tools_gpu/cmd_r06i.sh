mkdir -p gpurun_out/r06i
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 --help > $R/gpurun_out/r06i/help.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc 'select(TCC_EA0_RDREQ,[DIMENSION_INSTANCE=[0]])' -d $R/gpurun_out/r06i/p1 -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --warmup-secs 0 --no-cpu-baseline > $R/gpurun_out/r06i/p1.log 2>&1
echo rc=$?
ls -R $R/gpurun_out/r06i/p1 2>/dev/null | head
