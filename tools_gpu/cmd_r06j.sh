# per-channel HBM request counters of gen_pipe_kernel on fast / slow demes (placement)
mkdir -p gpurun_out/r06j
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
Y=$R/tools_gpu/tcc_channels.yaml
chs() { local s=""; for c in $(seq 0 15); do s="$s DM_$1_CH$c"; done; echo $s; }
xcs() { local s=""; for c in $(seq 0 7); do s="$s DM_$1_XCC$c"; done; echo $s; }
i=0
for set in "$(chs RD)" "$(chs WR)" "$(chs RDSTALL)" "$(xcs RD) $(xcs WR)"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 -E $Y --pmc $set --kernel-include-regex gen_pipe -d $R/gpurun_out/r06j/p$i -o run --output-format csv -- python3 $R/tools_gpu/placement_pmc_probe.py 4 4 > $R/gpurun_out/r06j/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"; grep -v "^W2026\|^I2026\|^E2026" $R/gpurun_out/r06j/p$i.log | tail -3 | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
done
exit 0
