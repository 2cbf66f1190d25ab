# m = 4 on the bitset path (DM_BD_MAXM=4), serialized kernels, one process:
# the golden NSGA-II cases (case 4 is m = 4), then the m = 4 bitset tests.
mkdir -p gpurun_out/r03m4
export DM_BD_MAXM=4 AMD_SERIALIZE_KERNEL=3
timeout -k 10 120 python tools_gpu/golden_nsga2_probe.py 4 0 1 2 3 5 > gpurun_out/r03m4/probe.out 2>&1; echo "probe rc=$?"
grep -v amdgpu.ids gpurun_out/r03m4/probe.out | tail -20
