mkdir -p gpurun_out/r06k
export DEAPMI_LIB=$PWD/deap_amd/libdeapmi_prof.so
timeout -k 10 300 python3 tools_gpu/peel_phase_probe2.py c5 12 gpurun_out/r06k/phase_c5.json > gpurun_out/r06k/phase_c5.txt 2>&1 || { tail -20 gpurun_out/r06k/phase_c5.txt; exit 1; }
tail -62 gpurun_out/r06k/phase_c5.txt
