set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread -k "nsga2 or nondominated or crowd or front or dtlz or sel_nsga or dominance or segmented" > gpurun_out/r06l/pytest.txt 2>&1 || { tail -30 gpurun_out/r06l/pytest.txt; exit 1; }
tail -2 gpurun_out/r06l/pytest.txt
bash tools_gpu/ab_lib.sh r06l/ab_c5 "--config c5 --steps 5 --warmup 2 --warmup-secs 0" old || exit 1
bash tools_gpu/ab_lib.sh r06l/ab_c5b "--config c5 --steps 5 --warmup 2 --warmup-secs 0" old || exit 1
export DEAPMI_LIB=$PWD/deap_amd/libdeapmi_prof.so
timeout -k 10 300 python3 tools_gpu/peel_phase_probe2.py c5 12 gpurun_out/r06l/phase_c5.json > gpurun_out/r06l/phase_c5.txt 2>&1 || { tail -20 gpurun_out/r06l/phase_c5.txt; exit 1; }
tail -3 gpurun_out/r06l/phase_c5.txt
