set -o pipefail
# M = 4 on the bitset tables once more, after the count kernel moved the fourth
# objective's tables out of LDS (73,992 B, the three-objective footprint)
OUT=gpurun_out/r06m4b
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
DM_BD_M4=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "nsga2_matches_reference or sort_nondominated or dominance_paths or bitset_dominance or nsga2_at_full_size or sel_nsga2_at_full or dtlz1-4 or evolved_c5" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
DM_BD_M4=1 timeout -k 10 300 python bench.py --config c5 --nobj 4 --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_c5m4_bitset.out 2>&1 || { tail -20 $OUT/bench_c5m4_bitset.out; exit 1; }
tail -1 $OUT/bench_c5m4_bitset.out | cut -c1-700
timeout -k 10 300 python bench.py --config c5 --nobj 4 --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_c5m4_compare.out 2>&1 || { tail -20 $OUT/bench_c5m4_compare.out; exit 1; }
tail -1 $OUT/bench_c5m4_compare.out | cut -c1-700
DM_BD_M4=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $OUT/kt_c5m4_bitset -- python3 bench.py --config c5 --nobj 4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/kt.out 2>&1 || { tail -20 $OUT/kt.out; exit 1; }
echo "== done"
