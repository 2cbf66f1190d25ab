set -o pipefail
STEPS="pytest smoke bench_c3 bench_c2 bench_c5 bench_c5x" TAG=r06fin4 bash tools_gpu/run.sh && SHAPES="zdt1 c3d30" STEPS="shapes kt_shapes kt_c5" TAG=r06fin4 bash tools_gpu/run.sh
