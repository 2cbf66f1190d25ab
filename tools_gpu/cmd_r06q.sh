set -o pipefail
STEPS="pytest smoke bench_c3 bench_c2 bench_c5 bench_c5x" TAG=r06fin2 bash tools_gpu/run.sh
