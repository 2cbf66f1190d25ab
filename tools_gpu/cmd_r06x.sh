set -o pipefail
STEPS="pytest smoke bench_c3" TAG=r06fin5 bash tools_gpu/run.sh
