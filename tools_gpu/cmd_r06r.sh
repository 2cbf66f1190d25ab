set -o pipefail
STEPS="kt_c3 kt_c5 pmc_c3 shapes kt_shapes" TAG=r06fin3 bash tools_gpu/run.sh
