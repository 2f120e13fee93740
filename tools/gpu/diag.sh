set -o pipefail
mkdir -p gpurun_out
ARGS="--config 4" bash tools/gpu/ab_args.sh "GW_DIAG=0" "GW_DIAG=1" "GW_DIAG=2" "GW_DIAG=0" || exit 1
