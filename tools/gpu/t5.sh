set -o pipefail
mkdir -p gpurun_out
bash tools/gpu/simprof.sh c3r1 c3 1 || exit 1
bash tools/gpu/simprof.sh c5r8 c5 8 || exit 1
ARGS="--config 4" bash tools/gpu/ab_args.sh "GW_RANK_SORT=12" "GW_RANK_SORT=0" "GW_RANK_SORT=12" "GW_RANK_SORT=0" || exit 1
