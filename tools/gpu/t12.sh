set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_t12.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/t_t12.log | head -20; tail -30 gpurun_out/t_t12.log; exit 1; }
tail -1 gpurun_out/t_t12.log
ARGS="--no-config5" bash tools/gpu/ab_args.sh "GW_RANK_SORT=12" "GW_RANK_SORT=12" || exit 1
bash tools/gpu/sim.sh s12 c5 || exit 1
ARGS="--config 4" bash tools/gpu/ab_args.sh "GW_RANK_SORT=12" || exit 1
