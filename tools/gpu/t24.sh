set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_t24.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/t_t24.log | head -20; tail -30 gpurun_out/t_t24.log; exit 1; }
tail -1 gpurun_out/t_t24.log
ARGS="--config 4" bash tools/gpu/ab_args.sh "GW_X=0" "GW_X=0" || exit 1
ARGS="--no-config5" bash tools/gpu/ab_args.sh "GW_X=0" || exit 1
