# GPU parity suite, then the capacity A/B bench
set -o pipefail
mkdir -p gpurun_out
tag=${1:-cur}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/t_$tag.log | head -30; tail -5 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
bash tools/gpu/ab_cap.sh
