set -o pipefail
tag=${1:-r03ah}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_boundary.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
bash tools/gpu/abtrees.sh $tag "3 4" prev || exit 1
