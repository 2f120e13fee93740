# decomposed-world GPU test first (fresh process), then the full GPU suite + bench
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_dworld.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/dw_$tag.log 2>&1 || { echo "DWORLD FAILED"; tail -60 gpurun_out/dw_$tag.log; exit 1; }
tail -2 gpurun_out/dw_$tag.log
bash tools/gpu/test_bench.sh $tag
