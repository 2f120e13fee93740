# decomposed world: GPU tests, router cost, 2-rank rehearsal of the world bench (gloo, one GPU)
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_dworld.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/dw_$tag.log 2>&1 || { echo "DWORLD FAILED"; tail -60 gpurun_out/dw_$tag.log; exit 1; }
tail -3 gpurun_out/dw_$tag.log
timeout -k 10 200 python -u tools/bench_router.py 8 > gpurun_out/router_$tag.log 2>&1 || { tail -30 gpurun_out/router_$tag.log; exit 1; }
cat gpurun_out/router_$tag.log
bash tools/gpu/world2.sh $tag
