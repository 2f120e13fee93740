# GPU tests, then the bench without CPU baselines (N=1 incl. config #5), then a
# 2-rank world rehearsal on the one GPU over gloo.  usage: bash tools/gpu/world.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --client-msgs 0 > gpurun_out/bench_$tag.json.log 2>&1 || { tail -30 gpurun_out/bench_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_$tag.json.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --comm gloo --device 0 --steps 5 --warmup 3 --no-config5 > gpurun_out/w2_$tag.log 2>&1 || { tail -30 gpurun_out/w2_$tag.log; exit 1; }
tail -1 gpurun_out/w2_$tag.log | cut -c1-400
