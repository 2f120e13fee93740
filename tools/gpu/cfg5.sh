# config #5 (16M uniform world): N=1 on the one GPU, then a 2-rank gloo rehearsal sharing it
set -o pipefail
mkdir -p gpurun_out
tag=${1:-cur}
timeout -k 10 400 python -u bench.py --config 5 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/c5_$tag.log 2>&1 || { tail -20 gpurun_out/c5_$tag.log; exit 1; }
tail -1 gpurun_out/c5_$tag.log | cut -c1-900
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 \
  bench.py --config 5 --gpus 2 --steps 10 --warmup 5 --comm gloo --device 0 --no-cpu-baseline > gpurun_out/c5w2_$tag.log 2>&1 || { tail -30 gpurun_out/c5w2_$tag.log; exit 1; }
tail -1 gpurun_out/c5w2_$tag.log | cut -c1-600
