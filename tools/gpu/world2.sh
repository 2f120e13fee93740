# rehearsal of the decomposed-world bench with 2 ranks sharing the one GPU (gloo halo exchange)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-cur}
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 10 --warmup 5 --comm gloo --device 0 --no-cpu-baseline > gpurun_out/w2_$tag.log 2>&1 || { tail -40 gpurun_out/w2_$tag.log; exit 1; }
tail -1 gpurun_out/w2_$tag.log | cut -c1-1500
