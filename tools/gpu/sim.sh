# projected per-rank costs of the decomposed world (tools/sim_ranks.py): R strips on the one GPU
# usage: bash tools/gpu/sim.sh <tag> [which...]
set -o pipefail
tag=${1:-cur}
shift || true
mkdir -p gpurun_out
for w in ${@:-c3 c5}; do
  timeout -k 10 540 python -u tools/sim_ranks.py --which $w --ranks 1,2,4,8 --warmup 20 --steps 10 --out gpurun_out/sim_${w}_$tag.json > gpurun_out/sim_${w}_$tag.log 2>&1 || { tail -20 gpurun_out/sim_${w}_$tag.log; exit 1; }
  cut -c1-400 gpurun_out/sim_${w}_$tag.log
done
