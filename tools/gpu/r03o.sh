# decomposed-world rehearsal at HEAD: 1M (config #3 as a world) and 16M (config #5) at 1 and 8 strips
set -o pipefail
tag=${1:-r03o}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sim_ranks.py --which c3 --ranks 1,8 --warmup 20 --steps 10 --out gpurun_out/sim_c3_$tag.json > gpurun_out/sim_c3_$tag.log 2>&1 || { tail -20 gpurun_out/sim_c3_$tag.log; exit 1; }
cat gpurun_out/sim_c3_$tag.log
timeout -k 10 500 python -u tools/sim_ranks.py --which c5 --ranks 1,8 --warmup 10 --steps 5 --out gpurun_out/sim_c5_$tag.json > gpurun_out/sim_c5_$tag.log 2>&1 || { tail -20 gpurun_out/sim_c5_$tag.log; exit 1; }
cat gpurun_out/sim_c5_$tag.log
