set -o pipefail
tag=${1:-r03w}
mkdir -p gpurun_out
for pm in 0 96; do
  GW_PAIR_MAX=$pm timeout -k 10 400 python -u tools/sim_ranks.py --which c5 --ranks 1,8 --warmup 10 --steps 5 > gpurun_out/sim_c5_${tag}_pm$pm.log 2>&1 || { tail -20 gpurun_out/sim_c5_${tag}_pm$pm.log; exit 1; }
  grep -o '"ranks": [0-9]*\|"step_ms": [0-9.]*\|"diff": [0-9.]*' gpurun_out/sim_c5_${tag}_pm$pm.log | tr '\n' ' '; echo " pair_max=$pm"
done
