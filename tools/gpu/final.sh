# round-end refresh: GPU tests, smoke, default bench (CPU baselines), profile and PMC of config #3,
# then config #4 / #2 bench lines, config #4 PMC and profile, the decomposed-world rehearsal
set -o pipefail
tag=${1:-r02e}
mkdir -p gpurun_out
bash tools/gpu/round.sh $tag || exit 1
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_${tag}_c4.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c4.json.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c4.json.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/bench_${tag}_c2.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c2.json.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c2.json.log | cut -c1-300
bash tools/gpu/prof.sh ${tag}_c4 --config 4 > /dev/null && head -12 gpurun_out/prof_${tag}_c4_per_step.txt || exit 1
bash tools/gpu/pmc.sh ${tag}_c4 4 > gpurun_out/pmc_${tag}_c4.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}_c4.log; exit 1; }
bash tools/gpu/sim.sh $tag c3 c5 || exit 1
