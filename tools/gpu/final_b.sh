# config #4 bench + kernel table + PMC passes, then the decomposed-world rehearsals (1/2/4/8 strips)
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out
bash tools/gpu/pmc.sh ${tag}c4 4 > gpurun_out/pmc_${tag}c4.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}c4.log; exit 1; }
tail -1 gpurun_out/pmc_${tag}c4.log
cp gpurun_out/pmc_${tag}c4/pmc_config4.json profiles/pmc_config4.json
timeout -k 10 420 python -u bench.py --config 4 --no-cpu-baseline --no-config5 --client-msgs 0 > gpurun_out/bench_${tag}_c4.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c4.json.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c4.json.log | cut -c1-300
bash tools/gpu/prof.sh ${tag}c4 --config 4 > /dev/null && head -14 gpurun_out/prof_${tag}c4_per_step.txt || exit 1
bash tools/gpu/sim.sh $tag c3 c5 || exit 1
