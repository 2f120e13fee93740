# round measurement, part A: default bench line (CPU baselines, config #5 key), kernel profile, PMC of config #3
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 480 python -u bench.py > gpurun_out/bench_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_$tag.json.log | cut -c1-300
bash tools/gpu/prof.sh $tag > /dev/null && head -8 gpurun_out/prof_${tag}_per_step.txt || exit 1
bash tools/gpu/pmc.sh $tag 3 > gpurun_out/pmc_$tag.log 2>&1 || { tail -20 gpurun_out/pmc_$tag.log; exit 1; }
tail -1 gpurun_out/pmc_$tag.log
