# round-end refresh at the final kernel sources: PMC of configs #3 and #4 first (the bench reads
# their traffic when the source hash matches), then the bench lines and kernel tables
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
bash tools/gpu/pmc.sh $tag 3 > gpurun_out/pmc_$tag.log 2>&1 || { tail -20 gpurun_out/pmc_$tag.log; exit 1; }
bash tools/gpu/pmc.sh ${tag}_c4 4 > gpurun_out/pmc_${tag}_c4.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}_c4.log; exit 1; }
cp gpurun_out/pmc_$tag/pmc_config3.json profiles/pmc_config3.json && cp gpurun_out/pmc_${tag}_c4/pmc_config4.json profiles/pmc_config4.json || exit 1
timeout -k 10 420 python -u bench.py > gpurun_out/bench_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_$tag.json.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_${tag}_c4.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c4.json.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c4.json.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/bench_${tag}_c2.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c2.json.log; exit 1; }
bash tools/gpu/prof.sh $tag > /dev/null && head -4 gpurun_out/prof_${tag}_per_step.txt || exit 1
bash tools/gpu/prof.sh ${tag}_c4 --config 4 > /dev/null && head -4 gpurun_out/prof_${tag}_c4_per_step.txt || exit 1
