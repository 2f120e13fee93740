# round measurement, part B: configs #4, #2, #5 (bench + profiles), PMC of config #4, CPU baseline table
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_c4_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_c4_$tag.json.log | cut -c1-300
bash tools/gpu/prof.sh c4_$tag --config 4 > /dev/null && head -12 gpurun_out/prof_c4_${tag}_per_step.txt || exit 1
timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/bench_c2_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_c2_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_c2_$tag.json.log | cut -c1-300
bash tools/gpu/c5prof.sh $tag > /dev/null && head -12 gpurun_out/c5prof_${tag}_per_step.txt || exit 1
bash tools/gpu/pmc.sh c4_$tag 4 > gpurun_out/pmc_c4_$tag.log 2>&1 || { tail -20 gpurun_out/pmc_c4_$tag.log; exit 1; }
tail -1 gpurun_out/pmc_c4_$tag.log
timeout -k 10 400 python -u tools/cpu_table.py --threads 16 --budget 20 > gpurun_out/cpu_table_$tag.json 2> gpurun_out/cpu_table_$tag.err || { tail -5 gpurun_out/cpu_table_$tag.err; exit 1; }
echo cpu table done
