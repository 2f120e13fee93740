# round-end refresh, part A: tests, smoke, default bench, config #3 profile + PMC, config #4 / #2 bench lines
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
bash tools/gpu/round.sh $tag || exit 1
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_${tag}_c4.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c4.json.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c4.json.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/bench_${tag}_c2.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c2.json.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c2.json.log | cut -c1-300
