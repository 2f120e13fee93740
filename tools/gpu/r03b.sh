set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/t_r03b.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/t_r03b.log; exit 1; }
tail -25 gpurun_out/t_r03b.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r03b.json.log 2>&1 || { tail -30 gpurun_out/bench_r03b.json.log; exit 1; }
tail -1 gpurun_out/bench_r03b.json.log | cut -c1-1500
bash tools/gpu/prof.sh r03b > /dev/null && head -40 gpurun_out/prof_r03b_per_step.txt
