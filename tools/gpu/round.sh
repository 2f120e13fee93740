# GPU tests, smoke, the PMC passes of config #3 (copied to profiles/ so the bench line carries their
# traffic), the default bench (CPU baselines included), a kernel profile; each step under its own
# time limit.   usage: bash tools/gpu/round.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_$tag.log 2>&1 || { tail -20 gpurun_out/s_$tag.log; exit 1; }
tail -1 gpurun_out/s_$tag.log
bash tools/gpu/pmc.sh $tag 3 > gpurun_out/pmc_$tag.log 2>&1 || { tail -20 gpurun_out/pmc_$tag.log; exit 1; }
tail -1 gpurun_out/pmc_$tag.log
cp gpurun_out/pmc_$tag/pmc_config3.json profiles/pmc_config3.json
timeout -k 10 420 python -u bench.py > gpurun_out/bench_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_$tag.json.log | cut -c1-600
bash tools/gpu/prof.sh $tag > /dev/null && head -12 gpurun_out/prof_${tag}_per_step.txt || exit 1
