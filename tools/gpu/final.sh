# round-end evidence in one call: GPU tests, smoke, PMC passes of configs #3 and #4 (copied to
# profiles/ so the bench lines carry their traffic), the default bench line (CPU baselines included),
# config #4's line, kernel tables of both, the decomposed-world rehearsals and the 8(f) kernel tables.
# usage: bash tools/gpu/final.sh <tag> [a|b]   then, here: bash tools/gpu/keep_evidence.sh <tag> <prefix>
# (phase a: tests, smoke, PMC passes; phase b: bench lines, kernel tables, 8(f) tables, rehearsals;
# no phase: both -- each phase fits one gpurun call)
set -o pipefail
tag=${1:-final}
phase=${2:-ab}
mkdir -p gpurun_out
if [[ $phase == *a* ]]; then
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_$tag.log 2>&1 || { tail -20 gpurun_out/s_$tag.log; exit 1; }
tail -1 gpurun_out/s_$tag.log
bash tools/gpu/pmc.sh $tag 3 > gpurun_out/pmc_$tag.log 2>&1 || { tail -20 gpurun_out/pmc_$tag.log; exit 1; }
cp gpurun_out/pmc_$tag/pmc_config3.json profiles/pmc_config3.json
bash tools/gpu/pmc.sh ${tag}c4 4 > gpurun_out/pmc_${tag}c4.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}c4.log; exit 1; }
cp gpurun_out/pmc_${tag}c4/pmc_config4.json profiles/pmc_config4.json
fi
[[ $phase == *b* ]] || exit 0
timeout -k 10 480 python -u bench.py > gpurun_out/bench_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_$tag.json.log | cut -c1-400
timeout -k 10 420 python -u bench.py --config 4 --no-cpu-baseline --no-config5 --client-msgs 0 > gpurun_out/bench_${tag}_c4.json.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c4.json.log; exit 1; }
bash tools/gpu/prof.sh $tag > /dev/null && head -8 gpurun_out/prof_${tag}_per_step.txt || exit 1
bash tools/gpu/prof.sh ${tag}c4 --config 4 > /dev/null && head -8 gpurun_out/prof_${tag}c4_per_step.txt || exit 1
bash tools/gpu/fprof.sh $tag > gpurun_out/fprof_$tag.txt 2>&1 || { tail -20 gpurun_out/fprof_$tag.txt; exit 1; }
bash tools/gpu/sim.sh $tag c3 c5 || exit 1
