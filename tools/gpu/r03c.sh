# round 3 step c: GPU tests, bench (with the e2e breakdown), kernel profile of config #3 and #4, strip rehearsal
# (test failures by assertion (pytest rc 1) do not stop the later steps; any other exit status does)
set -o pipefail
tag=${1:-r03c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=20 > gpurun_out/t_$tag.log 2>&1
rc=$?
tail -22 gpurun_out/t_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS ABORTED rc=$rc"; exit 1; fi
timeout -k 10 420 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$tag.json.log 2>&1 || { tail -30 gpurun_out/bench_$tag.json.log; exit 1; }
tail -1 gpurun_out/bench_$tag.json.log | cut -c1-2500
bash tools/gpu/prof.sh $tag > /dev/null && head -30 gpurun_out/prof_${tag}_per_step.txt || exit 1
bash tools/gpu/prof.sh ${tag}_c4 --config 4 > /dev/null && head -20 gpurun_out/prof_${tag}_c4_per_step.txt || exit 1
timeout -k 10 400 python -u tools/sim_ranks.py --which c3 --ranks 1,8 --warmup 20 --steps 10 --out gpurun_out/sim_c3_$tag.json > gpurun_out/sim_c3_$tag.log 2>&1 || { tail -20 gpurun_out/sim_c3_$tag.log; exit 1; }
cut -c1-1500 gpurun_out/sim_c3_$tag.log
exit $rc
