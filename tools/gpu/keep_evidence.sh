# copy a GPU call's evidence (gpurun_out/) into profiles/ under the given prefix (run here, after the
# call; tools/gpu/final.sh names what it writes by <tag>)
# usage: bash tools/gpu/keep_evidence.sh <tag> <out-prefix>
set -o pipefail
tag=$1; pre=$2
[ -f gpurun_out/pmc_$tag/pmc_config3.json ] && cp gpurun_out/pmc_$tag/pmc_config3.json profiles/pmc_config3.json
[ -f gpurun_out/pmc_${tag}c4/pmc_config4.json ] && cp gpurun_out/pmc_${tag}c4/pmc_config4.json profiles/pmc_config4.json
for i in 1 2 3 4; do
  [ -f gpurun_out/pmc_$tag/p$i.txt ] && cp gpurun_out/pmc_$tag/p$i.txt profiles/${pre}_pmc_p$i.txt
  [ -f gpurun_out/pmc_${tag}c4/p$i.txt ] && cp gpurun_out/pmc_${tag}c4/p$i.txt profiles/${pre}_config4_pmc_p$i.txt
done
[ -f gpurun_out/bench_$tag.json.log ] && tail -1 gpurun_out/bench_$tag.json.log > profiles/${pre}_bench.json
[ -f gpurun_out/bench_${tag}_c4.json.log ] && tail -1 gpurun_out/bench_${tag}_c4.json.log > profiles/${pre}_config4_bench.json
for s in "" c4; do
  [ -f gpurun_out/prof_${tag}${s}_per_step.txt ] && cp gpurun_out/prof_${tag}${s}_per_step.txt profiles/${pre}${s:+_config4}_per_step.txt
  [ -f gpurun_out/prof_${tag}${s}_kernel_stats.csv ] && cp gpurun_out/prof_${tag}${s}_kernel_stats.csv profiles/${pre}${s:+_config4}_kernel_stats.csv
done
for w in msgs bycl; do
  [ -f gpurun_out/fprof_${tag}_${w}_kernel_stats.csv ] && cp gpurun_out/fprof_${tag}_${w}_kernel_stats.csv profiles/${pre}_8f_${w}_kernel_stats.csv
done
[ -f gpurun_out/fprof_$tag.txt ] && cp gpurun_out/fprof_$tag.txt profiles/${pre}_8f.txt
for w in c3 c5; do
  [ -f gpurun_out/sim_${w}_$tag.json ] && cp gpurun_out/sim_${w}_$tag.json profiles/${pre}_sim_$w.json
done
[ -f gpurun_out/t_$tag.log ] && grep -E "passed|failed" gpurun_out/t_$tag.log | tail -1 > profiles/${pre}_gpu_tests.txt
true
