# round-end refresh, part B: config #4 profile + PMC, the decomposed-world rehearsal
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
bash tools/gpu/prof.sh ${tag}_c4 --config 4 > /dev/null && head -12 gpurun_out/prof_${tag}_c4_per_step.txt || exit 1
bash tools/gpu/pmc.sh ${tag}_c4 4 > gpurun_out/pmc_${tag}_c4.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}_c4.log; exit 1; }
bash tools/gpu/sim.sh $tag c3 c5 || exit 1
