# copy a GPU call's evidence (gpurun_out/) into profiles/ under the given tag (run here, after the call)
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
true
