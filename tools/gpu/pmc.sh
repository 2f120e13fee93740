# PMC passes over a short bench (one counter group per rocprofv3 run, kernel trace only)
# usage: bash tools/gpu/pmc.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out/pmc_$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -o run -- python3 bench.py --steps 3 --warmup 10 --no-cpu-baseline --profile-stages 0 > gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$tag/p$i.log; exit 1; }
  f=$(find gpurun_out/pmc_$tag/p$i -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_summary.py "$f" --json gpurun_out/pmc_$tag/pmc.json > gpurun_out/pmc_$tag/p$i.txt && rm -f "$f" $(find gpurun_out/pmc_$tag/p$i -name '*kernel_trace.csv')
  cat gpurun_out/pmc_$tag/p$i.txt
done
cp gpurun_out/pmc_$tag/pmc.json gpurun_out/pmc_${tag}.json
