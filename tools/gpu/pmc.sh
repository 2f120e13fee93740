# PMC passes over a short bench (one counter group per rocprofv3 run, kernel trace only)
# usage: bash tools/gpu/pmc.sh <tag> [config]   -> gpurun_out/pmc_<tag>/pmc_config<config>.json
set -o pipefail
tag=${1:-cur}
cfg=${2:-3}
out=gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/p$i -o run -- python3 bench.py --config $cfg --steps 3 --warmup 10 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
  f=$(find $out/p$i -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_summary.py "$f" --json $out/pmc.json > $out/p$i.txt && rm -f "$f" $(find $out/p$i -name '*kernel_trace.csv')
  cat $out/p$i.txt
done
python3 tools/pmc_summary.py --finalize $out/pmc.json --config $cfg --out $out/pmc_config$cfg.json
