# one PMC group over a short config-#3 bench under several env settings; k_mover rows only
# usage: bash tools/gpu/pmc_ab.sh <tag> "<counters>" "<ENV=VAL ...>" ...
set -o pipefail
tag=$1; grp=$2; shift 2
mkdir -p gpurun_out/pmcab_$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for spec in "$@"; do
  i=$((i+1)); out=gpurun_out/pmcab_$tag/p$i
  timeout -s KILL 120 env $spec rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out -o run -- python3 bench.py --steps 3 --warmup 10 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 > $out.log 2>&1 || { echo "pass $i failed"; tail -5 $out.log; exit 1; }
  f=$(find $out -name '*counter_collection.csv' | head -1)
  echo "== $spec"; python3 tools/pmc_summary.py "$f" | grep -E 'k_mover|k_sync_write' ; rm -f "$f"
done
