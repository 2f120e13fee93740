# one PMC group over a short config-#3 bench in this tree and in built trees _ab/<name>; kernel rows matching a pattern
# usage: bash tools/gpu/pmc_trees.sh <tag> "<counters>" "<kernel regex>" <name>...
set -o pipefail
tag=$1; grp=$2; pat=$3; shift 3
mkdir -p gpurun_out/pmct_$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in cur "$@"; do
  dir=$GRAFT_REPO_ROOT; [ $t = cur ] || dir=$GRAFT_REPO_ROOT/_ab/$t
  out=$GRAFT_REPO_ROOT/gpurun_out/pmct_$tag/$t
  (cd $dir && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out -o run -- python3 bench.py --steps 3 --warmup 10 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5) > $out.log 2>&1 || { echo "$t failed"; tail -5 $out.log; exit 1; }
  f=$(find $out -name '*counter_collection.csv' | head -1)
  echo "== $t"; python3 tools/pmc_summary.py "$f" | grep -E "$pat"; rm -f "$f"
done
