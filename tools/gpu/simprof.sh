# kernel statistics of tools/sim_ranks.py runs (all ranks' kernels together)
# usage: bash tools/gpu/simprof.sh <tag> <which> <ranks>
set -o pipefail
tag=${1:-cur}; which=${2:-c5}; ranks=${3:-8}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_$tag -o run -- python3 tools/sim_ranks.py --which $which --ranks $ranks --warmup 20 --steps 5 > gpurun_out/sprof_$tag.log 2>&1 || { tail -20 gpurun_out/sprof_$tag.log; exit 1; }
kt=$(find gpurun_out/sprof_$tag -name '*kernel_trace.csv' | head -1)
ks=$(find gpurun_out/sprof_$tag -name '*kernel_stats.csv' | head -1)
cp "$ks" gpurun_out/sprof_${tag}_kernel_stats.csv
python3 tools/prof_summary.py "$kt" $((ranks * 5)) > gpurun_out/sprof_${tag}_per_rank_tick.txt || true
rm -f "$kt"
head -45 gpurun_out/sprof_${tag}_per_rank_tick.txt
