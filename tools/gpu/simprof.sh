# kernel table per rank-tick of the decomposed-world rehearsal (R strips on the one GPU)
# usage: bash tools/gpu/simprof.sh <tag> <c3|c5> <ranks>
set -o pipefail
tag=$1; which=$2; R=$3
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/simprof_$tag -o run -- python3 tools/sim_ranks.py --which $which --ranks $R --warmup 10 --steps 10 > gpurun_out/simprof_$tag.log 2>&1 || { tail -20 gpurun_out/simprof_$tag.log; exit 1; }
kt=$(find gpurun_out/simprof_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py "$kt" $((10 * R)) > gpurun_out/simprof_${tag}_per_rank_tick.txt
rm -f "$kt"
head -60 gpurun_out/simprof_${tag}_per_rank_tick.txt
