# rocprofv3 kernel trace + stats of a short bench run; summary per step.
# usage: bash tools/gpu/prof.sh <tag> [extra bench args]
set -o pipefail
tag=${1:-cur}
shift || true
extra="$*"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 5 --warmup ${WARMUP:-30} --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 $extra > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
kt=$(find gpurun_out/prof_$tag -name '*kernel_trace.csv' | head -1)
ks=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$kt" 5 > gpurun_out/prof_${tag}_per_step.txt
cp "$ks" gpurun_out/prof_${tag}_kernel_stats.csv
rm -f "$kt"
head -45 gpurun_out/prof_${tag}_per_step.txt
tail -1 gpurun_out/prof_$tag.log
