# kernel profile of the config #5 world at N=1 (16M entities in one context)
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof_$tag -o run -- python3 bench.py --config 5 --steps 3 --warmup 5 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 > gpurun_out/c5prof_$tag.log 2>&1 || { tail -20 gpurun_out/c5prof_$tag.log; exit 1; }
kt=$(find gpurun_out/c5prof_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py "$kt" 3 > gpurun_out/c5prof_${tag}_per_step.txt
rm -f "$kt"
head -30 gpurun_out/c5prof_${tag}_per_step.txt
tail -1 gpurun_out/c5prof_$tag.log | cut -c1-400
