# host/device timeline of a short config-#3 bench: HIP runtime API + kernel trace, summarised
set -o pipefail
tag=${1:-rt}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d gpurun_out/rt_$tag -o run -- python3 bench.py --steps 5 --warmup 20 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 > gpurun_out/rt_$tag.log 2>&1 || { tail -20 gpurun_out/rt_$tag.log; exit 1; }
python3 tools/rt_gaps.py gpurun_out/rt_$tag 3 --seq > gpurun_out/rt_${tag}_gaps.txt && cat gpurun_out/rt_${tag}_gaps.txt
find gpurun_out/rt_$tag -name '*.csv' -size +20M -delete
