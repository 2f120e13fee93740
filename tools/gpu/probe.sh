# host wall time of the client paths call by call (tools/probe_msgs.py), then the same under a HIP
# runtime + kernel trace: API calls and kernels inside each call
# usage: bash tools/gpu/probe.sh <tag>
set -o pipefail
tag=${1:-p}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/probe_msgs.py > gpurun_out/probe_$tag.log 2>&1 || { tail -20 gpurun_out/probe_$tag.log; exit 1; }
tail -1 gpurun_out/probe_$tag.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d gpurun_out/probe_$tag -o run -- python3 tools/probe_msgs.py --reps 3 > gpurun_out/probe_${tag}_trace.log 2>&1 || { tail -20 gpurun_out/probe_${tag}_trace.log; exit 1; }
python3 tools/api_window.py gpurun_out/probe_$tag > gpurun_out/probe_${tag}_api.txt && head -120 gpurun_out/probe_${tag}_api.txt
find gpurun_out/probe_$tag -name '*.csv' -size +20M -delete
