set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in 0 1; do
GW_BK_PROBE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe_$m -o run -- python3 bench.py --steps 5 --warmup 30 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 > gpurun_out/probe_$m.log 2>&1 || exit 1
kt=$(find gpurun_out/probe_$m -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py "$kt" 5 | grep -E "k_bucket|k_bk|k_flatten|gpu-busy"
rm -f "$kt"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py -x -v --timeout 280 --timeout-method thread -k "config4 or large" > gpurun_out/t_c4.log 2>&1; tail -5 gpurun_out/t_c4.log
