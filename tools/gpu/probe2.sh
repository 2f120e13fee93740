set -o pipefail
mkdir -p gpurun_out
GW_BK_PROBE=2 GW_DEBUG_STATS=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --client-msgs 0 --e2e-steps 0 --no-config5 > gpurun_out/probe2.log 2>&1 || { tail gpurun_out/probe2.log; exit 1; }
grep "gw_tick" gpurun_out/probe2.log | tail -4
