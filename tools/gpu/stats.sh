# one short bench run printing per-tick device counters (needs a -DGW_SEG_STATS=1 build for the seg counters)
set -o pipefail
mkdir -p gpurun_out
GW_DEBUG_STATS=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 30 --no-cpu-baseline > gpurun_out/stats.log 2>&1
grep gw_tick gpurun_out/stats.log | tail -4
