# parity tests, then bench at each grid cell density (GW_CELLS_PER_D)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
for c in 1 2 3 4; do
  GW_CELLS_PER_D=$c timeout -k 10 120 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/b_cpd$c.log 2>&1 || exit 1
  python - "$c" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/b_cpd{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("cpd",sys.argv[1],"ms",round(l["ms_per_step"],3),"dev_us",round(l["device_us_per_step"],1),{k:v["avg_us"] for k,v in l["stages"].items()})
PY
done
