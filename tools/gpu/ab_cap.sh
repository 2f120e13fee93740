# cost of slot capacity (a strip's global id range) on config #3
set -o pipefail
mkdir -p gpurun_out
for cap in 0 8000000 16000000; do
  extra=""; [ $cap -gt 0 ] && extra="--capacity $cap"
  timeout -k 10 150 python -u bench.py --steps 20 --no-cpu-baseline $extra > gpurun_out/cap_$cap.log 2>&1 || { tail -20 gpurun_out/cap_$cap.log; exit 1; }
  python3 - $cap <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/cap_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("cap",sys.argv[1],"ms",round(l["ms_per_step"],3),"dev_us",round(l["device_us_per_step"],1),{k:v["avg_us"] for k,v in l["stages"].items()})
PY
done
