# config #4 with small-space mode on / off, config #5 at N=1
set -o pipefail
mkdir -p gpurun_out
for sm in 1 0; do
GW_SMALL=$sm timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --e2e-steps 0 > gpurun_out/ab4_$sm.json.log 2>&1 || { tail -20 gpurun_out/ab4_$sm.json.log; exit 1; }
python3 - "$sm" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/ab4_{sys.argv[1]}.json.log").read().strip().splitlines()[-1])
print("small",sys.argv[1],"c4 ms",round(l["ms_per_step"],4),{k:v["avg_us"] for k,v in l.get("stages",{}).items()})
PY
done
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --e2e-steps 0 > gpurun_out/c5_n1.json.log 2>&1 || { tail -20 gpurun_out/c5_n1.json.log; exit 1; }
python3 - <<'PY'
import json
l=json.loads(open("gpurun_out/c5_n1.json.log").read().strip().splitlines()[-1])
print("c5 ms",round(l["ms_per_step"],4),{k:v["avg_us"] for k,v in l.get("stages",{}).items()})
PY
