set -o pipefail
mkdir -p gpurun_out
for cpd in 2 1; do
GW_CELLS_PER_D=$cpd timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --e2e-steps 0 > gpurun_out/abc_$cpd.json.log 2>&1 || { tail -20 gpurun_out/abc_$cpd.json.log; exit 1; }
python3 - "$cpd" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/abc_{sys.argv[1]}.json.log").read().strip().splitlines()[-1])
print("cells_per_d",sys.argv[1],"c4 ms",round(l["ms_per_step"],4),{k:v["avg_us"] for k,v in l.get("stages",{}).items()})
PY
done
GW_CELLS_PER_D=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --e2e-steps 0 --no-config5 --client-msgs 0 > gpurun_out/abc3_1.json.log 2>&1 || exit 1
python3 - <<'PY'
import json
l=json.loads(open("gpurun_out/abc3_1.json.log").read().strip().splitlines()[-1])
print("c3 cells_per_d 1 ms",round(l["ms_per_step"],4),{k:v["avg_us"] for k,v in l.get("stages",{}).items()})
PY
