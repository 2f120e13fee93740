# A/B of runtime tuning knobs on the default bench: bash tools/gpu/ab.sh "ENV=.. ENV=.." "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab_$i.log 2>&1 || { tail -5 gpurun_out/ab_$i.log; exit 1; }
  python3 - "$i" "$cfg" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[2],"| ms",round(l["ms_per_step"],3),{k:v["avg_us"] for k,v in l["stages"].items()})
PY
done
