# A/B of runtime knobs on a bench configuration: ARGS="--config 4" bash tools/gpu/ab_args.sh "ENV=.." "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --steps 10 --warmup 10 --no-cpu-baseline --client-msgs 0 $ARGS > gpurun_out/aba_$i.log 2>&1 || { tail -5 gpurun_out/aba_$i.log; exit 1; }
  python3 - "$i" "$cfg" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/aba_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[2],"| ms",round(l["ms_per_step"],3),{k:v["avg_us"] for k,v in l["stages"].items()})
PY
done
