# same-box A/B of env knobs on the decomposed-world rehearsal (tools/sim_ranks.py)
# usage: bash tools/gpu/simenv.sh <tag> <which> <ranks> "<envA>" "<envB>" ...  ("-" for none)
set -o pipefail
tag=$1; which=$2; ranks=$3; shift 3
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    envs=(); [ "$spec" = "-" ] || read -ra envs <<< "$spec"
    out=gpurun_out/simenv_${tag}_${i}_$rep
    env "${envs[@]}" timeout -k 10 300 python -u tools/sim_ranks.py --which $which --ranks $ranks --warmup 20 --steps 10 --out $out.json > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))[-1]; print(sys.argv[2], d['ranks'], round(d['step_ms'],4), d['rank0_device_us_per_stage'])" $out.json "[$spec]"
  done
done
