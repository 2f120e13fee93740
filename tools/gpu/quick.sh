# GPU tests, a short bench (no CPU baselines, no config #5) and a kernel profile.
# usage: bash tools/gpu/quick.sh <tag> [pytest -k expr]
set -o pipefail
tag=${1:-cur}
sel=${2:-}
mkdir -p gpurun_out
if [ -n "$sel" ]; then ksel=(-k "$sel"); else ksel=(); fi
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "${ksel[@]}" > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error" gpurun_out/t_$tag.log | head -20; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --client-msgs 0 --no-config5 > gpurun_out/bench_$tag.json.log 2>&1 || { tail -30 gpurun_out/bench_$tag.json.log; exit 1; }
python3 - "$tag" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json.log").read().strip().splitlines()[-1])
print("ms",round(l["ms_per_step"],4),"dev_us",round(l["device_us_per_step"] or 0,1),"frac",round(l["roofline"]["frac"],4),{k:v["avg_us"] for k,v in l.get("stages",{}).items()}, "e2e", l.get("t_e2e",{}).get("ms_per_step"))
PY
bash tools/gpu/prof.sh $tag > /dev/null && head -30 gpurun_out/prof_${tag}_per_step.txt
