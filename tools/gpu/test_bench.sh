# parity tests, then a short bench and a kernel profile
# usage: bash tools/gpu/test_bench.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -2 gpurun_out/t_$tag.log
timeout -k 10 120 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/b_$tag.log 2>&1 || { tail -20 gpurun_out/b_$tag.log; exit 1; }
python3 - "$tag" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/b_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("ms",round(l["ms_per_step"],3),"dev_us",round(l["device_us_per_step"],1),{k:v["avg_us"] for k,v in l["stages"].items()})
PY
bash tools/gpu/prof.sh $tag
