# quick.sh + a config #4 bench line and kernel table
set -o pipefail
tag=${1:-cur}
bash tools/gpu/quick.sh $tag "$2" || exit 1
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --e2e-steps 0 > gpurun_out/bench_c4_$tag.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_$tag.json.log; exit 1; }
python3 - "$tag" <<'PY'
import json,sys
l=json.loads(open(f"gpurun_out/bench_c4_{sys.argv[1]}.json.log").read().strip().splitlines()[-1])
print("c4 ms",round(l["ms_per_step"],4),{k:v["avg_us"] for k,v in l.get("stages",{}).items()})
PY
