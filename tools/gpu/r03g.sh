# A/B of k_mover launch shapes and grid resolution at config #3; e2e of both caller paths
set -o pipefail
tag=${1:-r03g}
mkdir -p gpurun_out
bash tools/gpu/ab.sh $tag "3" "3 GW_MOVER_WPB=2" "3 GW_MOVER_WPB=4" "3 GW_CELLS_PER_D=3" "3 GW_WALK_MIN=0" "3 GW_WALK_MIN=1000000" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config5 --client-msgs 0 > gpurun_out/e2e_$tag.log 2>&1 || { tail -20 gpurun_out/e2e_$tag.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/e2e_$tag.log').read().strip().splitlines()[-1]); print(json.dumps(d['t_e2e'])); print(json.dumps(d['t_e2e_wire']))"
