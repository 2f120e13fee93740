# PCIe probe; A/B of the paired diff kernel at configs #3 and #4; e2e of config #3 with the wire view
set -o pipefail
tag=${1:-r03f}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/pcie > gpurun_out/pcie_$tag.txt 2>&1 || { cat gpurun_out/pcie_$tag.txt; exit 1; }
cat gpurun_out/pcie_$tag.txt
bash tools/gpu/ab.sh $tag "3" "3 GW_PAIR_MAX=0" "3 GW_PAIR_MAX=48" "4" "4 GW_PAIR_MAX=0" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config5 --client-msgs 0 --e2e-steps 4 > gpurun_out/e2e_$tag.log 2>&1 || { tail -20 gpurun_out/e2e_$tag.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/e2e_$tag.log').read().strip().splitlines()[-1]); print(json.dumps(d['t_e2e']))"
