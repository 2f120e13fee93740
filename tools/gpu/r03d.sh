# round 3 step d: PCIe probe; A/B of the diff kernels (current vs GW_PAIR_MAX=0 vs the round-2
# tree in _ab/r02) at configs #3 and #4; config #3 at 3 cells per AOI distance; kernel timeline of
# the 8-strip 1M world rehearsal (fixed per-tick cost)
set -o pipefail
tag=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/pcie > gpurun_out/pcie_$tag.txt 2>&1 || { cat gpurun_out/pcie_$tag.txt; exit 1; }
cat gpurun_out/pcie_$tag.txt
B="--no-cpu-baseline --no-config5 --e2e-steps 0 --client-msgs 0"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('stages',{}); print(sys.argv[2], round(d['ms_per_step'],4), {k: v['avg_us'] for k, v in s.items()})" "$1" "$2"; }
for cfg in 3 4; do
  timeout -k 10 300 python -u bench.py $B --config $cfg > gpurun_out/ab_${tag}_cur_c$cfg.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_cur_c$cfg.log; exit 1; }
  show gpurun_out/ab_${tag}_cur_c$cfg.log "cur c$cfg"
  (cd _ab/r02 && timeout -k 10 300 python -u bench.py $B --config $cfg) > gpurun_out/ab_${tag}_r02_c$cfg.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_r02_c$cfg.log; exit 1; }
  show gpurun_out/ab_${tag}_r02_c$cfg.log "r02 c$cfg"
done
GW_PAIR_MAX=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/ab_${tag}_nopair_c3.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_nopair_c3.log; exit 1; }
show gpurun_out/ab_${tag}_nopair_c3.log "nopair c3"
GW_CELLS_PER_D=3 timeout -k 10 300 python -u bench.py $B > gpurun_out/ab_${tag}_cpd3_c3.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_cpd3_c3.log; exit 1; }
show gpurun_out/ab_${tag}_cpd3_c3.log "cpd3 c3"
GW_CELLS_PER_D=3 GW_PAIR_MAX=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/ab_${tag}_cpd3np_c3.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_cpd3np_c3.log; exit 1; }
show gpurun_out/ab_${tag}_cpd3np_c3.log "cpd3 nopair c3"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sim8_$tag -o run -- python3 tools/sim_ranks.py --which c3 --ranks 8 --warmup 10 --steps 5 > gpurun_out/sim8_$tag.log 2>&1 || { tail -20 gpurun_out/sim8_$tag.log; exit 1; }
cut -c1-1200 gpurun_out/sim8_$tag.log | tail -2
