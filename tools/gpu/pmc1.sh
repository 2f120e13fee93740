# one PMC pass (SQ counters) over a short bench of a config
set -o pipefail
cfg=${1:-4}
mkdir -p gpurun_out/pmc1_$cfg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmc1_$cfg/p -o run -- python3 bench.py --config $cfg --steps 3 --warmup 10 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 > gpurun_out/pmc1_$cfg/log 2>&1 || { tail -5 gpurun_out/pmc1_$cfg/log; exit 1; }
f=$(find gpurun_out/pmc1_$cfg/p -name '*counter_collection.csv' | head -1)
python3 tools/pmc_summary.py "$f" --json gpurun_out/pmc1_$cfg/pmc.json > gpurun_out/pmc1_$cfg/p.txt && rm -f "$f" $(find gpurun_out/pmc1_$cfg/p -name '*kernel_trace.csv')
head -12 gpurun_out/pmc1_$cfg/p.txt
