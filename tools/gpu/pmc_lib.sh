# SQ issue counters of one kernel for several library builds (GW_LIB_PATH), config #3 unless given
# usage: bash tools/gpu/pmc_ab.sh <tag> <kernel-substring> <cfg> <name>...   (cur = goworld_amd/lib)
set -o pipefail
tag=$1; kern=$2; cfg=$3; shift 3
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in "$@"; do
  lib=$PWD/goworld_amd/lib/libgpuaoi.so; [ $t = cur ] || lib=$PWD/goworld_amd/lib_$t/libgpuaoi.so
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"; do
    i=$((i+1))
    out=gpurun_out/pmcab_${tag}_${t}_p$i
    GW_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out -o run -- python3 bench.py --config $cfg --steps 3 --warmup 10 --no-cpu-baseline --profile-stages 0 --client-msgs 0 --e2e-steps 0 --no-config5 > $out.log 2>&1 || { echo "pass failed"; tail -5 $out.log; exit 1; }
    f=$(find $out -name '*counter_collection.csv' | head -1)
    echo "== $t p$i"; python3 tools/pmc_summary.py "$f" | grep "$kern"
    rm -f "$f" $(find $out -name '*kernel_trace.csv')
  done
done
