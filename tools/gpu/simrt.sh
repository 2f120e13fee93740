# decomposed-world rehearsal at R strips: per-stage device times under several env settings, then a
# HIP runtime + kernel trace of the same rehearsal with the GPU idle gaps of a rank-tick
# usage: [SIMRT_TRACE=0] bash tools/gpu/simrt.sh <tag> <c3|c5> <R> ["ENV=VAL ..."]...
set -o pipefail
tag=$1; which=$2; R=$3; shift 3
mkdir -p gpurun_out
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['step_ms'],4), d.get('rank0_device_us_per_stage'), d['host_us_per_rank_step'])" "$1" "$2"; }
i=0
for spec in "" "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $spec python3 -u tools/sim_ranks.py --which $which --ranks $R --warmup 20 --steps 10 > gpurun_out/simrt_${tag}_$i.log 2>&1 || { tail -20 gpurun_out/simrt_${tag}_$i.log; exit 1; }
  show gpurun_out/simrt_${tag}_$i.log "[$spec]"
done
[ "${SIMRT_TRACE:-1}" = 0 ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d gpurun_out/simrt_$tag -o run -- python3 tools/sim_ranks.py --which $which --ranks $R --warmup 10 --steps 5 > gpurun_out/simrt_${tag}_trace.log 2>&1 || { tail -20 gpurun_out/simrt_${tag}_trace.log; exit 1; }
python3 tools/rt_gaps.py gpurun_out/simrt_$tag 4 > gpurun_out/simrt_${tag}_gaps.txt && cat gpurun_out/simrt_${tag}_gaps.txt
kt=$(find gpurun_out/simrt_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py "$kt" $((15 * R)) > gpurun_out/simrt_${tag}_per_rank_tick.txt && head -40 gpurun_out/simrt_${tag}_per_rank_tick.txt
find gpurun_out/simrt_$tag -name '*.csv' -size +20M -delete
