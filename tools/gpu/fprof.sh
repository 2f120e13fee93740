# kernel tables of the SURVEY 8(f) paths at config #3: the client messages (gw_client_events + gw_fanout of one
# AllClients call per mover, 5 ticks) and the gate's per-client regroup (GW_SYNC_BY_CLIENT collect)
# usage: bash tools/gpu/fprof.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--no-cpu-baseline --profile-stages 0 --e2e-steps 0 --no-config5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof_${tag}_msgs -o run -- python3 bench.py $B --steps 2 --warmup 3 --client-msgs 5 > gpurun_out/fprof_${tag}_msgs.log 2>&1 || { tail -20 gpurun_out/fprof_${tag}_msgs.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof_${tag}_bycl -o run -- python3 bench.py $B --steps 5 --warmup 3 --client-msgs 0 --sync-by-client > gpurun_out/fprof_${tag}_bycl.log 2>&1 || { tail -20 gpurun_out/fprof_${tag}_bycl.log; exit 1; }
for w in msgs bycl; do
  ks=$(find gpurun_out/fprof_${tag}_$w -name '*kernel_stats.csv' | head -1)
  cp "$ks" gpurun_out/fprof_${tag}_${w}_kernel_stats.csv
  find gpurun_out/fprof_${tag}_$w -name '*kernel_trace.csv' -delete
  echo "== $w"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:22]: print(f\"{r['Name'][:60]:60s} calls {int(r['Calls']):5d} total_us {float(r['TotalDurationNs'])/1e3:10.1f} avg_us {float(r['AverageNs'])/1e3:8.1f}\")
" gpurun_out/fprof_${tag}_${w}_kernel_stats.csv
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(json.dumps(d.get('client_msgs'))[:600]); print('ms', d['ms_per_step'])" gpurun_out/fprof_${tag}_$w.log
done
