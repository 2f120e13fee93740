# the client paths (tools/probe_msgs.py) under a kernel trace at several sort digit widths
# (GW_SORT_DB): per-call host times and the sort / fan-out / record kernels' average durations
# usage: bash tools/gpu/sortab.sh <tag> <db> ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  GW_SORT_DB=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sab_${tag}_$v -o run -- python3 tools/probe_msgs.py > gpurun_out/sab_${tag}_$v.log 2>&1 || { tail -20 gpurun_out/sab_${tag}_$v.log; exit 1; }
  echo "== GW_SORT_DB=$v"; grep '^{' gpurun_out/sab_${tag}_$v.log
  python3 - "gpurun_out/sab_${tag}_$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("os_", "fanout", "records_seg", "client_compact", "sync_write")):
        print(f"  {n[:60]:60s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs']) / 1e3:8.1f}")
PY
  find gpurun_out/sab_${tag}_$v -name '*trace.csv' -delete
done
