# A/B of knobs on the bench's stage times.  usage: bash tools/gpu/ab.sh <tag> "<cfg> <ENV=VAL ...>" ...
# each argument: a config number, then env assignments (none = defaults)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
B="--no-cpu-baseline --no-config5 --e2e-steps 0 --client-msgs 0"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('stages',{}); print(sys.argv[2], round(d['ms_per_step'],4), {k: v['avg_us'] for k, v in s.items()})" "$1" "$2"; }
i=0
for spec in "$@"; do
  i=$((i+1))
  set -- $spec
  cfg=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py $B --config $cfg > gpurun_out/ab_${tag}_$i.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_$i.log; exit 1; }
  show gpurun_out/ab_${tag}_$i.log "c$cfg $*"
done
