# same-box A/B of environment knobs on one library build, alternating, twice
# usage: bash tools/gpu/envab.sh <tag> <config> "<envA>" "<envB>" ... [-- extra bench args]
#   each env spec is a space-separated list of VAR=value ("-" for none)
set -o pipefail
tag=$1; cfg=$2; shift 2
specs=(); extra=()
while [ $# -gt 0 ]; do if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi; specs+=("$1"); shift; done
mkdir -p gpurun_out
B="--no-cpu-baseline --no-config5 --e2e-steps 0 --client-msgs 0"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('stages',{}); print(sys.argv[2], round(d['ms_per_step'],4), {k: v['avg_us'] for k, v in s.items()})" "$1" "$2"; }
for rep in 1 2; do
  i=0
  for spec in "${specs[@]}"; do
    i=$((i+1))
    log=$PWD/gpurun_out/envab_${tag}_${i}_c${cfg}_$rep.log
    envs=(); [ "$spec" = "-" ] || read -ra envs <<< "$spec"
    env "${envs[@]}" timeout -k 10 300 python -u bench.py $B --config $cfg "${extra[@]}" > $log 2>&1 || { tail -20 $log; exit 1; }
    show $log "[$spec] c$cfg"
  done
done
