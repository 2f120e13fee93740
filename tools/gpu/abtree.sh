# same-box A/B of this tree against a built older tree in _ab/<name> (git worktree):
# usage: bash tools/gpu/abtree.sh <tag> <name> <config>...   (alternates cur / old per config, twice)
set -o pipefail
tag=$1; old=$2; shift 2
mkdir -p gpurun_out
B="--no-cpu-baseline --no-config5 --e2e-steps 0 --client-msgs 0"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('stages',{}); print(sys.argv[2], round(d['ms_per_step'],4), {k: v['avg_us'] for k, v in s.items()})" "$1" "$2"; }
for cfg in "$@"; do
  for rep in 1 2; do
    timeout -k 10 300 python -u bench.py $B --config $cfg > gpurun_out/abt_${tag}_cur_c${cfg}_$rep.log 2>&1 || { tail -20 gpurun_out/abt_${tag}_cur_c${cfg}_$rep.log; exit 1; }
    show gpurun_out/abt_${tag}_cur_c${cfg}_$rep.log "cur c$cfg"
    (cd _ab/$old && timeout -k 10 300 python -u bench.py $B --config $cfg) > gpurun_out/abt_${tag}_old_c${cfg}_$rep.log 2>&1 || { tail -20 gpurun_out/abt_${tag}_old_c${cfg}_$rep.log; exit 1; }
    show gpurun_out/abt_${tag}_old_c${cfg}_$rep.log "$old c$cfg"
  done
done
