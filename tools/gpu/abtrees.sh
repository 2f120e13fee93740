# same-box A/B over several built trees (. and _ab/<name>...), alternating, twice
# usage: bash tools/gpu/abtrees.sh <tag> "<configs>" <name>...
set -o pipefail
tag=$1; cfgs=$2; shift 2
mkdir -p gpurun_out
B="--no-cpu-baseline --no-config5 --e2e-steps 0 --client-msgs 0"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('stages',{}); print(sys.argv[2], round(d['ms_per_step'],4), {k: v['avg_us'] for k, v in s.items()})" "$1" "$2"; }
for cfg in $cfgs; do
  for rep in 1 2; do
    for t in cur "$@"; do
      dir=.; [ $t = cur ] || dir=_ab/$t
      log=$PWD/gpurun_out/abts_${tag}_${t}_c${cfg}_$rep.log
      (cd $dir && timeout -k 10 300 python -u bench.py $B --config $cfg) > $log 2>&1 || { tail -20 $log; exit 1; }
      show $log "$t c$cfg"
    done
  done
done
