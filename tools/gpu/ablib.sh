# same-box A/B of library builds (goworld_amd/lib = "cur", goworld_amd/lib_<name>/libgpuaoi.so),
# alternating, twice, via GW_LIB_PATH (same Python, same bench)
# usage: bash tools/gpu/ablib.sh <tag> "<configs>" <name>... [-- extra bench args]
set -o pipefail
tag=$1; cfgs=$2; shift 2
names=(); extra=()
while [ $# -gt 0 ]; do if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi; names+=("$1"); shift; done
mkdir -p gpurun_out
B="--no-cpu-baseline --no-config5 --e2e-steps 0 --client-msgs 0"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d.get('stages',{}); print(sys.argv[2], round(d['ms_per_step'],4), {k: v['avg_us'] for k, v in s.items()})" "$1" "$2"; }
for cfg in $cfgs; do
  for rep in 1 2; do
    for t in cur "${names[@]}"; do
      lib=$PWD/goworld_amd/lib/libgpuaoi.so; [ $t = cur ] || lib=$PWD/goworld_amd/lib_$t/libgpuaoi.so
      log=$PWD/gpurun_out/abl_${tag}_${t}_c${cfg}_$rep.log
      GW_LIB_PATH=$lib timeout -k 10 300 python -u bench.py $B --config $cfg "${extra[@]}" > $log 2>&1 || { tail -20 $log; exit 1; }
      show $log "$t c$cfg"
    done
  done
done
