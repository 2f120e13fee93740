set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for t in cur base; do
    lib=$PWD/goworld_amd/lib/libgpuaoi.so; [ $t = cur ] || lib=$PWD/goworld_amd/lib_$t/libgpuaoi.so
    GW_LIB_PATH=$lib timeout -k 10 300 python -u tools/sim_ranks.py --which c5 --ranks 8 --warmup 20 --steps 10 --out gpurun_out/simab_${t}_$rep.json > gpurun_out/simab_${t}_$rep.log 2>&1 || { tail -20 gpurun_out/simab_${t}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))[-1]; print(sys.argv[2], d['ranks'], round(d['step_ms'],4), d['host_us_per_rank_step'], d['rank0_device_us_per_stage'])" gpurun_out/simab_${t}_$rep.json $t
  done
done
