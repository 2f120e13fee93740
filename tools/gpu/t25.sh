set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_t25.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/t_t25.log | head -20; tail -30 gpurun_out/t_t25.log; exit 1; }
tail -1 gpurun_out/t_t25.log
ARGS="--config 4" bash tools/gpu/ab_args.sh "GW_X=0" || exit 1
ARGS="--no-config5" bash tools/gpu/ab_args.sh "GW_X=0" "GW_X=0" || exit 1
bash tools/gpu/pmc.sh r02g 3 > gpurun_out/pmc_r02g.log 2>&1 || { tail -20 gpurun_out/pmc_r02g.log; exit 1; }
bash tools/gpu/pmc.sh r02g_c4 4 > gpurun_out/pmc_r02g_c4.log 2>&1 || { tail -20 gpurun_out/pmc_r02g_c4.log; exit 1; }
bash tools/gpu/prof.sh r02g > /dev/null && head -8 gpurun_out/prof_r02g_per_step.txt
