set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_t27.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" gpurun_out/t_t27.log | head -20; tail -30 gpurun_out/t_t27.log; exit 1; }
tail -1 gpurun_out/t_t27.log
bash tools/gpu/prof.sh t27 > /dev/null && grep -E "busy|k_flat_items|k_bk_count|k_bucket_scatter" gpurun_out/prof_t27_per_step.txt || exit 1
bash tools/gpu/prof.sh t27c4 --config 4 > /dev/null && grep -E "busy|k_flat_items|k_bk_count|k_bucket_scatter" gpurun_out/prof_t27c4_per_step.txt || exit 1
