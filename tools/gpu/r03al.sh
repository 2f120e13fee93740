set -o pipefail
tag=${1:-r03al}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
bash tools/gpu/r03o.sh $tag > /dev/null || exit 1
grep -o '"ranks": [0-9]*\|"step_ms": [0-9.]*\|speedup_vs_1_excl_exchange": [0-9.]*' gpurun_out/sim_c3_$tag.log gpurun_out/sim_c5_$tag.log | tr '\n' ' '
