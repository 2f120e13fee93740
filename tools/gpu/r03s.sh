set -o pipefail
tag=${1:-r03s}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
bash tools/gpu/ab.sh $tag "3" "3 GW_DIRTY_SPAN=8" "3 GW_DIRTY_SPAN=4" "3 GW_DIRTY_SPAN=2" "4" "4 GW_DIRTY_SPAN=4" || exit 1
bash tools/gpu/simprof.sh ${tag}c3 c3 8 | head -30
