set -o pipefail
tag=${1:-r03r}
bash tools/gpu/ab.sh $tag "3" "3 GW_DIRTY_SPAN=8" "3 GW_DIRTY_SPAN=4" "3 GW_DIRTY_SPAN=2" "4" "4 GW_DIRTY_SPAN=4" || exit 1
bash tools/gpu/simprof.sh ${tag}c5 c5 8
