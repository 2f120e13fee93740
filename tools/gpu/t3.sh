set -o pipefail
mkdir -p gpurun_out
bash tools/gpu/prof.sh c4t3 --config 4 > /dev/null && head -40 gpurun_out/prof_c4t3_per_step.txt || exit 1
bash tools/gpu/simprof.sh c5r8 c5 8 || exit 1
bash tools/gpu/simprof.sh c3r1 c3 1 || exit 1
