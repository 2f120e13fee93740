# GPU parity suites (golden + parity + step mode) under non-default knobs, one
# process per knob set (some knobs are read once per process)
# usage: bash tools/gpu/knobs.sh <tag>
set -o pipefail
tag=${1:-knobs}
mkdir -p gpurun_out
for spec in "GW_OVERLAP_COLLECT=0" "GW_MOVER_COMPACT=0" "GW_GATE_COUNTS=0 GW_GATE_DIRECT=0" "GW_SMALL=0" "GW_MOVER_HALVES=0 GW_SYNC_HALVES=0" "GW_PAIR_MAX=96"; do
  read -ra envs <<< "$spec"
  log=gpurun_out/knobs_${tag}_$(echo "$spec" | tr ' =' '__').log
  env "${envs[@]}" timeout -k 10 420 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_step_mode.py -m gpu -x -q --timeout 150 --timeout-method thread > $log 2>&1 || { echo "FAILED under $spec"; tail -30 $log; exit 1; }
  echo "[$spec] $(tail -1 $log)"
done
