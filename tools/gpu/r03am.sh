set -o pipefail
tag=${1:-r03am}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline --client-msgs 0 --e2e-steps 0 > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$tag.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config5']['ms_per_step'], d['config5']['value'])"
(cd _ab/prev && timeout -k 10 420 python -u bench.py --no-cpu-baseline --client-msgs 0 --e2e-steps 0) > gpurun_out/bench_${tag}_prev.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_prev.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_${tag}_prev.log').read().strip().splitlines()[-1]); print('prev', d['ms_per_step'], d['config5']['ms_per_step'], d['config5']['value'])"
