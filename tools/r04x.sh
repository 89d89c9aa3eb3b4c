set -o pipefail
mkdir -p gpurun_out/r04x
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r04x/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04x/pytest_gpu.log; exit 1; }
for c in cfg3 cfg2 cfg4 cfg5; do
  timeout -k 10 400 python -u bench.py --workload $c --no-cpu > gpurun_out/r04x/bench_$c.json 2> gpurun_out/r04x/bench_$c.log || exit 1
done
