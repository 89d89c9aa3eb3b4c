set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r04m/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04m/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r04m/bench_cfg3.json 2> gpurun_out/r04m/bench_cfg3.log
timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu > gpurun_out/r04m/bench_cfg2.json 2> gpurun_out/r04m/bench_cfg2.log
timeout -k 10 300 python -u bench.py --workload cfg4 --no-cpu > gpurun_out/r04m/bench_cfg4.json 2> gpurun_out/r04m/bench_cfg4.log
