set -o pipefail
mkdir -p gpurun_out/r04u
timeout -k 10 600 python -u -m pytest tests/test_gpu_churn.py tests/test_gpu_golden.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04u/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04u/pytest.log; exit 1; }
export PSAMD_AB=1
for lb in 1 0 1; do
  PSAMD_LB_PLACE=$lb PSAMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/r04u/bench_cfg5_lb$lb.json 2> gpurun_out/r04u/bench_cfg5_lb$lb.log || exit 1
done
