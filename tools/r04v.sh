set -o pipefail
mkdir -p gpurun_out/r04v
timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_api.py tests/test_gpu_drain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04v/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04v/pytest.log; exit 1; }
export PSAMD_AB=1
for v in 1 0 1 0; do
  echo "sig=$v" >> gpurun_out/r04v/ab.log
  PSAMD_SIG_WINDOWS=$v timeout -k 10 200 python -u tools/ab_opts.py --workload cfg2 --reps 3 --steps 2000 --variants '[{}]' 2>> gpurun_out/r04v/ab.log > /dev/null || exit 1
done
PSAMD_SIG_WINDOWS=1 timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu > gpurun_out/r04v/bench_cfg2.json 2> gpurun_out/r04v/bench_cfg2.log
