set -o pipefail
mkdir -p gpurun_out/r04w
timeout -k 10 900 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_api.py tests/test_gpu_drain.py tests/test_gpu_parity.py tests/test_gpu_groups.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04w/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04w/pytest.log; exit 1; }
export PSAMD_AB=1
for v in 1 0 1 0; do
  echo "reuse=$v" >> gpurun_out/r04w/ab.log
  PSAMD_UPLOAD_REUSE=$v timeout -k 10 200 python -u tools/ab_opts.py --workload cfg2 --reps 3 --steps 2000 --variants '[{}]' 2>> gpurun_out/r04w/ab.log > /dev/null || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04w/trace_cfg2 -o cfg2 -- python3 tools/ab_opts.py --workload cfg2 --reps 1 --steps 300 --variants '[{}]' > /dev/null 2> gpurun_out/r04w/trace.log
