set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pair.py tests/test_gpu_parity.py tests/test_gpu_flood.py tests/test_gpu_async.py tests/test_gpu_groups.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b/pytest.log 2>&1 || { echo PYTEST_FAILED; exit 1; }
timeout -k 10 300 python -u tools/chain_profile.py --steps 3 > gpurun_out/r04b/chain_prof_cfg3.json 2> gpurun_out/r04b/chain_prof.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 3 > gpurun_out/r04b/bench_cfg3.json 2> gpurun_out/r04b/bench_cfg3.log
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 500 --warmup 5 --no-cpu --no-general --sustain 3 > gpurun_out/r04b/bench_cfg2.json 2> gpurun_out/r04b/bench_cfg2.log
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 200 --warmup 5 --no-cpu --no-general --sustain 0 > gpurun_out/r04b/bench_cfg4.json 2> gpurun_out/r04b/bench_cfg4.log
