set -o pipefail
mkdir -p gpurun_out/r04r
timeout -k 10 900 python -u -m pytest tests/test_gpu_flood.py tests/test_gpu_pair.py tests/test_gpu_fullsize.py tests/test_gpu_groups.py tests/test_gpu_dist.py tests/test_gpu_churn.py tests/test_gpu_golden.py tests/test_gpu_chain.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r04r/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04r/pytest.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu > gpurun_out/r04r/bench_cfg2.json 2> gpurun_out/r04r/bench_cfg2.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04r/trace_cfg2 -o cfg2 -- python3 bench.py --workload cfg2 --no-cpu --steps 60 --warmup 3 --sustain 0 > gpurun_out/r04r/bench_cfg2_traced.json 2> gpurun_out/r04r/bench_cfg2_traced.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04r/trace_lb -o lb -- python3 tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 > gpurun_out/r04r/lb_cfg4_peer4_traced.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04r/trace_cfg5 -o cfg5 -- python3 bench.py --workload cfg5 --no-cpu --steps 4 --warmup 1 > gpurun_out/r04r/bench_cfg5_traced.json 2> gpurun_out/r04r/bench_cfg5_traced.log
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/r04r/bench_cfg5.json 2> gpurun_out/r04r/bench_cfg5.log
timeout -k 10 400 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{}, {"chain_per_wave": 2}, {"chain_per_wave": 3}, {"chain_per_wave": 4}]' > gpurun_out/r04r/ab_cfg3_per.json 2> gpurun_out/r04r/ab_cfg3_per.log
timeout -k 10 400 python -u tools/ab_opts.py --workload cfg4 --reps 3 --steps 100 --variants '[{}, {"chain_per_wave": 2}]' > gpurun_out/r04r/ab_cfg4_per.json 2> gpurun_out/r04r/ab_cfg4_per.log
