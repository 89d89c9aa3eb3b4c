set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pair.py tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_groups.py tests/test_gpu_fullsize.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r04e/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04e/pytest.log; exit 1; }
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg3 --reps 4 --steps 200 --variants '[{}, {"chain_words": 4096}, {"chain_words": 16384}, {"chain_max": 5}]' > gpurun_out/r04e/ab_cfg3.json 2> gpurun_out/r04e/ab_cfg3.log
timeout -k 10 300 python -u tools/chain_profile.py --steps 3 > gpurun_out/r04e/chain_prof_cfg3.json 2> gpurun_out/r04e/chain_prof.log
