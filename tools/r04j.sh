set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04j/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04j/pytest.log; exit 1; }
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg3 --reps 4 --steps 200 --variants '[{}, {"chain_persist": 0}]' > gpurun_out/r04j/ab_cfg3.json 2> gpurun_out/r04j/ab_cfg3.log
timeout -k 10 300 python -u tools/chain_profile.py --steps 3 > gpurun_out/r04j/chain_prof_cfg3.json 2> gpurun_out/r04j/chain_prof.log
