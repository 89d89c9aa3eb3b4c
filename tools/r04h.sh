set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04h/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04h/pytest.log; exit 1; }
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg3 --reps 4 --steps 200 --variants '[{}, {"chain_max": 4}]' > gpurun_out/r04h/ab_cfg3.json 2> gpurun_out/r04h/ab_cfg3.log
timeout -k 10 300 python -u tools/chain_profile.py --steps 3 > gpurun_out/r04h/chain_prof_cfg3.json 2> gpurun_out/r04h/chain_prof.log
