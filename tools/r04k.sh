set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04k/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04k/pytest.log; exit 1; }
timeout -k 10 500 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{"chain_waves": 0}, {"chain_waves": 14}, {"chain_waves": 12}, {"chain_waves": 10}, {"chain_waves": 8}, {"chain_waves": 6}]' > gpurun_out/r04k/ab_cfg3.json 2> gpurun_out/r04k/ab_cfg3.log
PSAMD_AB=1 PSAMD_CHAIN_WAVES=16 timeout -k 10 300 python -u tools/chain_profile.py --steps 3 --out gpurun_out/r04k/cp16.bin > gpurun_out/r04k/chain_prof_w16.json 2> gpurun_out/r04k/chain_prof.log
PSAMD_AB=1 PSAMD_CHAIN_WAVES=10 timeout -k 10 300 python -u tools/chain_profile.py --steps 3 --out gpurun_out/r04k/cp10.bin > gpurun_out/r04k/chain_prof_w10.json 2>> gpurun_out/r04k/chain_prof.log
