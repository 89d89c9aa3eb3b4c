set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04l/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04l/pytest.log; exit 1; }
timeout -k 10 500 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{"chain_waves": 0}, {"chain_waves": 12}, {"chain_waves": 8}, {"chain_waves": 14}]' > gpurun_out/r04l/ab_cfg3.json 2> gpurun_out/r04l/ab_cfg3.log
PSAMD_AB=1 PSAMD_CHAIN_WAVES=12 timeout -k 10 300 python -u tools/chain_profile.py --steps 3 --out gpurun_out/r04l/cp12.bin > gpurun_out/r04l/chain_prof_w12.json 2> gpurun_out/r04l/chain_prof.log
PSAMD_AB=1 PSAMD_CHAIN_WAVES=8 timeout -k 10 300 python -u tools/chain_profile.py --steps 3 --out gpurun_out/r04l/cp8.bin > gpurun_out/r04l/chain_prof_w8.json 2>> gpurun_out/r04l/chain_prof.log
