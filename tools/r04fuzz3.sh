set -o pipefail
mkdir -p gpurun_out/r04fuzz3
timeout -k 10 500 python -u tools/fuzz_gpu.py --cases 1500 --seed 406 > gpurun_out/r04fuzz3/fuzz_all_seed406.log 2>&1 || { echo FUZZ_FAILED; tail -20 gpurun_out/r04fuzz3/fuzz_all_seed406.log; exit 1; }
tail -n 1 gpurun_out/r04fuzz3/fuzz_all_seed406.log
timeout -k 10 400 python -u tools/fuzz_gpu.py --cases 2000 --seed 407 --kinds pipeline modes churn > gpurun_out/r04fuzz3/fuzz_pmc_seed407.log 2>&1 || { echo FUZZ_FAILED; tail -20 gpurun_out/r04fuzz3/fuzz_pmc_seed407.log; exit 1; }
tail -n 1 gpurun_out/r04fuzz3/fuzz_pmc_seed407.log
