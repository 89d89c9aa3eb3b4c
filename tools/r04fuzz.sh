set -o pipefail
mkdir -p gpurun_out/r04fuzz
timeout -k 10 500 python -u tools/fuzz_gpu.py --cases 1200 --seed 401 > gpurun_out/r04fuzz/fuzz_all_seed401.log 2>&1 || { echo FUZZ_FAILED; tail -20 gpurun_out/r04fuzz/fuzz_all_seed401.log; exit 1; }
tail -n 2 gpurun_out/r04fuzz/fuzz_all_seed401.log
timeout -k 10 400 python -u tools/fuzz_gpu.py --cases 1500 --seed 402 --kinds pipeline modes > gpurun_out/r04fuzz/fuzz_pipeline_seed402.log 2>&1 || { echo FUZZ_FAILED; tail -20 gpurun_out/r04fuzz/fuzz_pipeline_seed402.log; exit 1; }
tail -n 2 gpurun_out/r04fuzz/fuzz_pipeline_seed402.log
