set -o pipefail
mkdir -p gpurun_out/r04fuzz2
timeout -k 10 400 python -u tools/fuzz_gpu.py --cases 1500 --seed 403 --kinds pipeline > gpurun_out/r04fuzz2/fuzz_pipeline_seed403.log 2>&1 || { echo FUZZ_FAILED; tail -20 gpurun_out/r04fuzz2/fuzz_pipeline_seed403.log; exit 1; }
tail -n 2 gpurun_out/r04fuzz2/fuzz_pipeline_seed403.log
timeout -k 10 500 python -u tools/fuzz_gpu.py --cases 1200 --seed 404 > gpurun_out/r04fuzz2/fuzz_all_seed404.log 2>&1 || { echo FUZZ_FAILED; tail -20 gpurun_out/r04fuzz2/fuzz_all_seed404.log; exit 1; }
tail -n 2 gpurun_out/r04fuzz2/fuzz_all_seed404.log
