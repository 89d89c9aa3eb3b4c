set -o pipefail
mkdir -p gpurun_out/r04o
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04o/trace_cfg2 -o cfg2 -- python3 bench.py --workload cfg2 --no-cpu --steps 60 --warmup 3 --sustain 0 > gpurun_out/r04o/bench_cfg2.json 2> gpurun_out/r04o/bench_cfg2.log
PSAMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu --steps 6 --warmup 2 > gpurun_out/r04o/bench_cfg5.json 2> gpurun_out/r04o/bench_cfg5.log
