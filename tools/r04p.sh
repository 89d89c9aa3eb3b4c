set -o pipefail
mkdir -p gpurun_out/r04p
export PSAMD_AB=1
for v in 0 1000000000000 0 1000000000000; do
  echo "fork_bytes=$v" >> gpurun_out/r04p/ab.log
  PSAMD_REDUCE_FORK_BYTES=$v timeout -k 10 200 python -u tools/ab_opts.py --workload cfg2 --reps 3 --steps 2000 --variants '[{}]' >> gpurun_out/r04p/ab.json 2>> gpurun_out/r04p/ab.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04p/trace_cfg2 -o cfg2 -- python3 bench.py --workload cfg2 --no-cpu --steps 60 --warmup 3 --sustain 0 > gpurun_out/r04p/bench_cfg2.json 2> gpurun_out/r04p/bench_cfg2.log
timeout -k 10 300 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{}]' > gpurun_out/r04p/ab_cfg3.json 2> gpurun_out/r04p/ab_cfg3.log
timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 6 > gpurun_out/r04p/lb_cfg4_peer4.log 2>&1
