set -o pipefail
mkdir -p gpurun_out/r04s
for c in 0 1 0 1; do
  echo "system_events=$c" >> gpurun_out/r04s/lb2.log
  PSAMD_SYSTEM_EVENTS=$c timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 2>&1 | grep "ratio" >> gpurun_out/r04s/lb2.log || exit 1
done
for c in 0 1; do
  echo "system_events=$c" >> gpurun_out/r04s/ab2.log
  PSAMD_SYSTEM_EVENTS=$c timeout -k 10 300 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{}]' 2>> gpurun_out/r04s/ab2.log >/dev/null || exit 1
done
