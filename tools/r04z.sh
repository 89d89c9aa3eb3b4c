set -o pipefail
mkdir -p gpurun_out/r04z
for t in old new old new; do
  if [ $t = old ]; then d=tools/r03tree; else d=.; fi
  echo "$t" >> gpurun_out/r04z/lb.log
  (cd $d && timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 2>&1 | grep "ratio") >> gpurun_out/r04z/lb.log || exit 1
done
