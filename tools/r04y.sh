set -o pipefail
mkdir -p gpurun_out/r04y
export PSAMD_AB=1
for v in 1 0 1; do
  echo "xchg_overlap=$v" >> gpurun_out/r04y/lb.log
  PSAMD_XCHG_OVERLAP=$v timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 2>&1 | grep "ratio" >> gpurun_out/r04y/lb.log || exit 1
done
