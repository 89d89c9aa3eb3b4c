set -o pipefail
mkdir -p gpurun_out/r04n
export PSAMD_AB=1
for v in "0 0" "8 1500000000" "8 800000000" "6 1500000000"; do
  set -- $v
  echo "small=$1 bytes=$2" >> gpurun_out/r04n/ab.log
  PSAMD_CHAIN_WAVES_SMALL=$1 PSAMD_CHAIN_SMALL_BYTES=$2 timeout -k 10 200 python -u tools/ab_opts.py --workload cfg3 --reps 3 --steps 200 --variants '[{}]' >> gpurun_out/r04n/ab.json 2>> gpurun_out/r04n/ab.log || exit 1
done
