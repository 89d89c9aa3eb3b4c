set -o pipefail
mkdir -p gpurun_out/r04ab
export PSAMD_AB=1
PSAMD_PAD_ALIGN=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ab/pytest_align16.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04ab/pytest_align16.log; exit 1; }
for w in cfg2 cfg3 cfg4; do
  st=2000; [ $w = cfg3 ] && st=200; [ $w = cfg4 ] && st=100
  for v in "2 1" "16 1" "16 0" "2 0"; do
    set -- $v
    echo "$w align=$1 slice=$2" >> gpurun_out/r04ab/ab.log
    PSAMD_PAD_ALIGN=$1 PSAMD_CHAIN_SLICE_SMALL=$2 timeout -k 10 300 python -u tools/ab_opts.py --workload $w --reps 3 --steps $st --variants '[{}]' 2>> gpurun_out/r04ab/ab.log > /dev/null || exit 1
  done
done
