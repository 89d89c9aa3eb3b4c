set -o pipefail
mkdir -p gpurun_out/r04ac
export PSAMD_AB=1
PSAMD_CHAIN2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_groups.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ac/pytest_chain2.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04ac/pytest_chain2.log; exit 1; }
for w in cfg2 cfg3 cfg4; do
  st=2000; [ $w = cfg3 ] && st=200; [ $w = cfg4 ] && st=100
  for v in 1 0 1 0; do
    echo "$w chain2=$v" >> gpurun_out/r04ac/ab.log
    PSAMD_CHAIN2=$v timeout -k 10 300 python -u tools/ab_opts.py --workload $w --reps 3 --steps $st --variants '[{}]' 2>> gpurun_out/r04ac/ab.log > /dev/null || exit 1
  done
done
