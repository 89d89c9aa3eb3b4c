set -o pipefail
mkdir -p gpurun_out/r04aa
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_fullsize.py tests/test_gpu_pair.py tests/test_gpu_groups.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r04aa/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r04aa/pytest.log; exit 1; }
export PSAMD_AB=1
for w in cfg2 cfg3 cfg4; do
  st=2000; [ $w = cfg3 ] && st=200; [ $w = cfg4 ] && st=100
  for v in 1 0; do
    echo "$w slice_small=$v" >> gpurun_out/r04aa/ab.log
    PSAMD_CHAIN_SLICE_SMALL=$v timeout -k 10 300 python -u tools/ab_opts.py --workload $w --reps 3 --steps $st --variants '[{}]' 2>> gpurun_out/r04aa/ab.log > /dev/null || exit 1
  done
done
PSAMD_CHAIN_SLICE_SMALL=1 timeout -k 10 200 python3 tools/chain_profile.py --workload cfg2 --steps 3 > gpurun_out/r04aa/chain_prof_cfg2.json 2> gpurun_out/r04aa/chain_prof_cfg2.log
