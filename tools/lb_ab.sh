export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# A/B of the multi-rank exchange overlap on the 4-rank cfg4 loopback (peer hash)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lbab
timeout -k 10 400 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 > gpurun_out/lbab/overlap.log 2>&1
PSAMD_XCHG_OVERLAP=0 timeout -k 10 400 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 > gpurun_out/lbab/no_overlap.log 2>&1
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/lbab/dist_tests.log 2>&1
PSAMD_XCHG_OVERLAP=0 timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/lbab/dist_tests_noov.log 2>&1
