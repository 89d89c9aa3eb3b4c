export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# A/B: alternating chunk direction (PSAMD_REVERSE) x phase-B store policy (PSAMD_NT_BYTES) on cfg3 / cfg4
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/abmall
mkdir -p $O
B="python -u bench.py --steps 300 --warmup 5 --no-cpu --no-general --sustain 0"
for W in cfg3 cfg4; do
  timeout -k 10 200 $B --workload $W > $O/${W}_base.json 2>$O/${W}_base.err
  PSAMD_REVERSE=1 timeout -k 10 200 $B --workload $W > $O/${W}_rev.json 2>$O/${W}_rev.err
  PSAMD_REVERSE=1 PSAMD_NT_BYTES=1000000000000000 timeout -k 10 200 $B --workload $W > $O/${W}_rev_cache.json 2>$O/${W}_rev_cache.err
  PSAMD_NT_BYTES=1000000000000000 timeout -k 10 200 $B --workload $W > $O/${W}_cache.json 2>$O/${W}_cache.err
done
PSAMD_REVERSE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pair.py tests/test_gpu_flood.py tests/test_gpu_dist.py > $O/tests_rev.log 2>&1
