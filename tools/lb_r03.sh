export PSAMD_AB=1  # plan options from the environment (A/B tools only)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lb
timeout -k 10 400 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 4 > gpurun_out/lb/cfg4_peer4.log 2>&1
timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg3 --scale 1.0 --partition peer --steps 4 > gpurun_out/lb/cfg3_peer4.log 2>&1
timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg3 --scale 1.0 --partition peer --steps 4 --staggered > gpurun_out/lb/cfg3_peer4_stag.log 2>&1
timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition subtree --steps 4 > gpurun_out/lb/cfg4_subtree4.log 2>&1
PSAMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload cfg5 --steps 6 --warmup 2 --no-cpu > gpurun_out/lb/cfg5_timing.json 2> gpurun_out/lb/cfg5_timing.err
