#!/bin/bash
# Driver command on the final tree (traffic from the refreshed PMC entry), async/dist tests,
# 4-rank loopback benches (overlap streams created lazily).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/pytest_async_dist.log 2>&1
tail -n 1 $O/pytest_async_dist.log
echo "[final2] driver command $(date +%T)"
timeout -k 10 400 python -u bench.py > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 8"
echo "[final2] loopback $(date +%T)"
$LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
$LB --workload cfg4 --partition subtree > $O/lb_cfg4_subtree4.log 2>&1
$LB --workload cfg3 --partition peer > $O/lb_cfg3_peer4.log 2>&1
$LB --workload cfg3 --partition peer --staggered > $O/lb_cfg3_peer4_stag.log 2>&1
for f in $O/lb_*.log; do tail -n 1 $f; done
echo "[final2] done $(date +%T)"
