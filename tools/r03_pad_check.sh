#!/bin/bash
# GPU suite, fuzz and loopback benches on the padded-row default.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03pad}
mkdir -p $O
echo "[pad] tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 1 $O/pytest_gpu.log
echo "[pad] fuzz $(date +%T)"
timeout -k 10 300 python -u tools/fuzz_gpu.py --cases 1000 --seed 71 > $O/fuzz_seed71.log 2>&1
tail -n 1 $O/fuzz_seed71.log
timeout -k 10 300 python -u tools/fuzz_gpu.py --cases 200 --seed 72 --kinds dist --max-world 8 > $O/fuzz_dist_seed72.log 2>&1
tail -n 1 $O/fuzz_dist_seed72.log
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 4"
echo "[pad] loopback $(date +%T)"
$LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
$LB --workload cfg4 --partition subtree > $O/lb_cfg4_subtree4.log 2>&1
$LB --workload cfg3 --partition peer > $O/lb_cfg3_peer4.log 2>&1
$LB --workload cfg3 --partition peer --staggered > $O/lb_cfg3_peer4_stag.log 2>&1
for f in $O/lb_*.log; do tail -n 1 $f; done
echo "[pad] done $(date +%T)"
