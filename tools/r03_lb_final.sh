#!/bin/bash
# 4-rank loopback benches on the final tree.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03lb}
mkdir -p $O
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 8"
$LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
$LB --workload cfg4 --partition subtree > $O/lb_cfg4_subtree4.log 2>&1
$LB --workload cfg3 --partition peer > $O/lb_cfg3_peer4.log 2>&1
$LB --workload cfg3 --partition peer --staggered > $O/lb_cfg3_peer4_stag.log 2>&1
for f in $O/lb_*.log; do tail -n 1 $f; done
