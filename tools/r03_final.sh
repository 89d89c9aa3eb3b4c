#!/bin/bash
# Round-3 final evidence: bench line with CPU baseline, traces and PMC passes (gpu_check),
# cfg2/cfg4/cfg5 lines, 4-rank loopback benches.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03f}
TESTS=0 PMC=1 bash tools/gpu_check.sh $TAG
O=gpurun_out/$TAG
for W in cfg4 cfg2; do
  echo "[final] $W $(date +%T)"
  timeout -k 10 300 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 > $O/bench_$W.json 2> $O/bench_$W.err
done
echo "[final] cfg5 $(date +%T)"
timeout -k 10 300 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 8"
echo "[final] loopback $(date +%T)"
$LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
$LB --workload cfg4 --partition subtree > $O/lb_cfg4_subtree4.log 2>&1
$LB --workload cfg3 --partition peer > $O/lb_cfg3_peer4.log 2>&1
$LB --workload cfg3 --partition peer --staggered > $O/lb_cfg3_peer4_stag.log 2>&1
for f in $O/lb_*.log; do tail -n 1 $f; done
echo "[final] done $(date +%T)"
