#!/bin/bash
# 4-rank loopback with fewer hardware queues (the ranks' launches serialise
# instead of contending for HBM); each run under its own time limit.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ap
mkdir -p $O
for Q in 2 1 2 1; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 150 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 8 --workload cfg4 --partition peer > $O/lb_q$Q.log 2>&1
  echo "queues=$Q $(tail -n 1 $O/lb_q$Q.log)"
done
