#!/bin/bash
# 4-rank loopback on one GPU: HIP maps the ranks' streams onto the process's
# hardware queues (GPU_MAX_HW_QUEUES, 4 by default): with 4 ranks two of them
# share a queue and their launches serialise.  A queue per rank's stream:
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ao
mkdir -p $O
for Q in 4 8 16 8 4; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 8 --workload cfg4 --partition peer > $O/lb_q$Q.log 2>&1
  echo "queues=$Q $(tail -n 1 $O/lb_q$Q.log)"
done
