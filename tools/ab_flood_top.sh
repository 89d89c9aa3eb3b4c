#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# The k_flood / multi-round-launch split (PSAMD_FLOOD_TOP_BYTES) with chains, cfg2 / cfg3 / cfg4.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abtop}
mkdir -p $O
B="python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 0"
for W in cfg2 cfg3 cfg4; do
  for T in 1048576 4194304 16777216 67108864; do
    echo "[ab_top] $W $T $(date +%T)"
    PSAMD_FLOOD_TOP_BYTES=$T timeout -k 10 200 $B --workload $W > $O/${W}_$T.json 2> $O/${W}_$T.err
  done
done
echo "[ab_top] done $(date +%T)"
