#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# General path (start rounds 0..7) by the longest launch (PSAMD_CHAIN 2/4/6).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abgen}
mkdir -p $O
for L in 2 4 6; do
  echo "[ab_general] chain $L $(date +%T)"
  PSAMD_CHAIN=$L timeout -k 10 300 python -u bench.py --general-only --steps 20 --warmup 3 --no-cpu > $O/general_chain$L.json 2> $O/general_chain$L.err
done
echo "[ab_general] done $(date +%T)"
