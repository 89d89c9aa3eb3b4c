#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Per-launch device times (tools/round_timing.py) under planner switches.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RT_OUT:-rt2}
mkdir -p $O
RT="timeout -k 10 120 python -u tools/round_timing.py"
i=0
while read -r w envs; do
  i=$((i+1))
  env $envs $RT $w > $O/$(printf %02d $i)_$w.txt 2>&1
done <<'LIST'
cfg3 PSAMD_CHAIN=5
cfg3 PSAMD_CHAIN=6
cfg3 PSAMD_FLOOD=0 PSAMD_CHAIN=5
cfg3 PSAMD_FLOOD=0 PSAMD_CHAIN=6
cfg4 PSAMD_X=0
cfg4 PSAMD_FLOOD=0
cfg4 PSAMD_FLOOD=0 PSAMD_CHAIN=6
LIST
echo done
