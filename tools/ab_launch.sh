#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# The planner's launch cost (PSAMD_LAUNCH_BYTES: a launch's ramp and tail as row bytes):
# cfg3 plans 3+4+4+1 rounds at 16 MB, 4+4+4 at 128 MB.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ablaunch}
mkdir -p $O
B="python -u bench.py --steps 300 --warmup 5 --no-cpu --no-general --sustain 0"
for rep in 1 2; do
  for W in cfg3 cfg2 cfg4; do
    for LB in 16e6 128e6; do
      echo "[ab_launch] $W $LB $rep $(date +%T)"
      PSAMD_LAUNCH_BYTES=$LB timeout -k 10 200 $B --workload $W > $O/${W}_${LB}_$rep.json 2> $O/${W}_${LB}_$rep.err
    done
  done
done
echo "[ab_launch] done $(date +%T)"
