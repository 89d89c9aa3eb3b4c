#!/bin/bash
# Evidence on the current default schedule: cfg3 bench line (with the CPU baseline),
# kernel traces of the headline and general path, PMC passes, then cfg4 / cfg2 lines
# and the driver's own bench command.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03b}
TESTS=0 PMC=1 bash tools/gpu_check.sh $TAG
O=gpurun_out/$TAG
for W in cfg4 cfg2; do
  echo "[evidence] $W $(date +%T)"
  timeout -k 10 300 python -u bench.py --workload $W --steps 50 --warmup 5 --sustain 0 > $O/bench_$W.json 2> $O/bench_$W.err
done
echo "[evidence] driver command $(date +%T)"
timeout -k 10 400 python -u bench.py > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
echo "[evidence] done $(date +%T)"
