#!/bin/bash
# Round-end evidence: GPU suite, driver bench command with CPU baseline, kernel
# traces + PMC passes (gpu_check), cfg2/cfg4/cfg5 lines, 4-rank loopback.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
echo "[final] smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -n 1 $O/smoke.log
echo "[final] driver command $(date +%T)"
timeout -k 10 400 python -u bench.py > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
TESTS=0 PMC=1 bash tools/gpu_check.sh $TAG
for W in cfg4 cfg2; do
  echo "[final] $W $(date +%T)"
  timeout -k 10 300 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 > $O/bench_$W.json 2> $O/bench_$W.err
done
echo "[final] cfg5 $(date +%T)"
timeout -k 10 300 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
echo "[final] loopback $(date +%T)"
timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 8 --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
tail -n 1 $O/lb_cfg4_peer4.log
echo "[final] done $(date +%T)"
