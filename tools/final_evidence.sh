#!/bin/bash
# Round-end evidence: smoke, the driver's bench command (with the CPU
# baseline), the GPU suite + kernel traces + PMC passes (gpu_check), the
# cfg2/cfg4/cfg5 lines and cfg4 on 2 / 4 processes sharing the GPU (IPC transport).
# Every GPU step has its own time limit; set -e stops at the first failure.
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
PMC=1 bash tools/gpu_check.sh $TAG
for W in cfg4 cfg2; do
  echo "[final] $W $(date +%T)"
  timeout -k 10 300 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 > $O/bench_$W.json 2> $O/bench_$W.err
done
echo "[final] cfg5 $(date +%T)"
timeout -k 10 300 python -u bench.py --workload cfg5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
for N in 2 4; do
  echo "[final] $N processes on one GPU (IPC transport, owners' rows in place) $(date +%T)"
  timeout -k 10 300 python -u bench.py --gpus $N --workload cfg4 --no-cpu > $O/bench_cfg4_g${N}_ipc.json 2> $O/bench_cfg4_g${N}_ipc.err
  tail -c 300 $O/bench_cfg4_g${N}_ipc.json
done
echo "[final] done $(date +%T)"
