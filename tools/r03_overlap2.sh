#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Window-init overlap for every pipelined tree window + reduce on its own stream: tests and benches.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03ovl3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -x -q --timeout 200 --timeout-method thread > $O/pytest_async.log 2>&1
tail -n 1 $O/pytest_async.log
B="python -u bench.py --steps 300 --warmup 5 --no-cpu --no-general --sustain 0"
for rep in 1 2; do
  for W in cfg2 cfg4 cfg3; do
    for OV in 1 0; do
      echo "[ovl] $W overlap=$OV $rep $(date +%T)"
      PSAMD_OVERLAP=$OV timeout -k 10 200 $B --workload $W > $O/${W}_ov${OV}_$rep.json 2> $O/${W}_ov${OV}_$rep.err
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 1 $O/pytest_gpu.log
echo "[ovl] done $(date +%T)"
