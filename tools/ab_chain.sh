#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Chain parity tests, then the chain-length A/B (PSAMD_CHAIN = 2 pairs, 3, 4, 6) on cfg3 / cfg4 / cfg2.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abchain}
mkdir -p $O
echo "[ab_chain] tests $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_pair.py tests/test_gpu_churn.py tests/test_gpu_dist.py tests/test_gpu_golden.py > $O/tests.log 2>&1
tail -n 2 $O/tests.log
B="python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 0"
for W in cfg3 cfg4 cfg2; do
  for L in 2 3 4 6; do
    echo "[ab_chain] $W chain $L $(date +%T)"
    PSAMD_CHAIN=$L timeout -k 10 200 $B --workload $W > $O/${W}_chain$L.json 2> $O/${W}_chain$L.err
  done
done
echo "[ab_chain] done $(date +%T)"
