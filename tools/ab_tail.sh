#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# A chain ending at the window's last round may take one round more (PSAMD_CHAIN_TAIL): cfg3 A/B, chain tests.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abtail}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_async.py tests/test_gpu_pair.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
B="python -u bench.py --steps 500 --warmup 5 --no-cpu --no-general --sustain 0"
for rep in 1 2 3; do
  for T in 1 0; do
    echo "[ab_tail] cfg3 tail=$T $rep $(date +%T)"
    PSAMD_CHAIN_TAIL=$T timeout -k 10 200 $B --workload cfg3 > $O/cfg3_t${T}_$rep.json 2> $O/cfg3_t${T}_$rep.err
  done
done
PSAMD_CHAIN_TAIL=1 timeout -k 10 120 python -u tools/round_timing.py cfg3 > $O/rt_tail1.txt 2>&1
PSAMD_CHAIN_TAIL=0 timeout -k 10 120 python -u tools/round_timing.py cfg3 > $O/rt_tail0.txt 2>&1
echo "[ab_tail] done $(date +%T)"
