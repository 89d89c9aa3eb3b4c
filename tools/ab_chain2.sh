#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Full GPU suite on the chain default, then chain tuning A/B: compact LDS (20 waves/CU)
# and the per-wave row-word target, on cfg3 / cfg4.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abchain2}
mkdir -p $O
echo "[ab_chain2] tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 2 $O/pytest.log
B="python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 0"
for W in cfg3 cfg4; do
  for V in base compact w4096 w16384 compact_w4096; do
    case $V in
      base) E="";;
      compact) E="PSAMD_CHAIN_COMPACT=1";;
      w4096) E="PSAMD_CHAIN_WORDS=4096";;
      w16384) E="PSAMD_CHAIN_WORDS=16384";;
      compact_w4096) E="PSAMD_CHAIN_COMPACT=1 PSAMD_CHAIN_WORDS=4096";;
    esac
    echo "[ab_chain2] $W $V $(date +%T)"
    env $E timeout -k 10 200 $B --workload $W > $O/${W}_$V.json 2> $O/${W}_$V.err
  done
done
echo "[ab_chain2] cfg5 $(date +%T)"
PSAMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload cfg5 --steps 10 --warmup 3 --no-cpu > $O/cfg5.json 2> $O/cfg5.err
echo "[ab_chain2] done $(date +%T)"
