#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Chains from round 1 instead of k_flood for the leading rounds (PSAMD_FLOOD=0), smaller top splits.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abnoflood}
mkdir -p $O
B="python -u bench.py --steps 300 --warmup 5 --no-cpu --no-general --sustain 0"
run() {  # name workload env...
  local n=$1 w=$2; shift 2
  echo "[ab_noflood] $n $w $(date +%T)"
  env "$@" timeout -k 10 200 $B --workload $w > $O/${w}_$n.json 2> $O/${w}_$n.err
}
for rep in 1 2; do
  run base$rep cfg3 PSAMD_X=0
  run noflood$rep cfg3 PSAMD_FLOOD=0
  run noflood_w2k$rep cfg3 PSAMD_FLOOD=0 PSAMD_CHAIN_WORDS=2048
  run top256k$rep cfg3 PSAMD_FLOOD_TOP_BYTES=262144
done
run base cfg2 PSAMD_X=0
run noflood cfg2 PSAMD_FLOOD=0
run base cfg4 PSAMD_X=0
run noflood cfg4 PSAMD_FLOOD=0
echo "[ab_noflood] done $(date +%T)"
