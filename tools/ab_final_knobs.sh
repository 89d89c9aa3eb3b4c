#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Last knob sweep on the final tree: chain length, chain run size, deep-window floor for cfg4.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abknobs}
mkdir -p $O
B="python -u bench.py --steps 500 --warmup 5 --no-cpu --no-general --sustain 0"
run() { local n=$1 w=$2; shift 2; env "$@" timeout -k 10 200 $B --workload $w > $O/${w}_$n.json 2> $O/${w}_$n.err; }
for rep in 1 2; do
  run base$rep cfg3 PSAMD_X=0
  run chain5_$rep cfg3 PSAMD_CHAIN=5
  run words16k_$rep cfg3 PSAMD_CHAIN_WORDS=16384
  run base$rep cfg4 PSAMD_X=0
  run deep10_$rep cfg4 PSAMD_OVERLAP_ROUNDS=10
done
echo done
