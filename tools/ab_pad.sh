#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Row padding to an even word count from PSAMD_PAD_WORDS words (16-B stores): cfg3 and the
# 4-rank loopback (63-word rows), then the per-launch sweep.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abpad}
mkdir -p $O
B="python -u bench.py --steps 300 --warmup 5 --no-cpu --no-general --sustain 0"
for P in 64 16 8; do
  echo "[ab_pad] cfg3 $P $(date +%T)"
  PSAMD_PAD_WORDS=$P timeout -k 10 200 $B --workload cfg3 > $O/cfg3_$P.json 2> $O/cfg3_$P.err
  PSAMD_PAD_WORDS=$P PSAMD_FLOOD=0 timeout -k 10 200 $B --workload cfg3 > $O/cfg3_nf_$P.json 2> $O/cfg3_nf_$P.err
done
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 4 --workload cfg4 --partition peer"
for P in 64 16; do
  echo "[ab_pad] loopback $P $(date +%T)"
  PSAMD_PAD_WORDS=$P $LB > $O/lb_cfg4_peer4_$P.log 2>&1
done
RT_OUT=rt2 bash tools/rt_sweep.sh
echo "[ab_pad] done $(date +%T)"
