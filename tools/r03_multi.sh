#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Round-3 GPU session: the 4-rank loopback exchange (overlap on/off, both
# partitions, staggered), its kernel trace, cfg5 host timing, and the MALL
# A/B (chunk direction x phase-B store policy).  Every GPU step under its own
# time limit; set -e stops at the first failure.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03m
mkdir -p $O
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 4"
echo "[r03m] loopback $(date +%T)"
$LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
PSAMD_XCHG_OVERLAP=0 $LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4_nooverlap.log 2>&1
$LB --workload cfg4 --partition subtree > $O/lb_cfg4_subtree4.log 2>&1
$LB --workload cfg3 --partition peer > $O/lb_cfg3_peer4.log 2>&1
$LB --workload cfg3 --partition peer --staggered > $O/lb_cfg3_peer4_stag.log 2>&1
tail -n 1 $O/lb_*.log
echo "[r03m] cfg5 $(date +%T)"
PSAMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload cfg5 --steps 6 --warmup 2 --no-cpu > $O/cfg5_timing.json 2> $O/cfg5_timing.err
echo "[r03m] trace $(date +%T)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$O/lbtrace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/loopback_bench.py" --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 3 \
  > "$GRAFT_REPO_ROOT/$O/lb_cfg4_peer4_traced.log" 2>&1
cd "$GRAFT_REPO_ROOT"
echo "[r03m] mall A/B $(date +%T)"
B="python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 0"
for W in cfg3 cfg4; do
  timeout -k 10 200 $B --workload $W > $O/ab_${W}_base.json 2>$O/ab_${W}_base.err
  PSAMD_REVERSE=1 timeout -k 10 200 $B --workload $W > $O/ab_${W}_rev.json 2>$O/ab_${W}_rev.err
  PSAMD_REVERSE=1 PSAMD_NT_BYTES=1000000000000000 timeout -k 10 200 $B --workload $W > $O/ab_${W}_rev_cache.json 2>$O/ab_${W}_rev_cache.err
done
echo "[r03m] done $(date +%T)"
