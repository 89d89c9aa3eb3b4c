#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Zero-copy loopback exchange: multi-rank parity, then the 4-rank loopback benches and a trace.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${ZC_OUT:-r03zc}
mkdir -p $O
echo "[zc] tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
tail -n 1 $O/tests.log
LB="timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 4"
echo "[zc] loopback $(date +%T)"
$LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4.log 2>&1
PSAMD_XCHG_OVERLAP=1 $LB --workload cfg4 --partition peer > $O/lb_cfg4_peer4_overlap.log 2>&1
$LB --workload cfg4 --partition subtree > $O/lb_cfg4_subtree4.log 2>&1
$LB --workload cfg3 --partition peer > $O/lb_cfg3_peer4.log 2>&1
$LB --workload cfg3 --partition peer --staggered > $O/lb_cfg3_peer4_stag.log 2>&1
tail -n 1 $O/lb_*.log
echo "[zc] fuzz dist $(date +%T)"
timeout -k 10 300 python -u tools/fuzz_gpu.py --cases 300 --seed 61 --kinds dist --max-world 8 > $O/fuzz_dist_seed61.log 2>&1
tail -n 1 $O/fuzz_dist_seed61.log
echo "[zc] trace $(date +%T)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$O/lbtrace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/loopback_bench.py" --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 3 \
  > "$GRAFT_REPO_ROOT/$O/lb_cfg4_peer4_traced.log" 2>&1
echo "[zc] done $(date +%T)"
