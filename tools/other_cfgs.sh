#!/bin/bash
# cfg4 / cfg5 benches with kernel traces, and the 4-rank loopback probe.
#   tools/other_cfgs.sh <tag>
set -euo pipefail
TAG=${1:-cfgs}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for W in cfg4 cfg5; do
  echo "[other_cfgs] $W $(date +%T)"
  timeout -k 10 400 python -u bench.py --workload $W --steps 10 --warmup 2 > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  cut -c1-300 "$OUT/bench_$W.json"
done
echo "[other_cfgs] loopback $(date +%T)"
timeout -k 10 300 python -u tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --steps 3 > "$OUT/loopback4.log" 2>&1
tail -5 "$OUT/loopback4.log"
cd /tmp && export TMPDIR=/tmp
for W in cfg4 cfg5; do
  echo "[other_cfgs] trace $W $(date +%T)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_$W" -o run -- \
    python3 "$ROOT/bench.py" --workload $W --steps 5 --warmup 1 --no-cpu > "$OUT/bench_trace_$W.json" 2> "$OUT/bench_trace_$W.err"
done
echo "[other_cfgs] done $(date +%T)"
