#!/bin/bash
# Collects the rocprofv3 evidence for bench.py's roofline line on an MI355X box.
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats (per-kernel average duration)
# 2) separate PMC passes: FETCH_SIZE, then WRITE_SIZE (TCC slots: 3 + 2, one
#    pass each, MI355X_MICROARCH.md §rocprofv3 PMC slots)
set -euo pipefail
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 5 --warmup 1 --no-cpu)
echo "[profile] trace $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
echo "[profile] pmc FETCH_SIZE $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu "${@:3}" > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
echo "[profile] pmc WRITE_SIZE $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$OUT/pmc_write" -o run -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu "${@:3}" > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
echo "[profile] done $(date +%T)"
find "$OUT" -name "*.csv" | head -20
