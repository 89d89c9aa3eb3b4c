#!/bin/bash
# One GPU session: parity tests, bench A/B, kernel-trace profile.
#   tools/gpu_check.sh <tag> [pytest -k expr]
# Every GPU step has its own time limit; the script stops at the first
# failure (set -e), so nothing runs on the GPU after a fault or a timeout.
set -euo pipefail
TAG=${1:-x}
KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "[gpu_check] tests $(date +%T)"
if [ -n "$KEXPR" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$KEXPR" > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
fi
tail -3 "$OUT/pytest.log"
echo "[gpu_check] bench $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
echo "[gpu_check] bench A/B (PSAMD_NO_LEVEL=1) $(date +%T)"
PSAMD_NO_LEVEL=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > "$OUT/bench_nolevel.json" 2> "$OUT/bench_nolevel.err"
cat "$OUT/bench_nolevel.json"
echo "[gpu_check] trace $(date +%T)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cat {} \;
echo "[gpu_check] done $(date +%T)"
