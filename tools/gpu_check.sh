#!/bin/bash
# One GPU session: parity tests, bench, optional A/B, kernel trace, PMC passes.
#   [AB="ENV=1 ..."] [PMC=1] [TRACE=0] [TESTS=0] [BENCH_ARGS=...] tools/gpu_check.sh <tag> [pytest -k expr]
# Every GPU step has its own time limit; the script stops at the first
# failure (set -e), so nothing runs on the GPU after a fault or a timeout.
set -euo pipefail
TAG=${1:-x}
KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
BARGS=${BENCH_ARGS:-}
mkdir -p "$OUT"
cd "$ROOT"
if [ "${TESTS:-1}" = 1 ]; then
  echo "[gpu_check] tests $(date +%T)"
  KARGS=()
  [ -n "$KEXPR" ] && KARGS=(-k "$KEXPR")
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${KARGS[@]}" > "$OUT/pytest.log" 2>&1
  tail -2 "$OUT/pytest.log"
fi
echo "[gpu_check] bench $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --sustain 3 $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
if [ -n "${AB:-}" ]; then
  echo "[gpu_check] bench A/B ($AB) $(date +%T)"
  env $AB timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu $BARGS > "$OUT/bench_ab.json" 2> "$OUT/bench_ab.err"
  cat "$OUT/bench_ab.json"
fi
cd /tmp && export TMPDIR=/tmp
if [ "${TRACE:-1}" = 1 ]; then
  echo "[gpu_check] trace $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu --no-general --sustain 0 $BARGS > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_general" -o run -- \
    python3 "$ROOT/bench.py" --steps 4 --warmup 1 --no-cpu --general-only $BARGS > "$OUT/bench_trace_general.json" 2> "$OUT/bench_trace_general.err"
fi
if [ "${PMC:-0}" = 1 ]; then
  # headline kernel (no general-path leg), then the general-path leg alone
  for SET in main general; do
    EXTRA="--no-general"
    [ "$SET" = general ] && EXTRA="--general-only"
    for C in FETCH_SIZE WRITE_SIZE; do
      echo "[gpu_check] pmc $SET $C $(date +%T)"
      timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d "$OUT/pmc_${SET}/$C" -o run -- \
        python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu --sustain 0 $EXTRA $BARGS > "$OUT/pmc_${SET}_$C.json" 2> "$OUT/pmc_${SET}_$C.err"
    done
    python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_${SET}" > "$OUT/pmc_summary_${SET}.json"
  done
fi
echo "[gpu_check] done $(date +%T)"
