#!/bin/bash
# PMC passes over a short bench run: SQ stalls, then FETCH_SIZE, then WRITE_SIZE
# (one block-limited pass each; MI355X_MICROARCH.md §rocprofv3 PMC slots).
#   tools/pmc_all.sh <tag> [bench args]
set -uo pipefail
TAG=${1:-x}; shift || true
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 1 --warmup 1 --no-cpu)
run() { name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -T -f csv -d "$OUT/$name" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
  echo "$name rc=$?"; }
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SALU
run fetch FETCH_SIZE
run write WRITE_SIZE
