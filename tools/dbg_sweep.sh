#!/bin/bash
# k_expand component costs: PSAMD_DEBUG_EXPAND knobs (results wrong by design).
#   tools/dbg_sweep.sh <tag> "<dbg values>" [bench args]
set -euo pipefail
TAG=$1; VALS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for v in $VALS; do
  PSAMD_DEBUG_EXPAND=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-check "$@" > "$OUT/dbg_$v.json" 2> "$OUT/dbg_$v.err"
  python3 -c "
import json,sys; d=json.load(open('$OUT/dbg_$v.json')); l=d['last_step']
print('dbg=$v', 'ms/step %.3f'%d['ms_per_step'], 'expand_ms %.3f'%l['expand_ms'], 'run_ms %.3f'%l['run_ms'], 'host_ms %.3f'%l['host_ms'], 'per-round', l['expand_us_per_round'][12:21])"
done
