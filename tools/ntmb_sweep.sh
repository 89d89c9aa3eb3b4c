#!/bin/bash
# A/B of the k_pull nt threshold (PSAMD_PULL_NT_MB: rounds writing fewer row
# MB keep the default cache policy)   tools/ntmb_sweep.sh <tag> [bench args...]
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for MB in ${MBS:-0 32 64 128 256}; do
  PSAMD_PULL_NT_MB=$MB timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > "$OUT/mb$MB.json" 2> "$OUT/mb$MB.err"
  python -c "import json; d=json.load(open('$OUT/mb$MB.json')); print('mb=$MB', d['value'], d['ms_per_step'], d['roofline']['frac'], d['last_step'].get('expand_us_per_round'))"
done
