#!/bin/bash
# A/B of k_pull cache policies (PSAMD_PULL_NT = 0 plain, 1 nt stores, 2 nt loads, 3 both)
#   tools/nt_sweep.sh <tag> [bench args...]
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for NT in ${NTS:-0 1 2 3}; do
  PSAMD_PULL_NT=$NT timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > "$OUT/nt$NT.json" 2> "$OUT/nt$NT.err"
  python -c "import json; d=json.load(open('$OUT/nt$NT.json')); print('nt=$NT', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
