#!/bin/bash
# A/B of k_pull chunk size (PSAMD_PULL_WORDS)   tools/words_sweep.sh <tag> [bench args]
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for W in ${WORDS:-512 1024 1536 2048}; do
  PSAMD_PULL_WORDS=$W timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > "$OUT/w$W.json" 2> "$OUT/w$W.err"
  python -c "import json; d=json.load(open('$OUT/w$W.json')); print('words=$W', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
