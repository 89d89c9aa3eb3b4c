#!/bin/bash
# Alternating runs of bench.py (cfg3, 30 steps) under several environments.
#   tools/ab3.sh <tag> "<env 1>" "<env 2>" ... (each env a space-separated list)
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
i=0
for E in "$@"; do
  i=$((i + 1))
  env $E timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu > "$OUT/v$i.json" 2> "$OUT/v$i.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.4f ms' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/v$i.json" "[$E]"
done
