#!/bin/bash
# Alternating A/B of bench.py (cfg3, 30 steps) under two environments.
#   tools/ab_bench.sh <tag> "<env A>" "<env B>" [repeats]
set -euo pipefail
TAG=$1; A=$2; B=$3; N=${4:-3}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$N"); do
  for V in A B; do
    if [ $V = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu > "$OUT/${V}_$i.json" 2> "$OUT/${V}_$i.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.4f ms' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/${V}_$i.json" "$V($E)"
  done
done
