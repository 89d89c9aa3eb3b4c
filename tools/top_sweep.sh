#!/bin/bash
# Sweep of the top-launch threshold (PSAMD_PULL_TOP_MB): cfg3 bench per value.
#   tools/top_sweep.sh <tag> [values...]
set -euo pipefail
TAG=${1:-top}; shift || true
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
VALS=("$@")
[ ${#VALS[@]} -eq 0 ] && VALS=(0 8 16 32 64 128)
for V in "${VALS[@]}"; do
  PSAMD_PULL_TOP_MB=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > "$OUT/top_$V.json" 2> "$OUT/top_$V.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], '%.4f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], 'avg_us %.1f' % d['roofline']['avg_launch_us'])" "$OUT/top_$V.json" "$V"
done
