#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Bench A/B over environment settings (one bench run each, no CPU leg).
#   tools/env_sweep.sh <tag> "<VAR=val[,VAR2=val2]> ..." [bench args]
set -euo pipefail
TAG=$1; SETS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for set in $SETS; do
  name=${set//[=,]/_}
  env ${set//,/ } timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "
import json; d=json.load(open('$OUT/$name.json')); l=d['last_step']
print('$set', 'value %.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'expand_ms %.3f'%l['expand_ms'], 'run_ms %.3f'%l['run_ms'], 'frac %.3f'%d['roofline']['frac'], 'per-round', l['expand_us_per_round'][1:22])"
done
