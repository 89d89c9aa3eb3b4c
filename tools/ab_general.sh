#!/bin/bash
# A/B of the general-path leg (staggered cfg3) under env lists, alternating.
# usage: tools/ab_general.sh OUTDIR REPEATS "ENV1" "ENV2" ...
set -o pipefail
out=$1; reps=$2; shift 2
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    env $envs timeout -k 10 200 python -u bench.py --general-only --steps 8 --warmup 2 --no-cpu \
        > "$out/g${i}_$rep.json" 2> "$out/g${i}_$rep.err" || { echo "variant $i failed: $envs" >> "$out/summary.txt"; exit 1; }
    python3 -c "
import json
g=json.loads(open('$out/g${i}_$rep.json').read().strip().splitlines()[-1])['general_path']
print(f\"[$envs] ms/step {g['ms_per_step']:.3f} device ms/step {g['roofline']['device_ms_per_step']:.3f} compaction {g['compaction']['ms_per_step']:.2f}\")
" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
