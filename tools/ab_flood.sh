#!/bin/bash
# A/B of k_flood variants on the bench workload (timing only: --no-check).
# usage: tools/ab_flood.sh OUTDIR "ENV1" "ENV2" ...   (each ENV a space-separated list of VAR=value)
set -o pipefail
out=$1; shift
mkdir -p "$out"
wl=${WL:-cfg3}
i=0
for envs in "$@"; do
  i=$((i + 1))
  echo "== $envs" >> "$out/summary.txt"
  env $envs timeout -k 10 200 python -u bench.py --workload "$wl" --steps 10 --warmup 3 --no-cpu --no-check \
      > "$out/v$i.json" 2> "$out/v$i.err" || { echo "variant $i failed: $envs" >> "$out/summary.txt"; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$out/v$i.json').read().strip().splitlines()[-1])
r=d['roofline']
ks='  '.join(f\"{k}: {v['launches']}x{v['avg_launch_us']:.1f} us frac {v['frac']:.3f}\" for k, v in r.get('kernels', {}).items())
print(f\"  value {d['value']:.3e}  ms/step {d['ms_per_step']:.3f}  {r['kernel']} {r['avg_launch_us']:.1f} us  frac {r['frac']:.3f}  flood_rounds {d['last_step'].get('flood_rounds')}  [{ks}]\")
" >> "$out/summary.txt"
done
cat "$out/summary.txt"
