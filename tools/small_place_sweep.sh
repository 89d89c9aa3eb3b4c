#!/bin/bash
# A/B of the one-block top-level placement threshold (PSAMD_SMALL_PLACE) on cfg5
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/${1:-spw}
mkdir -p "$OUT"
cd "$ROOT"
for V in ${VALS:-0 512 2048 8192}; do
  PSAMD_SMALL_PLACE=$V PSAMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu --steps 20 > "$OUT/v$V.json" 2> "$OUT/v$V.err"
  python - "$OUT/v$V.err" "$V" <<'PY'
import re, sys
rows = [l for l in open(sys.argv[1]) if "gpu build" in l][5:]
f = lambda k: sum(float(re.search(k + r" ([0-9.]+) ms", l).group(1)) for l in rows) / len(rows)
print(f"small={sys.argv[2]}: placement enqueue {f('placement enqueue'):.3f} ms, drain {f('drain'):.3f} ms, n={len(rows)}")
PY
done
