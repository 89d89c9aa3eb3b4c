#!/bin/bash
# The held-back reduce A/B again, with PSAMD_AB=1 (r04ad set the switch without
# it, so both of its legs ran fused): bench.py cfg2 lines alternating.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aq
mkdir -p $O
for F in 1 0 1 0 1 0; do
  PSAMD_AB=1 PSAMD_FUSE_REDUCE=$F timeout -k 10 200 python -u bench.py --workload cfg2 --steps 2000 --warmup 5 --sustain 0 --no-cpu > $O/cfg2_f$F.json 2> $O/cfg2_f$F.err
  python -c "import json;d=json.loads(open('$O/cfg2_f$F.json').read().splitlines()[-1]);print('cfg2 fuse=$F', round(d['ms_per_step']*1e3,2), 'us/step')"
done
