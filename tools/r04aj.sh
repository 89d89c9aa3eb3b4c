#!/bin/bash
# k_expand: current children's words loaded ahead of their stores (hoist):
# full GPU suite, then the compaction leg A/B against PSAMD_EXPAND_HOIST=0.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04aj
mkdir -p $O
echo "[aj] tests $(date +%T)"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for H in 1 0 1 0; do
  echo "[aj] general hoist=$H $(date +%T)"
  PSAMD_AB=1 PSAMD_EXPAND_HOIST=$H timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu --general-only > $O/gen_h$H.json 2> $O/gen_h$H.err
  python -c "import json;d=json.loads(open('$O/gen_h$H.json').read().splitlines()[-1]);c=d['general_path']['compaction'];print('hoist=$H compaction ms/step',round(c['ms_per_step'],3),'k_expand frac',round(c['roofline']['frac'],3),'avg us',round(c['roofline']['avg_launch_us'],1))"
done
echo "[aj] done $(date +%T)"
