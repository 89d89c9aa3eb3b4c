#!/bin/bash
# Rebuild sort over the (depth, parent) bits only (stable radix sort, keys in
# peer order): churn parity, then cfg5 A/B against PSAMD_SORT_PEER_BITS=1.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ah
mkdir -p $O
echo "[ah] tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_churn.py tests/test_gpu_golden.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for F in 0 1 0 1; do
  echo "[ah] cfg5 peer_bits=$F $(date +%T)"
  PSAMD_AB=1 PSAMD_SORT_PEER_BITS=$F timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu > $O/cfg5_pb$F.json 2> $O/cfg5_pb$F.err
  python -c "import json;d=json.loads(open('$O/cfg5_pb$F.json').read().splitlines()[-1]);c=d['config'];print('ms/batch',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['breakdown_ms_per_step'].items() if isinstance(v,float)})"
done
echo "[ah] done $(date +%T)"
