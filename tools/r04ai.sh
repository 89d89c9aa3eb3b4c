#!/bin/bash
# cfg5 A/B repeated: sort over (depth, parent) bits (0) vs every bit (1).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ai
mkdir -p $O
for F in 1 0 1 0 1 0; do
  PSAMD_AB=1 PSAMD_SORT_PEER_BITS=$F timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu --steps 20 > $O/cfg5_pb$F.json 2> $O/cfg5_pb$F.err
  python -c "import json;d=json.loads(open('$O/cfg5_pb$F.json').read().splitlines()[-1]);print('peer_bits=$F ms/batch',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['breakdown_ms_per_step'].items()})"
done
