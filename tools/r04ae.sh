#!/bin/bash
# Full GPU suite on the host-path cuts + fused reduce, then cfg2 / cfg3 bench lines.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ae
mkdir -p $O
echo "[ae] tests $(date +%T)"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for W in cfg2 cfg3; do
  echo "[ae] bench $W $(date +%T)"
  timeout -k 10 300 python -u bench.py --workload $W --steps $([ $W = cfg2 ] && echo 2000 || echo 200) --warmup 5 --sustain 0 --no-cpu > $O/bench_$W.json 2> $O/bench_$W.err
  python -c "import json;d=json.loads(open('$O/bench_$W.json').read().splitlines()[-1]);print('$W', d['ms_per_step'])"
done
echo "[ae] done $(date +%T)"
