#!/bin/bash
# Chain launches with their whole-row chunks heaviest first (PSAMD_CHAIN_LPT):
# chain / fullsize parity with it on, then cfg3 / cfg4 A/B alternating.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04at
mkdir -p $O
PSAMD_AB=1 PSAMD_CHAIN_LPT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_fullsize.py tests/test_gpu_async.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for W in cfg3 cfg4; do
  for V in 1 0 1 0 1 0; do
    PSAMD_AB=1 PSAMD_CHAIN_LPT=$V timeout -k 10 200 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 --no-cpu --no-general > $O/${W}_l$V.json 2> $O/${W}_l$V.err
    python -c "import json;d=json.loads(open('$O/${W}_l$V.json').read().splitlines()[-1]);print('$W lpt=$V', round(d['ms_per_step'],4))"
  done
done
