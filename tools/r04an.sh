#!/bin/bash
# Device-scope end events for windows whose reduce stored the counters into
# pinned memory itself: async / dist parity, then cfg3 / cfg4 A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04an
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_dist.py tests/test_gpu_drain.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for W in cfg3 cfg4; do
  for V in 1 0 1 0 1 0; do
    PSAMD_AB=1 PSAMD_END_EVENT_DEVICE=$V timeout -k 10 200 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 --no-cpu --no-general > $O/${W}_ed$V.json 2> $O/${W}_ed$V.err
    python -c "import json;d=json.loads(open('$O/${W}_ed$V.json').read().splitlines()[-1]);print('$W end_event_device=$V', round(d['ms_per_step'],4))"
  done
done
