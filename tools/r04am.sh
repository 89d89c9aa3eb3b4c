#!/bin/bash
# Cross-window overlap (events, prefix stream) vs signalled windows (overlap
# off: one stream, pinned flag, reduce held back into the next init), bench.py
# lines alternating on one box: cfg3, cfg4, cfg2.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04am
mkdir -p $O
for W in cfg3 cfg4; do
  for V in 1 0 1 0 1 0; do
    PSAMD_AB=1 PSAMD_OVERLAP=$V timeout -k 10 200 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 --no-cpu --no-general > $O/${W}_ov$V.json 2> $O/${W}_ov$V.err
    python -c "import json;d=json.loads(open('$O/${W}_ov$V.json').read().splitlines()[-1]);print('$W overlap=$V', round(d['ms_per_step'],4), 'overlapped', d['plan']['overlapped_windows_timed'])"
  done
done
for V in 1 0; do
  PSAMD_AB=1 PSAMD_OVERLAP=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/driver_ov$V.json 2> $O/driver_ov$V.err
  python -c "import json;d=json.loads(open('$O/driver_ov$V.json').read().splitlines()[-1]);print('driver cmd overlap=$V', round(d['ms_per_step'],4), d['sustained']['ms_per_step'])"
done
