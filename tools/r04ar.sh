#!/bin/bash
# Shallow windows (under overlap_min_rounds) end signalled instead of
# overlapping their init: parity (async, flood, fullsize, pipeline fuzz), then
# cfg4 A/B against PSAMD_OVERLAP_SHALLOW=1 and a cfg3 line.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ar
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_flood.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u tools/fuzz_gpu.py --cases 800 --seed 405 --kinds pipeline modes > $O/fuzz.log 2>&1
tail -n 1 $O/fuzz.log
for V in 0 1 0 1 0 1; do
  PSAMD_AB=1 PSAMD_OVERLAP_SHALLOW=$V timeout -k 10 200 python -u bench.py --workload cfg4 --steps 300 --warmup 5 --sustain 0 --no-cpu --no-general > $O/cfg4_s$V.json 2> $O/cfg4_s$V.err
  python -c "import json;d=json.loads(open('$O/cfg4_s$V.json').read().splitlines()[-1]);print('cfg4 overlap_shallow=$V', round(d['ms_per_step'],4), 'overlapped', d['plan']['overlapped_windows_timed'])"
done
timeout -k 10 200 python -u bench.py --steps 300 --warmup 5 --sustain 0 --no-cpu --no-general > $O/cfg3.json 2> $O/cfg3.err
python -c "import json;d=json.loads(open('$O/cfg3.json').read().splitlines()[-1]);print('cfg3', round(d['ms_per_step'],4), 'overlapped', d['plan']['overlapped_windows_timed'])"
