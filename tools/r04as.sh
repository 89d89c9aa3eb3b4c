#!/bin/bash
# k_pull at 4 / 5 / 6 waves per SIMD by register allocation (PSAMD_PULL_SIMD)
# vs the defaults (one rank: 5 blocks per CU by an LDS pad; N ranks: full
# residency): 4-rank peer-hash loopback and cfg4 with k_pull rounds only.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04as
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for V in 0 4 5 6 0 4; do
  PSAMD_AB=1 PSAMD_PULL_SIMD=$V timeout -k 10 150 python -u tools/loopback_bench.py --world 4 --scale 1.0 --steps 6 --workload cfg4 --partition peer > $O/lb_s$V.log 2>&1
  echo "loopback pull_simd=$V $(tail -n 1 $O/lb_s$V.log)"
done
for V in 0 4 5 6; do
  PSAMD_AB=1 PSAMD_CHAIN=1 PSAMD_FLOOD=0 PSAMD_PULL_SIMD=$V timeout -k 10 150 python -u bench.py --workload cfg4 --steps 100 --warmup 3 --sustain 0 --no-cpu --no-general > $O/cfg4_s$V.json 2> $O/cfg4_s$V.err
  python -c "import json;d=json.loads(open('$O/cfg4_s$V.json').read().splitlines()[-1]);r=d['roofline'];print('cfg4 k_pull only, pull_simd=$V', round(d['ms_per_step'],4), {k:(round(v['achieved']),v['launches']) for k,v in r['kernels'].items()})"
done
