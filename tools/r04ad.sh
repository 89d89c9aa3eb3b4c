#!/bin/bash
# Held-back reduce fused into the next window's init (k_window_turn):
# async/flood/drain parity, then cfg2 and cfg3 A/B against PSAMD_FUSE_REDUCE=0.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ad
mkdir -p $O
echo "[ad] tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_flood.py tests/test_gpu_drain.py tests/test_gpu_chain.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 2 $O/pytest.log
for W in cfg2 cfg3; do
  for F in 1 0 1 0; do
    echo "[ad] $W fuse=$F $(date +%T)"
    PSAMD_FUSE_REDUCE=$F timeout -k 10 200 python -u tools/host_split.py --workload $W --steps $([ $W = cfg2 ] && echo 400 || echo 150) --reps 2 >> $O/host_split_$W.log 2>&1
    tail -n 1 $O/host_split_$W.log
  done
done
echo "[ad] done $(date +%T)"
