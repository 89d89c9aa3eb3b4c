#!/bin/bash
# k_pull_chain stages the topic root's row for level 0 (root_rows): chain /
# fullsize / async / flood / dist parity, then cfg3 / cfg4 / cfg2 A/B against
# PSAMD_CHAIN_ROOT_ROW=0.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ak
mkdir -p $O
echo "[ak] tests $(date +%T)"
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_fullsize.py tests/test_gpu_async.py tests/test_gpu_flood.py tests/test_gpu_pair.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
for R in 1 0 1 0; do
  PSAMD_AB=1 PSAMD_CHAIN_ROOT_ROW=$R timeout -k 10 200 python -u tools/host_split.py --workload cfg3 --steps 200 --reps 1 >> $O/hs_cfg3.log 2>&1
  echo "root_row=$R $(tail -n 1 $O/hs_cfg3.log)"
done
for R in 1 0 1 0; do
  PSAMD_AB=1 PSAMD_CHAIN_ROOT_ROW=$R timeout -k 10 200 python -u tools/host_split.py --workload cfg4 --steps 100 --reps 1 >> $O/hs_cfg4.log 2>&1
  echo "root_row=$R $(tail -n 1 $O/hs_cfg4.log)"
done
echo "[ak] done $(date +%T)"
