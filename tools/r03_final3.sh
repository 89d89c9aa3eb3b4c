#!/bin/bash
# Tail chains: pipelined-overlap fuzz, full GPU suite, traces and PMC passes of the final plan.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03h}
O=gpurun_out/$TAG
mkdir -p $O
echo "[final3] fuzz $(date +%T)"
timeout -k 10 400 python -u tools/fuzz_gpu.py --cases 700 --seed 91 --kinds pipeline > $O/fuzz_pipeline_seed91.log 2>&1
tail -n 1 $O/fuzz_pipeline_seed91.log
echo "[final3] suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 1 $O/pytest_gpu.log
TESTS=0 PMC=1 bash tools/gpu_check.sh $TAG
echo "[final3] done $(date +%T)"
