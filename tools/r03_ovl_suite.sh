set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ovl2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/fuzz_gpu.py --cases 1000 --seed 81 > $O/fuzz_seed81.log 2>&1
tail -n 1 $O/fuzz_seed81.log
