#!/bin/bash
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fuzz_r03
mkdir -p $O
timeout -k 10 900 python -u tools/fuzz_gpu.py --cases 4000 --seed 37 > $O/fuzz_4000_seed37.log 2>&1
tail -n 3 $O/fuzz_4000_seed37.log
timeout -k 10 240 python -u tools/fuzz_gpu.py --cases 150 --seed 53 --kinds dist --max-world 6 > $O/fuzz_dist_seed53.log 2>&1
tail -n 3 $O/fuzz_dist_seed53.log
