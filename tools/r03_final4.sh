#!/bin/bash
# The driver's bench command on the final tree (traffic from the refreshed PMC entry), cfg2/cfg4 lines,
# more pipelined-overlap fuzz cases.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03i}
mkdir -p $O
echo "[final4] smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -n 2 $O/smoke.log
echo "[final4] driver command $(date +%T)"
timeout -k 10 400 python -u bench.py > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
for W in cfg4 cfg2; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 300 --warmup 5 --sustain 0 > $O/bench_$W.json 2> $O/bench_$W.err
done
timeout -k 10 400 python -u tools/fuzz_gpu.py --cases 2100 --seed 92 --kinds pipeline > $O/fuzz_pipeline_seed92.log 2>&1
tail -n 1 $O/fuzz_pipeline_seed92.log
echo "[final4] done $(date +%T)"
