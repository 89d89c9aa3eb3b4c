#!/bin/bash
export PSAMD_AB=1  # plan options from the environment (A/B tools only)
# Flood split at 4 MB: GPU suite, driver bench command, cfg2; cfg5 kernel trace.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03c}
mkdir -p $O
echo "[r03c] tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -n 1 $O/pytest.log
echo "[r03c] driver command $(date +%T)"
timeout -k 10 400 python -u bench.py > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 200 --warmup 5 --sustain 0 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
for L in 5 6; do
  PSAMD_CHAIN=$L timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 0 > $O/cfg3_chain$L.json 2> $O/cfg3_chain$L.err
done
timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-cpu --no-general --sustain 0 > $O/cfg3_chain4.json 2> $O/cfg3_chain4.err
echo "[r03c] cfg5 trace $(date +%T)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$O/trace_cfg5" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload cfg5 --steps 10 --warmup 3 --no-cpu > "$GRAFT_REPO_ROOT/$O/bench_cfg5_traced.json" 2> "$GRAFT_REPO_ROOT/$O/bench_cfg5_traced.err"
echo "[r03c] done $(date +%T)"
