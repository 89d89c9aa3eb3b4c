#!/bin/bash
# One rocprofv3 PMC pass with SQ stall counters over a short cfg3 bench.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_${1:-sq}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR \
  -T -f csv -d "$OUT/sq1" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu > "$OUT/b1.json" 2> "$OUT/b1.err"
echo "sq1 rc=$?"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
  -T -f csv -d "$OUT/sq2" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu > "$OUT/b2.json" 2> "$OUT/b2.err"
echo "sq2 rc=$?"
