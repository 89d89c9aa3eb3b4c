# SQ counters of the compaction path (tools/compact_probe.py), two passes
set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cpsq}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR \
  -f csv -d $O/sq1 -o run -- python3 tools/compact_probe.py --steps 1 --timed 0 > $O/sq1.log 2>&1
echo sq1 done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
  -f csv -d $O/sq2 -o run -- python3 tools/compact_probe.py --steps 1 --timed 0 > $O/sq2.log 2>&1
echo sq2 done
