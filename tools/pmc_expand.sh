# SQ instruction counters of k_expand on the compaction leg (tools/compact_probe.py),
# one PMC pass per variant of PSAMD_NARROW (PSAMD_AB=1).
#   TAG=sqx bash tools/pmc_expand.sh
# COUNTERS overrides the pass's counter list (at most 8 SQ_ counters).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
O=$ROOT/gpurun_out/${TAG:-sqx}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp PSAMD_AB=1
for V in ${VARIANTS:-1 0}; do
  PSAMD_NARROW=$V timeout -s KILL 180 rocprofv3 --pmc ${COUNTERS:-SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY} -T -f csv -d $O/sq_$V -o run -- python3 $ROOT/tools/compact_probe.py --steps 2 --timed 0 > $O/sq_$V.json 2> $O/sq_$V.err
  echo "variant $V rc=$?"
done
