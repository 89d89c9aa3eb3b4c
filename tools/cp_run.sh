# compaction-path A/B on one box: library builds of tools/build_variant.sh
#   VARIANTS="A c16" PMCV="c16" TAG=cp2 bash tools/cp_run.sh
set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cp}; mkdir -p $O
L=go-libp2p-pubsub_amd/lib
lib() { if [ $1 = A ]; then echo $L/libpsengine.so; else echo $L/libpsengine_$1.so; fi; }
for V in $VARIANTS $VARIANTS; do
  PSENGINE_LIB_AB=$(lib $V) timeout -k 10 200 python -u tools/compact_probe.py --steps 6 --timed 2 ${PROBE_ARGS:-} > $O/t_$V.json 2>> $O/t.err
  echo "$V $(cut -c1-150 $O/t_$V.json)"
done
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for V in ${PMCV:-}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    PSENGINE_LIB_AB=$(lib $V) timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/pmc_${V}_$C -o run -- python3 tools/compact_probe.py --steps 1 --timed 0 > $O/pmc_${V}_$C.log 2>&1
    echo "pmc $V $C done"
  done
done
