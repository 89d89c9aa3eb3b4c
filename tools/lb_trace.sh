# kernel trace of the 4-rank cfg4 loopback (peer hash)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lbt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/lbt/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/loopback_bench.py --world 4 --workload cfg4 --scale 1.0 --partition peer --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/lbt/cfg4_peer4_traced.log 2>&1
