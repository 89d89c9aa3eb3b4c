# Process-per-rank runs on one GPU (the IPC transport, ps_dist_init_ipc):
# tests/test_gpu_ipc.py, then bench.py --gpus 2 / 4 on cfg4 and cfg3 (ranks
# share the GPU; each line reports shared_gpu.ratio_vs_one_rank).
#   TAG=ipcb [MODES="inplace zc"] bash tools/gpu_ipc_bench.sh
set -o pipefail
O=gpurun_out/${TAG:-ipcb}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ipc.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for M in ${MODES:-inplace}; do for W in cfg4 cfg3; do for N in 2 4; do
  timeout -k 10 300 python -u bench.py --gpus $N --workload $W --no-cpu --ipc-mode $M > $O/bench_${W}_g${N}_$M.json 2> $O/bench_${W}_g${N}_$M.err || { tail -30 $O/bench_${W}_g${N}_$M.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('shared_gpu',{}).get('ratio_vs_one_rank'))" $O/bench_${W}_g${N}_$M.json
done; done; done
