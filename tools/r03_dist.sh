#!/bin/bash
# The N>1 bench driver on this pool's one-GPU boxes: one rank through the
# torch.distributed path, and two ranks sharing the GPU on the message-sharded
# leg (gloo bootstrap, no RCCL between them).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03dist
mkdir -p $O
echo "[dist] force-dist $(date +%T)"
timeout -k 10 300 python -u bench.py --force-dist --steps 5 --warmup 2 --no-cpu > $O/force_dist.json 2> $O/force_dist.err
cat $O/force_dist.json | head -c 600; echo
echo "[dist] message-only x2 $(date +%T)"
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29557 \
  bench.py --gpus 2 --message-only --steps 3 --warmup 1 > $O/message_only2.json 2> $O/message_only2.err
cat $O/message_only2.json | head -c 600; echo
echo "[dist] done $(date +%T)"
