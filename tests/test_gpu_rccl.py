"""Two ranks over real RCCL (ps_dist_init: grouped ncclSend/ncclRecv), one
process per GPU as torch.distributed.run launches them (tools/rccl_pair.py):
the union of the ranks' hops, their summed deliveries and seen digests equal
a single engine's, under both partitions, level and compaction mode.

RCCL refuses two ranks on one device (`ncclCommInitRank: invalid usage`,
measured on the one-GPU box, profiles/r02/README.md), so this needs >= 2
visible GPUs; the loopback transport covers the exchange protocol on one GPU
(tests/test_gpu_dist.py)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("staggered", [False, True])
@pytest.mark.parametrize("partition", ["peer", "subtree"])
def test_two_rank_rccl_matches_single_engine(partition, staggered):
    import torch

    ndev = torch.cuda.device_count()  # (counting devices does not initialise the GPU)
    if ndev < 2:
        pytest.skip("one GPU visible: RCCL needs a device per rank")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(REPO, "tools", "rccl_pair.py"),
           "--partition", partition] + (["--staggered"] if staggered else [])
    env = dict(os.environ, PSAMD_DEVICES=str(ndev))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "RCCL_PAIR OK" in r.stdout
