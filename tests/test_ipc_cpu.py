"""CPU: the host side of the process-per-rank path (no GPU needed): the IPC
group id (ps_dist_ipc_id), argument checks of ps_dist_init_ipc / ps_dist_init
(a null engine returns PS_E_INVAL instead of crashing),
ps_device_count, the bench driver's transport choice, and the compaction
kernel's register budget with the flat path inlined (6 waves per SIMD)."""
import ctypes

import pytest

import psengine as PE
from psengine import dist as D


@pytest.fixture(scope="module")
def lib():
    return PE.load()


def test_ipc_group_ids_are_fresh_shm_names():
    ids = {PE.ipc_group_id() for _ in range(8)}
    assert len(ids) == 8
    for g in ids:
        assert len(g) == 128
        name = g.split(b"\0", 1)[0].decode()
        assert name.startswith("/psamd-ipc-") and "/" not in name[1:] and len(name) < 64


def test_dist_init_null_arguments(lib):
    dc = PE.DistConfig(0, 2, PE.PART_PEER, 0, PE.DIST_F_INPLACE, 0)
    gid = (ctypes.c_uint8 * 128).from_buffer_copy(PE.ipc_group_id())
    assert lib.ps_dist_init_ipc(None, ctypes.byref(dc), gid) == -1
    assert lib.ps_dist_init(None, ctypes.byref(dc), gid) == -1  # (in-place flag, null engine)
    assert lib.ps_dist_init_loopback(None, ctypes.byref(dc), None) == -1


def test_device_count_without_gpu():
    import os

    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU driver present")
    assert PE.device_count() == 0


@pytest.mark.parametrize("req,world,ndev,want", [
    ("auto", 8, 8, "rccl"), ("auto", 2, 1, "ipc"), ("auto", 4, 1, "ipc"), ("ipc", 8, 8, "ipc"),
    ("rccl", 2, 2, "rccl"), ("auto", 1, 0, "rccl")])
def test_transport_choice(req, world, ndev, want):
    assert D.pick_transport(req, world, ndev) == want


def test_rccl_refused_on_shared_gpus():
    with pytest.raises(SystemExit):
        D.pick_transport("rccl", 2, 1)


def test_expand_residency(tmp_path):
    """k_expand<false, false> (the staged instance with the flat path) stays
    within 80 VGPRs: 6 waves per SIMD (amdgpu_waves_per_eu(6))."""
    from test_abi import _kernel_regs

    regs = _kernel_regs(tmp_path)
    staged = {k: v for k, v in regs.items() if "k_expandILb0ELb0E" in k}
    assert staged, sorted(regs)
    for k, (vg, ag) in staged.items():
        assert vg + ag <= 80, (k, vg, ag)
