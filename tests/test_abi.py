"""CPU checks of the drop-in boundary: libpsengine.so builds for gfx950,
loads, and exports every entry point include/psengine.h declares; the ctypes
structs match the C layout.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import psengine as PE

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "psengine.h")


PLAN_HEADER = os.path.join(REPO, "include", "psengine_plan.h")


def declared(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ps_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from psengine import _build

    _build.build()
    return PE.load()


def test_header_symbols_exported(lib):
    names = declared()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", PE.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (ps_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    bound = {p[0] for p in PE.PROTOTYPES}
    assert set(names) == bound, set(names) ^ bound


def test_plan_probe_symbols_exported(lib):
    """The host-only planner probe (include/psengine_plan.h, tests only) is
    exported and bound by psengine.plan."""
    from psengine import plan as PL

    names = declared(PLAN_HEADER)
    assert names == sorted(p[0] for p in PL.PROTOTYPES)
    out = subprocess.run(["nm", "-D", "--defined-only", PE.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (ps_\w+)", out))
    assert not [n for n in names if n not in exported]
    PL.lib()


def test_code_object_is_gfx950(lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading",
                          PE.lib_path()], capture_output=True, text=True)
    text = out.stdout + out.stderr
    assert "gfx950" in text


def test_struct_layouts(lib):
    assert ctypes.sizeof(PE.Config) == 40
    assert ctypes.sizeof(PE.Stats) == 9 * 8 + 3 * 8 + 8 + PE.MAX_ROUNDS * 25 + 16 + 16 + 8
    src = open(HEADER).read()
    assert f"#define PS_MAX_ROUNDS {PE.MAX_ROUNDS}" in src
    for name, val in [("PS_F_RECORD_HOPS", PE.F_RECORD_HOPS), ("PS_F_TIME_KERNELS", PE.F_TIME_KERNELS)]:
        assert re.search(rf"#define {name} 0x{val:x}u", src)
    for name in ("NONE", "FLOOD", "PULL", "PAIR", "PAIR2", "EXPAND", "CHAIN", "CHAIN2"):  # ps_stats.round_kernel
        assert re.search(rf"#define PS_K_{name} {getattr(PE, 'K_' + name)}u", src)


def test_version_and_error_paths(lib):
    assert b"gfx950" in lib.ps_version()
    assert lib.ps_create(None, None) == -1  # PS_E_INVAL
    assert lib.ps_last_error(None) == b"null engine"
    cfg = PE.Config(0, 1, 2, 5, 0, 0, 0, 0, 1)
    h = ctypes.c_void_p()
    assert lib.ps_create(ctypes.byref(cfg), ctypes.byref(h)) == -1  # n_peers == 0


def test_abi_check(lib):
    """ps_abi_check accepts the sizes this binding was built with and refuses
    a caller compiled against another layout (ps_stats grew 32 B,
    ps_dist_config 8 B, without a version bump)."""
    assert lib.ps_abi_version() == PE.ABI_VERSION == 5
    sizes = (ctypes.sizeof(PE.Config), ctypes.sizeof(PE.Stats), ctypes.sizeof(PE.PlanOpts),
             ctypes.sizeof(PE.DistConfig))
    assert lib.ps_abi_check(PE.ABI_VERSION, *sizes) == 0
    assert lib.ps_abi_check(3, *sizes) == -1
    assert b"ABI version 3" in lib.ps_last_error(None)
    old = (sizes[0], sizes[1] - 40, sizes[2], sizes[3] - 8)  # the round-3 layouts
    assert lib.ps_abi_check(PE.ABI_VERSION, *old) == -1
    assert b"struct sizes" in lib.ps_last_error(None)
    assert b"abi 5" in lib.ps_version()


def _kernel_regs(tmp_path):
    """{kernel symbol: (vgpr_count, agpr_count)} from the gfx950 code
    objects' AMDGPU metadata notes (llvm-objdump --offloading extracts them
    next to its input, so it runs on a copy)."""
    import shutil

    so = tmp_path / "libpsengine.so"
    shutil.copy(PE.lib_path(), so)
    llvm = "/opt/rocm/lib/llvm/bin"
    subprocess.run([f"{llvm}/llvm-objdump", "--offloading", str(so)], capture_output=True, check=True,
                   cwd=tmp_path)
    regs = {}
    for co in sorted(tmp_path.glob("*gfx950*")):
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", str(co)], capture_output=True, text=True,
                               check=True).stdout
        for blk in notes.split("  - .agpr_count:")[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk).group(1)
            vg = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
            regs[name] = (vg, int(blk.split("\n")[0].strip()))
    return regs


def test_chain_residency_vgprs(lib, tmp_path):
    """The production k_pull_chain variants (kSimdWaves = 3) must allocate
    registers for exactly 3 waves per SIMD (512 VGPRs per lane, allocated
    in granules of 8, AGPRs from the same file): the round-4 residency gain
    (0.951 -> 0.902 ms/step on cfg3) rests on a clobbered
    v140, which a compiler change could silently undo.  The uncapped
    variants must fit more than 3, or the cap would be doing nothing."""
    regs = _kernel_regs(tmp_path)

    def waves(v):
        return 512 // ((v[0] + v[1] + 7) // 8 * 8)

    capped = {k: v for k, v in regs.items() if "k_pull_chain" in k and k.endswith("Lj3EEEvNS_8PullArgsEPKNS_10ChainChunkEjj")}
    free = {k: v for k, v in regs.items() if "k_pull_chain" in k and "Lj0EEEv" in k}
    assert len(capped) >= 3, sorted(regs)
    for k, v in capped.items():
        assert waves(v) == 3, (k, v)
    assert free
    for k, v in free.items():
        assert waves(v) > 3, (k, v)


def test_no_cpu_fallback_without_gpu(lib):
    """On a machine without a GPU the engine refuses to start (PS_E_DEVICE):
    there is no silent CPU path."""
    if os.path.exists("/dev/kfd"):
        pytest.skip("GPU driver present")
    with pytest.raises(PE.EngineError) as ei:
        PE.Engine(8)
    assert ei.value.code == -6


def test_struct_offsets_match_c(tmp_path):
    """Every field of the ctypes mirrors sits where the C compiler puts it
    (gcc on include/psengine.h)."""
    structs = {"ps_config": PE.Config, "ps_stats": PE.Stats, "ps_dist_config": PE.DistConfig,
               "ps_plan_opts": PE.PlanOpts, "ps_message": PE.MessageC, "ps_message_buf": PE.MessageBuf}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "psengine.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            cf = "type" if f == "type" else f
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {cf}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, cls in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_header_constants_match_python():
    """The PS_* values the Python binding mirrors equal the header's (the
    in-place exchange flag and path of round 5 included)."""
    import re
    hdr = open(os.path.join(REPO, "include", "psengine.h")).read()
    vals = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define (PS_\w+) (0x[0-9a-fA-F]+|\d+)u?", hdr)}
    pairs = {"PS_DIST_F_COPY": PE.DIST_F_COPY, "PS_DIST_F_INPLACE": PE.DIST_F_INPLACE,
             "PS_XCHG_NONE": PE.XCHG_NONE, "PS_XCHG_ZERO_COPY": PE.XCHG_ZERO_COPY, "PS_XCHG_COPY": PE.XCHG_COPY,
             "PS_XCHG_IN_PLACE": PE.XCHG_IN_PLACE, "PS_K_CHAIN": PE.K_CHAIN, "PS_K_FLOOD": PE.K_FLOOD}
    for name, py in pairs.items():
        assert vals[name] == py, name
