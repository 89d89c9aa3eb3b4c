"""Builds libpsengine.so in-tree with hipcc for gfx950 (no JIT cache, no pip)."""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # go-libp2p-pubsub_amd/
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libpsengine.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["kernels.hip", "pull.hip", "flood.hip", "gbuild.hip", "graph.cpp", "plan.cpp", "run.cpp", "api.cpp", "tree.cpp",
           "dist.cpp", "codec.cpp", "pubsub.cpp"]
HEADERS = ["kernels.hpp", "devutil.hpp", "gbuild.hpp", "tree.hpp", "dist.hpp", "engine.hpp"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(REPO, "include", "psengine.h"))
    deps.append(os.path.join(REPO, "include", "pubsub.hpp"))
    deps.append(os.path.join(REPO, "include", "psengine_plan.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    """Each source to an object in parallel (the kernels are launched from
    their own translation unit, so no relocatable device code), then one
    link into lib/libpsengine.so."""
    if not force and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(LIBDIR, "obj")
    os.makedirs(objdir, exist_ok=True)
    flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall",
             "-I" + os.path.join(REPO, "include"), "-I" + CSRC]

    def compile_one(f):
        obj = os.path.join(objdir, f + ".o")
        cmd = [HIPCC] + flags + ["-c", os.path.join(CSRC, f), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 4), 16))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared"] + objs
    cmd += ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    # hipcc leaves per-object offload bundles next to the output: not needed
    for f in os.listdir(LIBDIR):
        if f.startswith("libpsengine.so.") and not f.endswith(".tmp"):
            os.remove(os.path.join(LIBDIR, f))
    return LIB


CPP_TESTS = os.path.join(REPO, "tests", "cpp")
CPP_TEST_BIN = os.path.join(CPP_TESTS, "bin", "pubsub_test")


def build_cpp_tests(force: bool = False, verbose: bool = False) -> str:
    """tests/cpp/pubsub_test.cpp (the reference's tests against the C++ API
    mirror, include/pubsub.hpp) -> tests/cpp/bin/pubsub_test, linked to the
    in-tree libpsengine.so.  Host C++ only (g++)."""
    src = os.path.join(CPP_TESTS, "pubsub_test.cpp")
    hdr = os.path.join(REPO, "include", "pubsub.hpp")
    if (not force and os.path.exists(CPP_TEST_BIN) and
            os.path.getmtime(CPP_TEST_BIN) >= max(os.path.getmtime(src), os.path.getmtime(hdr))):
        return CPP_TEST_BIN
    os.makedirs(os.path.dirname(CPP_TEST_BIN), exist_ok=True)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(REPO, "include"),
           src, "-L" + LIBDIR, "-lpsengine", "-Wl,-rpath," + LIBDIR, "-o", CPP_TEST_BIN + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(CPP_TEST_BIN + ".tmp", CPP_TEST_BIN)
    return CPP_TEST_BIN
