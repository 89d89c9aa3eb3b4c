"""Shared pytest setup: import paths, the `gpu` marker, helpers."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("", "go-libp2p-pubsub_amd", "oracle"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP hot path)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def cfg4_full():
    """cfg4's full-size tree, dead mask and oracle reach (fullsize_common.Cfg4Tree),
    built once per session for the full-size and process-per-rank tests."""
    from fullsize_common import Cfg4Tree

    return Cfg4Tree()


@pytest.fixture(scope="session")
def cfg3_cut():
    """BASELINE cfg3's trees (the restated joins), the cut-tree dead mask and
    or_disseminate's per-topic expectations (fullsize_common.Expect), built
    once per session for the paced and process-per-rank tests."""
    import psengine as PE
    from fullsize_common import Expect, cfg3_dead_mask
    from psengine import workloads as WL

    wl = WL.cfg3()
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as eng:
        WL.build_engine_topics(eng, wl)
        parents = [eng.parents(t) for t in range(len(wl.topics))]
    live = cfg3_dead_mask(wl, parents)
    return wl, parents, live, Expect(wl, parents, live)
