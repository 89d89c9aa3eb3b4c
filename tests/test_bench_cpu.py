"""bench.py host logic on CPU: the roofline names the launch that runs, and
the committed PMC traffic is quoted only for its own kernel and workload."""
import types

import bench
import psengine as PE


def _st(mode, launches, windows):
    return types.SimpleNamespace(expand_mode=mode, expand_launches=launches, windows=windows)


def test_hot_kernel_labels():
    # one k_pull_top launch per window (every level of a single-GPU window)
    assert bench.hot_kernel(_st(PE.MODE_LEVEL_PULL, 1, 1)) == "k_pull_top"
    assert bench.hot_kernel(_st(PE.MODE_LEVEL_PULL, 3, 3)) == "k_pull_top"
    # per-level launches (multi-rank below the split level, deep windows)
    assert bench.hot_kernel(_st(PE.MODE_LEVEL_PULL, 12, 1)) == "k_pull"
    assert bench.hot_kernel(_st(PE.MODE_COMPACT, 1, 1)) == "k_expand"


def test_pmc_traffic_matches_kernel_and_workload():
    t, src = bench.pmc_traffic("k_pull_top", "cfg3")
    assert t is not None and t > 4.0e9 and "FETCH_SIZE" in src
    assert bench.pmc_traffic("k_pull", "cfg3")[0] is None
    assert bench.pmc_traffic("k_pull_top", "cfg4")[0] is None
