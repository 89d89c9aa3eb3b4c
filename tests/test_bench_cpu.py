"""bench.py host logic on CPU: the roofline names the launch that runs, and
the committed PMC traffic is quoted only for its own kernel and workload."""
import types

import bench
import psengine as PE


def _st(mode, launches, windows):
    return types.SimpleNamespace(expand_mode=mode, expand_launches=launches, windows=windows)


def test_hot_kernel_labels():
    # the kernel that ran the window's rounds, by ps_stats.expand_mode
    assert bench.hot_kernel(_st(PE.MODE_FLOOD, 1, 1)) == "k_flood"
    assert bench.hot_kernel(_st(PE.MODE_LEVEL_PULL, 12, 1)) == "k_pull"
    assert bench.hot_kernel(_st(PE.MODE_COMPACT, 1, 1)) == "k_expand"


def test_pmc_traffic_matches_kernel_and_workload():
    """The committed PMC traffic is quoted only for the kernel and workload it
    was measured on."""
    import json
    with open(bench.TRAFFIC_FILE) as fh:
        d = json.load(fh)
    t, src = bench.pmc_traffic(d["kernel"], d["workload"])
    assert t is not None and t > 0 and "FETCH_SIZE" in src
    assert bench.pmc_traffic(d["kernel"] + "_other", d["workload"])[0] is None
    assert bench.pmc_traffic(d["kernel"], d["workload"] + "_other")[0] is None
