"""bench.py host logic on CPU: the roofline names the launch that runs, and
the committed PMC traffic is quoted only for its own kernel and workload."""
import types

import bench
import psengine as PE


def _st(mode, launches, windows, rounds=20, flood_rounds=0, ms=None, by=None):
    ms = ms or [0.0] + [0.1] * rounds
    by = by or [0] + [1000] * rounds
    return types.SimpleNamespace(expand_mode=mode, expand_launches=launches, windows=windows, rounds=rounds,
                                 flood_rounds=flood_rounds, expand_ms=sum(ms), expand_bytes=sum(by),
                                 expand_ms_per_round=ms, expand_bytes_per_round=by)


def test_hot_kernel_labels():
    # the kernel that ran the window's rounds, by ps_stats.expand_mode
    assert bench.hot_kernel(_st(PE.MODE_FLOOD, 1, 1, flood_rounds=20)) == "k_flood"
    assert bench.hot_kernel(_st(PE.MODE_LEVEL_PULL, 12, 1)) == "k_pull"
    assert bench.hot_kernel(_st(PE.MODE_COMPACT, 1, 1)) == "k_expand"


def test_hybrid_window_split():
    """k_flood for rounds 1..12 (its time in round 1's slot), k_pull after:
    bytes, time and launches split per kernel; the roofline names the kernel
    with the most device time and lists both."""
    ms = [0.0, 0.05] + [0.0] * 11 + [0.2] * 8
    by = [0] + [10] * 12 + [1_000_000] * 8
    st = _st(PE.MODE_FLOOD, 9, 1, rounds=20, flood_rounds=12, ms=ms, by=by)
    sp = bench.kernel_split(st)
    assert sp["k_flood"] == (120, 0.05, 1)
    assert sp["k_pull"][0] == 8_000_000 and abs(sp["k_pull"][1] - 1.6) < 1e-9 and sp["k_pull"][2] == 8
    assert bench.hot_kernel(st) == "k_pull"
    roof = bench.roofline_of({k: list(v) for k, v in sp.items()})
    assert roof["kernel"] == "k_pull" and set(roof["kernels"]) == {"k_flood", "k_pull"}
    assert abs(roof["avg_launch_us"] - 200.0) < 1e-6
    # several windows: per-round slots mix windows, no split
    assert set(bench.kernel_split(_st(PE.MODE_FLOOD, 9, 2, flood_rounds=12, ms=ms, by=by))) == {"k_flood"}


def test_round_kernel_split():
    """ps_stats.round_kernel: k_flood (rounds 1..4, timed into round 1), two
    k_pull_pair launches (rounds 5+6, 8+9, each timed into its first round),
    k_pull for rounds 7 and 10: per-kernel bytes, time and launch counts."""
    ms = [0.0, 0.05, 0, 0, 0, 0.3, 0.0, 0.2, 0.5, 0.0, 0.1]
    by = [0, 1, 1, 1, 1, 100, 200, 300, 400, 500, 600]
    st = _st(PE.MODE_FLOOD, 5, 1, rounds=10, flood_rounds=4, ms=ms, by=by)
    st.round_kernel = [0] + [PE.K_FLOOD] * 4 + [PE.K_PAIR, PE.K_PAIR2, PE.K_PULL, PE.K_PAIR, PE.K_PAIR2,
                                                 PE.K_PULL] + [0] * (PE.MAX_ROUNDS - 11)
    sp = bench.kernel_split(st)
    assert sp["k_flood"] == (4, 0.05, 1)
    assert sp["k_pull_pair"][0] == 100 + 200 + 400 + 500 and abs(sp["k_pull_pair"][1] - 0.8) < 1e-9
    assert sp["k_pull_pair"][2] == 2
    assert sp["k_pull"][0] == 900 and abs(sp["k_pull"][1] - 0.3) < 1e-9 and sp["k_pull"][2] == 2
    assert bench.hot_kernel(st) == "k_pull_pair"


def test_pmc_traffic_matches_kernel_and_workload():
    """The committed PMC traffic is quoted only for the kernel and workload it
    was measured on."""
    import json
    with open(bench.TRAFFIC_FILE) as fh:
        d = json.load(fh)
    assert d["entries"]
    for x in d["entries"]:
        t, src = bench.pmc_traffic(x["kernel"], x["workload"])
        assert t is not None and t > 0 and "FETCH_SIZE" in src
        assert bench.pmc_traffic(x["kernel"] + "_other", x["workload"])[0] is None
        assert bench.pmc_traffic(x["kernel"], x["workload"] + "_other")[0] is None
