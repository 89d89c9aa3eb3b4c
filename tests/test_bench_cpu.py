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


def _args(**kw):
    base = dict(gpus=1, workload="cfg3")
    base.update(kw)
    return types.SimpleNamespace(**base)


def test_launch_plan_one_gpu_runs_here():
    assert bench.launch_plan(_args(), {}, []) is None
    assert bench.launch_plan(_args(gpus=4), {"WORLD_SIZE": "4"}, []) is None


def test_launch_plan_starts_n_ranks_without_a_launcher():
    """--gpus N without WORLD_SIZE: a child torch.distributed.run with N
    ranks on 127.0.0.1 and the same arguments."""
    argv = ["--gpus", "8", "--steps", "5", "--workload", "cfg4"]
    cmd = bench.launch_plan(_args(gpus=8, workload="cfg4"), {}, argv, port=29777)
    assert isinstance(cmd, list)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29777" in cmd
    i = cmd.index(bench.os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == argv


def test_launch_plan_refuses_mismatch_and_cfg5():
    assert isinstance(bench.launch_plan(_args(gpus=2), {"WORLD_SIZE": "4"}, []), str)
    assert isinstance(bench.launch_plan(_args(gpus=1), {"WORLD_SIZE": "2"}, []), str)
    assert isinstance(bench.launch_plan(_args(gpus=2, workload="cfg5"), {}, []), str)
    assert isinstance(bench.launch_plan(_args(gpus=0), {}, []), str)


def test_bench_mismatch_exits_nonzero():
    """A torchrun rank whose WORLD_SIZE differs from --gpus exits non-zero
    and prints no JSON line (checked before anything touches the GPU)."""
    import subprocess
    import sys
    env = dict(bench.os.environ, WORLD_SIZE="2", RANK="0")
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "4", "--no-cpu"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and p.stdout.strip() == ""
    assert "must agree" in p.stderr


def test_dist_bench_main_asserts_world():
    from psengine import dist
    import pytest
    env = dict(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    old = {k: bench.os.environ.get(k) for k in env}
    bench.os.environ.update(env)
    try:
        with pytest.raises(SystemExit):
            dist.bench_main(_args(gpus=4), bench.DESCR, bench.METRIC)
    finally:
        for k, v in old.items():
            if v is None:
                bench.os.environ.pop(k, None)
            else:
                bench.os.environ[k] = v
