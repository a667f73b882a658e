"""bench.py's launcher and bookkeeping on CPU (no GPU): `--gpus N` starts N ranks through
torch.distributed.run without the parent loading the engine or any GPU runtime; a world size that
contradicts --gpus is refused; the profile cross-check only trusts a profile of the same build."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env


def test_launcher_starts_ranks_without_loading_the_engine():
    code = (
        "import sys, json; sys.path.insert(0, %r); import bench\n"
        "argv = ['--gpus', '4', '--steps', '3']\n"
        "calls = []\n"
        "rc = bench.maybe_launch(bench.parse_args(argv), argv, run=lambda c: calls.append(c) or 7)\n"
        "heavy = [m for m in ('placement', 'torch', 'oracle', 'numpy') if m in sys.modules]\n"
        "print(json.dumps({'rc': rc, 'cmd': calls[0], 'heavy': heavy}))\n" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True, check=True)
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert got["rc"] == 7                      # the parent exits with the children's status
    assert got["heavy"] == []                  # nothing that loads the engine / a GPU runtime
    cmd = got["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]           # the ranks get the same arguments
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_single_gpu_and_ranks_do_not_relaunch():
    sys.path.insert(0, ROOT)
    import bench
    called = []
    env_ws = os.environ.pop("WORLD_SIZE", None)
    try:
        assert bench.maybe_launch(bench.parse_args([]), [], run=called.append) is None
        os.environ["WORLD_SIZE"] = "2"
        assert bench.maybe_launch(bench.parse_args(["--gpus", "2"]), ["--gpus", "2"], run=called.append) is None
    finally:
        os.environ.pop("WORLD_SIZE", None)
        if env_ws is not None:
            os.environ["WORLD_SIZE"] = env_ws
    assert called == []


def test_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                         capture_output=True, text=True)
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr


def test_default_is_strong_scaling():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.parse_args([]).scaling == "strong"


def test_profile_check_requires_same_build(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    prof = tmp_path / "p"
    prof.mkdir()
    (tmp_path / "LATEST").write_text("p\n")
    summ = {"source_hash": "abc", "workload": {"nodes": 100, "jobs": 10},
            "kernels": {"pe::fit_mask_planes_rows_kernel": {"avg_ns": 1.0e6, "calls": 5, "total_ns": 5e6},
                        "pe::encode_planes_kernel": {"avg_ns": 0.02e6, "calls": 5, "total_ns": 1e5}},
            "pmc": {"pe::fit_mask_planes_rows_kernel": {"hbm_traffic_bytes": 123.0, "SQ_INSTS_VALU": 5.0}}}
    (prof / "summary.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "PROFILES", str(tmp_path))
    ok = bench.profile_check("planes", 100, 10, 1.03, "abc")
    assert ok["profile_matches"] and ok["traffic"] == 123.0 and abs(ok["profile_step_ms"] - 1.02) < 1e-9
    assert not bench.profile_check("planes", 100, 10, 1.03, "other")["profile_matches"]     # other build
    assert bench.PROFILE_TOL == 0.05                                                      # pinned tolerance
    assert bench.profile_check("planes", 100, 10, 1.08, "abc")["traffic"] is None          # > 5 % apart
    assert bench.profile_check("planes", 100, 10, 1.20, "abc")["traffic"] is None
    assert bench.profile_check("planes", 100, 11, 1.03, "abc")["traffic"] is None          # other workload
    # a second profile of the same sources from a slower box: the closest step is taken
    slow = tmp_path / "q"
    slow.mkdir()
    summ2 = json.loads(json.dumps(summ))
    summ2["kernels"]["pe::fit_mask_planes_rows_kernel"]["avg_ns"] = 1.10e6
    summ2["pmc"]["pe::fit_mask_planes_rows_kernel"]["hbm_traffic_bytes"] = 124.0
    (slow / "summary.json").write_text(json.dumps(summ2))
    (tmp_path / "LATEST").write_text("p\nq\n")
    r = bench.profile_check("planes", 100, 10, 1.14, "abc")
    assert r["profile_matches"] and r["traffic"] == 124.0 and r["profile"].endswith("q/summary.json")
    r = bench.profile_check("planes", 100, 10, 1.03, "abc")
    assert r["profile_matches"] and r["traffic"] == 123.0
    assert not bench.profile_check("planes", 100, 10, 1.30, "abc")["profile_matches"]     # neither within 5 %


def test_aggregation_slices_partition_the_batch():
    """bench.py splits the aggregation batch over ranks by contiguous job slices: the slices'
    CalcPGMinResources results (C oracle) concatenate to the whole batch's."""
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    import oracle
    from placement import synth
    agg = synth.make_pg_batch(2001, 3)
    want = oracle.pg_min_resources(1, *agg)
    for world in (2, 3, 8):
        parts = [oracle.pg_min_resources(1, *bench.pg_slice(agg, r * 2001 // world, (r + 1) * 2001 // world))
                 for r in range(world)]
        for k in range(len(want)):
            np.testing.assert_array_equal(np.concatenate([p[k] for p in parts]), want[k])


def test_greedy_and_aggregation_profile_lookups(tmp_path, monkeypatch):
    """greedy_profile / agg_profile_ms read the committed profile's greedy (warm / cold) and
    aggregation passes only when its sources match; agg_roofline prices the call's kernel time
    against the box's PCIe rate."""
    sys.path.insert(0, ROOT)
    import bench
    prof = tmp_path / "p"
    prof.mkdir()
    (tmp_path / "LATEST").write_text("p\n")
    summ = {"source_hash": "abc", "kernels": {},
            "greedy": {"warm": {"pe::walk_kernel": {"avg_ns": 30000.0, "calls": 10, "total_ns": 3e5}},
                       "cold": {"pe::walk_kernel": {"avg_ns": 45000.0, "calls": 10, "total_ns": 4.5e5}}},
            "aggregation": {"pe::pg_agg_seg_kernel": {"avg_ns": 1e5, "calls": 56,
                                                      "total_ns": 2.8e6 * bench.AGG_PROFILE_CALLS}}}
    (prof / "summary.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "PROFILES", str(tmp_path))
    g = bench.greedy_profile("abc")
    assert g["warm"] == 30000.0 and g["cold"] == 45000.0 and g["profile"].endswith("p/summary.json")
    assert bench.greedy_profile("other") == {}
    assert abs(bench.agg_profile_ms("abc") - 2.8) < 1e-9 and bench.agg_profile_ms("other") is None
    # the call's wall time against the slower direction of the link: 42 MB in at 56 GB/s = 0.75 ms
    r = bench.agg_roofline(42_000_000, 14_000_000, 1.5, 1.4, 2.8, {"h2d_gbs": 56.0, "d2h_gbs": 55.0})
    assert r["bound"].startswith("pcie") and abs(r["achieved"] - 28.0) < 1e-9 and abs(r["bound_ms"] - 0.75) < 1e-9
    assert abs(r["frac"] - 0.5) < 1e-9 and abs(r["full_duplex_frac"] - 56.0 / 1.5 / 111.0) < 1e-9
    assert r["wire_frac"] is None
    # narrowed requests: 28 MB on the wire at 56 GB/s = 0.5 ms of the 1.5 ms call
    r = bench.agg_roofline(42_000_000, 14_000_000, 1.5, 1.4, 2.8, {"h2d_gbs": 56.0, "d2h_gbs": 55.0}, 28_000_000)
    assert abs(r["wire_frac"] - 0.5 / 1.5) < 1e-9 and r["wire_bytes"] == 28_000_000
    r = bench.agg_roofline(42_000_000, 14_000_000, 4.0, 3.9, None, None)
    assert r["call_ms"] == 4.0 and r["frac"] is None and r["peak"] is None
