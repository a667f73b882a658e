"""The zero-copy exchange's host merge (training-operator_amd/csrc/pe_merge.h, run by the exchange
thread and its helpers per group) against a sort of the union, at 2 / 4 / 8 / 16 / 32 ranks, through
tools/bench_merge.cc built with the host compiler (verdict r5 item 3: the merge is timed before the
8-GPU run does it)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench_merge(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bm") / "bench_merge")
    subprocess.run(["g++", "-O2", "-std=c++17", "-march=x86-64-v3", "-Wno-psabi",
                    "-I" + os.path.join(ROOT, "training-operator_amd", "csrc"),
                    os.path.join(ROOT, "tools", "bench_merge.cc"), "-o", exe], check=True)
    return exe


def test_host_merge_matches_sorted_union(bench_merge):
    r = subprocess.run([bench_merge, "-3", "2", "3", "4", "5", "8", "16", "32"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: 0 wrong merged lists" in r.stdout, r.stdout
