"""CPU tests of the per-group window hand-over (pe::WindowFeed, pe_resolver.cpp) and of the resolver
fed by it: tests/cpp/test_feed.cc, built here with g++ against the resolver source, plain and under
ThreadSanitizer (the resolver thread, the seed helper and the producer thread share the blob)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tests", "cpp", "test_feed.cc"),
       os.path.join(ROOT, "training-operator_amd", "csrc", "pe_resolver.cpp")]
INC = ["-I" + os.path.join(ROOT, "training-operator_amd", "csrc"), "-I" + os.path.join(ROOT, "include")]


def build_and_run(out, flags):
    subprocess.run(["g++", "-std=c++17", "-march=x86-64-v3", "-pthread", *flags, *INC, *SRC, "-o", out], check=True,
                   timeout=300)
    p = subprocess.run([out], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failed checks" in p.stdout
    assert "WARNING: ThreadSanitizer" not in p.stderr, p.stderr
    return p.stdout


def test_window_feed(tmp_path):
    out = build_and_run(str(tmp_path / "feed_tests"), ["-O2"])
    assert out.count("ok   fed resolve") == 6
    assert "ok   order/wait/idle/deadline" in out
    assert "ok   seed scorer start/stop handshake" in out


def test_seed_scorer_handshake_forced_yield(tmp_path):
    """The helper yields between reading its state and acting on it (PE_SEED_TEST_YIELD)."""
    out = build_and_run(str(tmp_path / "feed_yield"), ["-O2", "-DPE_SEED_TEST_YIELD"])
    assert "ok   seed scorer start/stop handshake" in out


def test_window_feed_tsan(tmp_path):
    probe = subprocess.run(["g++", "-fsanitize=thread", "-x", "c++", "-", "-o", str(tmp_path / "probe")],
                           input="int main(){}", text=True, capture_output=True)
    if probe.returncode != 0:
        pytest.skip("no ThreadSanitizer runtime")
    build_and_run(str(tmp_path / "feed_tsan"), ["-O1", "-g", "-fsanitize=thread", "-DPE_SEED_TEST_YIELD"])
