"""Runs the table-driven C++ tests of the host mirror (tests/cpp/test_host.cc)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "host_tests")


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "training-operator_amd", "host")], check=True)


def run(flag):
    if not os.path.exists(BIN):
        build()
    p = subprocess.run([BIN, flag], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failed checks" in p.stdout
    return p.stdout


def test_host_mirror_cpu_cases():
    build()
    out = run("--cpu")
    assert "TestRunEnforceMLPolicyPlugins" in out


@pytest.mark.gpu
def test_host_mirror_gpu_cases():
    out = run("--gpu")
    for name in ("TestNewInfo", "TestTrainingRuntimeNewObjects", "TestIntegrationPodGroup", "TestCalcPGMinResourcesMnist",
                 "TestNodeInventoryInformer", "TestSyncPodGroupV1", "TestBuildWireV2",
                 "TestResourcesPerNodeTotalRequests", "TestCalcPGMinResourcesTiePolicy"):
        assert "ok   " + name in out
