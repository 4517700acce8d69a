"""Runs the C++11 shim test (tests/cpp/test_shim.cpp): include/kadgpu.hpp's RoutingTableMirror,
NodeCacheMirror and DhtMirror over OpenDHT-shaped test doubles, against the oracle."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp")], check=True)
    return os.path.join(HERE, "cpp", "test_shim")


def test_cpp_shim_compiles():
    assert os.path.exists(_build())


@pytest.mark.gpu
def test_cpp_shim_parity():
    exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
    print("\n".join(l for l in r.stdout.splitlines() if l.startswith(("LATENCY", "mirror"))))
