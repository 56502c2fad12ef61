"""pytest configuration: the `gpu` marker, import paths, and in-tree builds.

`-m "not gpu"` runs on any CPU box (oracle vs golden fixtures, host logic, ABI exports,
multi-process gloo tests); `-m gpu` runs the parity tests proper on an MI355X through the
C ABI of icon-ray-tracing_amd/libicon_rt_hip.so.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "icon-ray-tracing_amd")
for p in (os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    config.addinivalue_line("markers", "slow: larger sizes; still minutes, not hours")


def _ensure_built():
    lib = os.path.join(PKG, "libicon_rt_hip.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", PKG, "lib"])
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()
