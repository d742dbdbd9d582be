"""Shared pytest setup: the `gpu` marker, paths, and on-demand builds of the CPU oracle
and the product library (both are plain `make` targets; no GPU needed to build)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "parquet-floor_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")


def _make(dirpath, target):
    subprocess.run(["make", "-s", "-C", dirpath, target], check=True)


@pytest.fixture(scope="session")
def oracle():
    from oracle_binding import Oracle
    lib = os.path.join(ROOT, "oracle", "libpf_oracle.so")
    if not os.path.exists(lib):
        _make(os.path.join(ROOT, "oracle"), "all")
    return Oracle(lib)


def golden_files():
    return sorted(f[:-len(".parquet")] for f in os.listdir(GOLDEN) if f.endswith(".parquet"))
