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


@pytest.fixture
def switches(monkeypatch):
    """switches(PF_NAME=value, ...): a context in which decoders run the diagnostics build of the
    library with those PfOpts switches (read at pf_ctx_create; the product library reads no
    environment). Decoders made inside must be closed inside."""
    import contextlib
    from pfloor import _native

    @contextlib.contextmanager
    def ctx(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, str(v))
        try:
            with _native.diagnostics():
                yield
        finally:
            for k in env:
                monkeypatch.delenv(k, raising=False)
    return ctx


def golden_files():
    return sorted(f[:-len(".parquet")] for f in os.listdir(GOLDEN) if f.endswith(".parquet"))


# ---- two-process config-3 test (test_gpu_shard.py): its workers start right after collection,
# before any test (and so this process) touches the GPU, and run alongside the other GPU tests.
_SHARD = {"procs": [], "out": None}
SHARD_TEST = "test_two_process_sharded_config3"


def pytest_collection_finish(session):
    if not any(it.name == SHARD_TEST for it in session.items):
        return
    import socket
    import tempfile
    out = tempfile.mkdtemp(prefix="pf_shard_")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    path = os.path.join(os.environ.get("PF_BENCH_DIR", "/tmp/pfloor_bench"), "lineitem_sf100rg_8000000_seed43.parquet")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    worker = os.path.join(ROOT, "tests", "shard_worker.py")
    for r in range(2):
        log = open(os.path.join(out, f"rank{r}.log"), "w")
        _SHARD["procs"].append(subprocess.Popen(
            [sys.executable, worker, "--rank", str(r), "--world", "2", "--port", str(port), "--path", path, "--out", out],
            stdout=log, stderr=subprocess.STDOUT))
    _SHARD["out"] = out


@pytest.fixture(scope="session")
def shard_run():
    return _SHARD["procs"], _SHARD["out"]
