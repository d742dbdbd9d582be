"""Config 3 (lineitem-shaped, 4,000,000-row row groups) sharded over two processes on the visible
GPU: each decodes its round-robin row groups (pfloor.shard) through libpfloor.so, bit-exact
against the oracle, and rank 0 reassembles both ranks' chunk digests in file order and checks
them against the oracle (tests/shard_worker.py). The two processes are started by conftest.py
right after collection, before this pytest process makes any GPU call (a process that has
initialised the GPU must not start others), and run while the other GPU tests do."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu


def test_two_process_sharded_config3(shard_run):
    procs, out = shard_run
    assert procs, "shard workers were not started (conftest.pytest_collection_finish)"
    for p in procs:
        try:
            p.wait(timeout=110)
        except Exception:
            p.kill()
            raise
    res = []
    for r in range(len(procs)):
        with open(os.path.join(out, f"rank{r}.json")) as f:
            res.append(json.load(f))
    for r in res:
        assert r["ok"], r.get("error")
    assert sorted(g for r in res for g in r["row_groups"]) == [0, 1]
    assert res[0]["reassembled_row_groups"] == 2
    assert all(r["chunks_checked"] == 16 for r in res)
