"""Multi-GPU path on CPU: world_size-2 `gloo` processes shard a file's row groups round-robin
(pfloor.shard), decode their own row groups (the CPU oracle stands in for the GPU here: no device
in this container), and rank 0 reassembles file order and checks it against a single-process
decode. Also checks the max-over-ranks timing reduction bench.py uses."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]
    import torch
    from oracle_binding import Oracle
    from pfloor.shard import row_groups_for_rank
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
        with o.open(path) as of:
            mine = {g: [of.decode(g, c) for c in range(of.num_columns)]
                    for g in row_groups_for_rank(of.num_row_groups, rank, world)}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)   # test harness only: the product path has no collective
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((gathered, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_two_rank_row_group_sharding(oracle):
    from pfloor.shard import reassemble
    path = os.path.join(GOLDEN, "c2_lineitem.parquet")
    with oracle.open(path) as of:
        nrg, ncol = of.num_row_groups, of.num_columns
        ref = [[of.decode(g, c) for c in range(ncol)] for g in range(nrg)]
    assert nrg >= 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    ordered = reassemble(gathered, nrg)
    for g in range(nrg):
        for c in range(ncol):
            a, b = ordered[g][c], ref[g][c]
            for k in ("values", "validity", "offsets", "chars"):
                if k in b:
                    assert np.array_equal(a[k], b[k]), (g, c, k)


def test_shard_helpers():
    from pfloor.shard import balance, reassemble, row_groups_for_rank
    assert row_groups_for_rank(151, 0, 8)[:3] == [0, 8, 16]
    assert sum(len(row_groups_for_rank(151, r, 8)) for r in range(8)) == 151
    assert abs(balance(151, 8) - 19 / (151 / 8)) < 1e-9      # SF100: 19 vs 18.9 row groups
    with pytest.raises(ValueError):
        reassemble([{0: 1}, {0: 2}], 2)
    with pytest.raises(ValueError):
        reassemble([{0: 1}, {}], 2)


def test_bench_work_plan_shards_row_groups():
    """bench.py's per-rank plan: SF1 x N logical row groups dealt round-robin (weak scaling), SF100's
    150 logical row groups dealt round-robin (strong), each rank's units dealt to its streams."""
    import sys
    sys.path.insert(0, ROOT)
    import argparse
    import bench

    class FakePF:
        def __init__(self, nrg, ncol):
            self.num_row_groups, self.num_columns = nrg, ncol

    for wl, nphys, expect_total in (("sf1", 6, None), ("sf100", 2, 150)):
        for world in (1, 2, 4, 8):
            seen = []
            for rank in range(world):
                a = argparse.Namespace(workload=wl)
                plan, n_log, mine = bench.units_for_rank(a, FakePF(nphys, 16), world, rank, 4)
                assert n_log == (expect_total or 6 * world)
                units = [u for ctx in plan for b in ctx for u in b]
                assert sorted(u[0] for u in units) == mine
                assert all(u[1] == u[0] % nphys for u in units)
                seen += mine
                if wl == "sf1":
                    assert len(mine) == 6 and len(plan) == 4 and all(len(ctx) == 1 for ctx in plan)
            assert sorted(seen) == list(range(n_log))
    a = argparse.Namespace(workload="wide")
    plan, _, _ = bench.units_for_rank(a, FakePF(1, 500), 1, 0, 4)
    cols = sorted(c for ctx in plan for b in ctx for u in b for c in u[2])
    assert cols == list(range(500)) and len(plan) == 4


def test_bench_column_split_plan_covers_every_chunk_once():
    """bench.py's column-split plan (SF1's, config 1's): column slices dealt LPT to the streams, with
    the per-workload BYTE_ARRAY weight and row-group slice multiplier. Every (row group, column) chunk
    is decoded by exactly one stream, for multipliers 1-3 and 1/2 ranks."""
    import sys
    sys.path.insert(0, ROOT)
    import argparse
    import random
    import bench

    class Col:
        def __init__(self, pt):
            self.physical_type = pt

    class FakePF:
        def __init__(self, nrg, ncol, seed):
            rng = random.Random(seed)
            self.num_row_groups, self.num_columns = nrg, ncol
            self.columns = [Col(6 if c % 5 == 4 else 2) for c in range(ncol)]
            self.size = {(p, c): rng.randint(1, 40) << 20 for p in range(nrg) for c in range(ncol)}

        def chunk_range(self, p, c):
            return (0, self.size[(p, c)])

    for wl in ("sf1", "flat"):
        for mult in (1, 2, 3):
            for world in (1, 2):
                seen = []
                for rank in range(world):
                    a = argparse.Namespace(workload=wl, split="columns", slice_mult=mult, string_weight=None,
                                           lpt_cost="compressed")
                    plan, n_log, mine = bench.units_for_rank(a, FakePF(6, 16, 7), world, rank, 4)
                    assert len(plan) <= 4
                    for ctx in plan:
                        for batch in ctx:
                            for g, p, cols in batch:
                                assert g in mine and p == g % 6
                                seen += [(g, c) for c in cols]
                assert sorted(seen) == sorted((g, c) for g in range(n_log) for c in range(16)), (wl, mult, world)
