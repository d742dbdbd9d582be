"""One rank of the two-process config-3 test (tests/test_gpu_shard.py): row groups of 4,000,000 rows
sharded round-robin (pfloor.shard), each rank decoding its own row groups on the visible GPU through
libpfloor.so and checking them bit-exactly against the CPU oracle; rank 0 then reassembles the
per-chunk digests of both ranks in file order (ORDERED delivery, ParquetReader.java:225-227) and
checks them against the oracle's digests of the whole file. Started by conftest.py before the
pytest process touches the GPU; writes <out>/rank<r>.json.

  python tests/shard_worker.py --rank R --world 2 --port P --path FILE --out DIR"""
import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), HERE]

RG_ROWS = 4_000_000
N_RG = 2


def digest(arrs):
    """sha256 of a decoded chunk in the canonical layout (validity bitmaps as their first n bits)."""
    import numpy as np
    h = hashlib.sha256()
    for k in ("values", "validity", "offsets", "chars", "list_offsets", "list_validity", "def_levels", "rep_levels"):
        if k in arrs:
            a = np.asarray(arrs[k])
            if k in ("validity", "list_validity"):
                n = int(arrs["num_slots"] if k == "validity" else arrs["num_rows"])
                a = np.unpackbits(a.view(np.uint8), bitorder="little")[:n]
            h.update(k.encode())
            h.update(a.tobytes())
    return h.hexdigest()


def make_file(path):
    import pyarrow.parquet as pq
    from pfloor import datagen
    if os.path.exists(path):
        return
    t = datagen.lineitem_table(RG_ROWS * N_RG, seed=43, scale=100.0)
    tmp = path + ".tmp"
    pq.write_table(t, tmp, compression="snappy", row_group_size=RG_ROWS)
    os.replace(tmp, path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--path", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {"rank": a.rank, "ok": False}
    t0 = time.time()
    try:
        import torch.distributed as dist
        if a.rank == 0:
            make_file(a.path)
        res["gen_s"] = round(time.time() - t0, 1)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port))
        dist.init_process_group("gloo", rank=a.rank, world_size=a.world)   # test harness only: digests, barrier
        from oracle_binding import Oracle
        from golden_util import assert_chunk_equal
        from pfloor.decoder import GpuDecoder, ParquetFile, decode_file
        from pfloor.shard import reassemble, row_groups_for_rank
        orc = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
        with ParquetFile(a.path) as pf:
            nrg, ncol = pf.num_row_groups, pf.num_columns
            assert nrg == N_RG and pf.row_group_rows(0) == RG_ROWS, (nrg, pf.row_group_rows(0))
        mine = row_groups_for_rank(nrg, a.rank, a.world)
        dec = GpuDecoder(0)
        per_rg = {}
        n_chunks = 0
        with cf.ThreadPoolExecutor(8) as ex:
            for g in mine:
                got = decode_file(a.path, row_groups=[g], decoder=dec)
                assert got["_status"] == 0, got["_error"]
                handles = [orc.open(a.path) for _ in range(ncol)]
                futs = [ex.submit(handles[c].decode, g, c) for c in range(ncol)]
                digs = []
                for c, fu in enumerate(futs):
                    assert_chunk_equal(got[(g, c)], fu.result(), f"rank{a.rank} rg{g} c{c}")
                    digs.append(digest(got[(g, c)]))
                    n_chunks += 1
                for h in handles:
                    h.close()
                per_rg[g] = digs
        dec.close()
        res.update(row_groups=mine, chunks_checked=n_chunks)
        gathered = [None] * a.world
        dist.all_gather_object(gathered, per_rg)
        if a.rank == 0:
            ordered = reassemble(gathered, nrg)
            with orc.open(a.path) as of:
                for g in range(nrg):
                    exp = [digest(of.decode(g, c)) for c in range(ncol)]
                    assert ordered[g] == exp, f"row group {g}: reassembled digests differ from the oracle's"
            res["reassembled_row_groups"] = nrg
        dist.barrier()
        dist.destroy_process_group()
        res["ok"] = True
    except Exception:
        res["error"] = traceback.format_exc()[-3000:]
    res["wall_s"] = round(time.time() - t0, 1)
    with open(os.path.join(a.out, f"rank{a.rank}.json"), "w") as f:
        json.dump(res, f)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
