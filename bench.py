#!/usr/bin/env python3
"""Benchmark: decode a TPC-H lineitem-shaped Parquet file (SF1: 6,001,215 rows, 16 columns,
Snappy + dictionary, 1 Mi-row row groups; BASELINE.json configs[1]) on MI355X.

One step = one pass of the hot path over the whole file: every page of all 96 column chunks
decompressed and decoded into columnar buffers in HBM, with the chunk bytes already resident in
HBM when the timed region starts (device-resident). N GPUs: one process per GPU, each decodes its
own SF1 file per step (row groups are independent; no collective on the data path) -> weak
scaling; `value` = decoded bytes of all ranks / max-over-ranks time.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parquet-floor_amd"))

SF1_ROWS = 6001215
RG_ROWS = 1 << 20
SEED = 42
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ROOF_PASSES = 3         # isolated decodes of context 0's share for the roofline kernel time


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_input(path, rows):
    import pyarrow.parquet as pq
    from pfloor import datagen
    t0 = time.time()
    t = datagen.lineitem_table(rows, seed=SEED)
    tmp = path + ".tmp"
    pq.write_table(t, tmp, compression="snappy", row_group_size=RG_ROWS)
    os.replace(tmp, path)
    log(f"[bench] wrote {path} ({os.path.getsize(path) / 1e6:.1f} MB) in {time.time() - t0:.1f}s")


def plan_file(path):
    """Chunk bytes (contiguous, 256-B aligned) + descriptors for every chunk of the file."""
    from pfloor.decoder import ParquetFile
    pf = ParquetFile(path)
    items, total = pf.plan(range(pf.num_row_groups), range(pf.num_columns))
    host = np.zeros(total, dtype=np.uint8)
    descs = []
    for rg, col, s, n, off in items:
        if n:
            pf.read_into(s, n, host.ctypes.data + off)
        descs.append(pf.chunk_desc(rg, col, off))
    return pf, items, host, descs


def page_stats(descs):
    """Algorithmic byte counts from the page headers."""
    comp = uncomp = snappy_in = snappy_out = 0
    pages = 0
    for d in descs:
        for i in range(d.n_pages):
            p = d.pages[i]
            pages += 1
            comp += p.compressed_size
            uncomp += p.uncompressed_size
            lvl = (p.rep_bytes + p.def_bytes) if p.page_type == 3 else 0
            if d.codec == 1 and (p.page_type != 3 or p.is_compressed):
                snappy_in += p.compressed_size - lvl
                snappy_out += p.uncompressed_size - lvl
    return dict(pages=pages, compressed=comp, uncompressed=uncomp, snappy_in=snappy_in, snappy_out=snappy_out)


def decoded_bytes(decs, parts, pf, items):
    tot = 0
    rows = 0
    for dec, idx in zip(decs, parts):
      for i, j in enumerate(idx):
        rg, col = items[j][0], items[j][1]
        ci = dec.info(i)
        c = pf.columns[col]
        b = ci.num_slots * ci.width
        if c.max_def > 0:
            b += (ci.num_slots + 7) // 8
        if c.physical_type == 6:
            b += 4 * (ci.num_slots + 1) + ci.num_chars
        if c.max_rep == 1:
            b += 4 * (ci.num_rows + 1) + (ci.num_rows + 7) // 8
        if c.max_rep > 0:
            b += 2 * ci.num_entries
        tot += b
    for rg in range(pf.num_row_groups):
        rows += pf.row_group_rows(rg)
    return tot, rows


def cpu_baseline(path, pf, seconds_budget=12.0, threads=8):
    """The CPU oracle (oracle/pf_oracle.c, a plain-C port of the decode; not the Java reference,
    which cannot run without a JDK + parquet-mr jars) on a bounded sample: row group 0, all
    16 chunks, decoded by `threads` host threads, repeated until ~seconds_budget."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import subprocess
    lib = os.path.join(ROOT, "oracle", "libpf_oracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle_binding import Oracle
    orc = Oracle(lib)
    of = orc.open(path)
    ncols = of.num_columns
    rows_rg0 = pf.row_group_rows(0)
    # decoded bytes of rg0 (from one decode pass)
    dec_bytes = 0
    for c in range(ncols):
        r = of.decode(0, c)
        assert r["status"] == 0, r["error"]
        for k in ("values", "validity", "offsets", "chars"):
            if k in r:
                dec_bytes += r[k].nbytes
    work = [(0, c) for c in range(ncols)]
    passes = 0
    t0 = time.perf_counter()
    while True:
        idx = [0]
        lock = threading.Lock()

        def run():
            while True:
                with lock:
                    if idx[0] >= len(work):
                        return
                    j = idx[0]
                    idx[0] += 1
                of.decode(*work[j])

        ts = [threading.Thread(target=run) for _ in range(threads)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        passes += 1
        if time.perf_counter() - t0 > seconds_budget or passes >= 20:
            break
    dt = time.perf_counter() - t0
    of.close()
    return {"value": round(dec_bytes * passes / dt / 1e9, 4), "unit": "decoded GB/s",
            "rows_per_s": round(rows_rg0 * passes / dt, 1), "cores": threads, "kind": "port",
            "sample": f"row group 0 of the SF1 file ({rows_rg0} rows x {ncols} chunks), {passes} passes, "
                      f"{threads} threads, oracle/pf_oracle.c (C port of parquet-mr 1.12.2 + snappy decode)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=SF1_ROWS)
    ap.add_argument("--data-dir", default=os.environ.get("PF_BENCH_DIR", "/tmp/pfloor_bench"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=4,
                    help="decode contexts (HIP streams) per GPU; row groups are dealt round-robin to them")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)   # barrier/timing only

    import torch
    from pfloor import _native
    from pfloor.decoder import GpuDecoder

    os.makedirs(args.data_dir, exist_ok=True)
    path = os.path.join(args.data_dir, f"lineitem_{args.rows}_seed{SEED}_rg{RG_ROWS}.parquet")
    if rank == 0 and not os.path.exists(path):
        make_input(path, args.rows)
    if dist:
        dist.barrier()

    device = local_rank
    torch.cuda.set_device(device)
    pf, items, host, descs = plan_file(path)
    st = page_stats(descs)
    # S contexts on this GPU (one HIP stream each): row group r goes to context r % S, so one row
    # group's latency-bound Snappy index / chain passes overlap another's decode kernels.
    S = max(1, min(args.streams, pf.num_row_groups))
    decs = [GpuDecoder(device) for _ in range(S)]
    dec = decs[0]
    parts = [[i for i, it in enumerate(items) if it[0] % S == k] for k in range(S)]
    part_descs = [[descs[i] for i in idx] for idx in parts]
    L = _native.lib()
    d_in = C.c_void_p()
    _native.check(L.pf_device_alloc(dec.h, host.nbytes, C.byref(d_in)), dec.h, "pf_device_alloc")
    _native.check(L.pf_memcpy_h2d(dec.h, d_in, host.ctypes.data, host.nbytes), dec.h, "h2d")

    def step():
        for d, dd in zip(decs, part_descs):
            d.decode(dd, d_in.value, host.nbytes, on_device=True)
        for d in decs:
            rc = d.wait()
            if rc != 0:
                raise RuntimeError(d.error())

    for _ in range(args.warmup):
        step()
    dbytes, rows = decoded_bytes(decs, parts, pf, items)
    stage_acc = {}
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for k, v in dec.timing().items():
            stage_acc[k] = stage_acc.get(k, 0.0) + v
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    stage_ms = {k: v / args.steps for k, v in stage_acc.items()}
    ms_per_step = dt / args.steps * 1e3
    n = world
    value = dbytes * n * args.steps / dt / 1e9

    # roofline of the dominant kernel stage: HIP events on context 0's stream, priced with the
    # algorithmic bytes of context 0's share of the pages
    st0 = page_stats(part_descs[0])
    dbytes0, _ = decoded_bytes(decs[:1], parts[:1], pf, items)
    kern_bytes = {
        "snappy_exec": st0["snappy_in"] + st0["snappy_out"],   # compressed read + decompressed written
        "snappy_parse": st0["snappy_in"],                       # compressed read (token index)
        "decode": st0["uncompressed"] + dbytes0,   # page bodies read + decoded bytes written
        "flat": st0["uncompressed"] + dbytes0,
    }
    dom = max((k for k in stage_ms if k != "h2d"), key=lambda k: stage_ms.get(k, 0.0))
    # per-launch kernel time of the dominant stage without a concurrent stream: with several contexts
    # the HIP events on context 0 also count the time its kernels wait for CUs held by context 1,
    # which rocprof's kernel durations do not. Context 0's share, decoded alone, ROOF_PASSES times
    # after the timed region (HIP events on its stream bracket exactly that stage's launches).
    iso = {}
    for _ in range(ROOF_PASSES):
        dec.decode(part_descs[0], d_in.value, host.nbytes, on_device=True)
        if dec.wait() != 0:
            raise RuntimeError(dec.error())
        for k, v in dec.timing().items():
            iso[k] = iso.get(k, 0.0) + v / ROOF_PASSES
    dom_ms = iso.get(dom, 0.0)
    dom_bytes = kern_bytes.get(dom)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if (dom_bytes and dom_ms > 0) else None
    # HBM traffic of the dominant kernel: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE per
    # launch over the whole file at 1 stream (tools/gpu_pmc.sh -> tools/pmc_traffic.json), scaled
    # to context 0's share of the algorithmic bytes
    traffic = None
    try:
        pmc = json.load(open(os.path.join(ROOT, "tools", "pmc_traffic.json")))
        whole = {"snappy_exec": st["snappy_in"] + st["snappy_out"]}
        if f"k_{dom}" in pmc and dom in whole and dom_bytes:
            traffic = round(pmc[f"k_{dom}"]["traffic_bytes"] * dom_bytes / whole[dom])
    except (OSError, ValueError, KeyError):
        pass
    b_alg = st["compressed"] + dbytes
    out = {
        "metric": "decoded GB/s + rows/s (node), lineitem-shape Snappy+dict, 1/2/4/8 GPUs",
        "value": round(value, 3), "unit": "decoded GB/s",
        "rows_per_s": round(rows * n * args.steps / dt, 1),
        "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (pyarrow-written lineitem-shaped file, seed 42)",
        "config": {"workload": f"lineitem SF1 ({rows} rows, 16 cols, {len(descs)} chunks, {st['pages']} pages), "
                               "Snappy + dictionary, 1Mi-row row groups, device-resident",
                   "rows": rows, "row_groups": pf.num_row_groups, "compressed_page_bytes": st["compressed"],
                   "uncompressed_page_bytes": st["uncompressed"], "decoded_bytes": dbytes,
                   "parallelism": f"row groups sharded per GPU x{n} (no collective), {S} decode streams per GPU"},
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "roofline": {"bound": "hbm", "kernel": f"k_{dom}", "achieved": round(achieved, 2) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None, "traffic": traffic,
                     "traffic_source": "rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE per launch (tools/gpu_pmc.sh)",
                     "algorithmic_bytes_per_launch": dom_bytes, "launch_ms": round(dom_ms, 4),
                     "launch_ms_source": f"HIP events on context 0's stream, its row groups decoded alone x{ROOF_PASSES} "
                                         "after the timed region",
                     "stage_ms_overlapped": round(stage_ms.get(dom, 0.0), 4)},
        "pipeline_roofline": {"b_alg": b_alg, "ms_per_step": round(ms_per_step, 4),
                              "achieved": round(b_alg * n / (ms_per_step * 1e-3) / 1e9, 2),
                              "frac": round(b_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
    }
    if rank == 0 and n == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(path, pf)
        except Exception as e:   # reported, never fatal
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    L.pf_device_free(dec.h, d_in)
    for d in decs:
        d.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
