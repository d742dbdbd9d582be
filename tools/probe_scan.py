"""Diagnostic: GPU page-header scan (pf_scan_pages) of every chunk of the SF1 bench file, bytes
resident in HBM, with and without CRC verification, beside the host walk (pf_file_chunk_desc).
Usage: python tools/probe_scan.py [reps]"""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-floor_amd")]
import bench  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor._native import PageDesc, ScanChunk, ScanResult, check, lib  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
path = bench.make_input(argparse.Namespace(workload="sf1", data_dir="/tmp/pfloor_bench"))
L = lib()
with ParquetFile(path) as pf:
    items, total = pf.plan(range(pf.num_row_groups), range(pf.num_columns))
    host = np.zeros(total, np.uint8)
    t0 = time.perf_counter()
    npages = 0
    descs = []
    for rg, col, s, n, off in items:
        pf.read_into(s, n, host.ctypes.data + off)
    t_read = time.perf_counter() - t0
    t0 = time.perf_counter()
    for rg, col, s, n, off in items:
        d = pf.chunk_desc(rg, col, off)
        descs.append(d)
        npages += d.n_pages
    t_host = time.perf_counter() - t0
    nv = [sum(d.pages[i].num_values for i in range(d.n_pages) if d.pages[i].page_type != 2) for d in descs]
dec = GpuDecoder(0)
dptr = C.c_void_p()
check(L.pf_device_alloc(dec.h, total, C.byref(dptr)), dec.h)
check(L.pf_memcpy_h2d(dec.h, dptr, host.ctypes.data, total), dec.h)
check(L.pf_sync(dec.h), dec.h)
cap = 1024
sc = (ScanChunk * len(items))(*[ScanChunk(off, n, v, i * cap, cap) for i, ((rg, col, s, n, off), v) in enumerate(zip(items, nv))])
pages = (PageDesc * (len(items) * cap))()
res = (ScanResult * len(items))()
for crc in (0, 1):
    ts = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        rc = L.pf_scan_pages(dec.h, sc, len(items), dptr, total, 1, crc, pages, res)
        ts.append(time.perf_counter() - t0)
        assert rc == 0, L.pf_last_error(dec.h)
    got = sum(res[i].n_pages for i in range(len(items)))
    assert got == npages
    ok = all(all(getattr(pages[i * cap + k], f) == getattr(descs[i].pages[k], f) for f, _ in PageDesc._fields_)
             for i in range(len(items)) for k in range(res[i].n_pages))
    print(f"pf_scan_pages verify_crc={crc}: {len(items)} chunks, {got} pages, {total / 1e6:.1f} MB, "
          f"median {np.median(ts[1:]) * 1e3:.3f} ms (sync call incl. copies), descs match host walk: {ok}", flush=True)
print(f"host walk (pf_file_chunk_desc, 1 thread): {t_host * 1e3:.3f} ms for {npages} pages", flush=True)
