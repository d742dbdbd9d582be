#!/usr/bin/env python3
"""Benchmark of the Parquet column-chunk decode path (BASELINE.json: "decoded GB/s + rows/s (node),
lineitem-shape Snappy+dict, 1/2/4/8 GPUs").

Workloads (--workload):
  sf1    (default; BASELINE configs[1]) TPC-H lineitem-shaped SF1: 6,001,215 rows, 16 columns,
         Snappy + dictionary, 1 Mi-row row groups, seed 42. At N GPUs the logical file is SF1 x N
         (the 6 row groups repeated N times = 6N row groups) sharded round-robin by pfloor.shard:
         weak scaling, every rank decodes 6 row groups per step.
  sf100  (configs[2]) lineitem-shaped SF100: 150 row groups of 4,000,000 rows sharded round-robin
         over the N GPUs (strong scaling). The two distinct synthetic row groups written on the box
         stand for the 150 (logical row group g decodes physical row group g % 2 in full).
  wide   (configs[3]) 1,000,000 rows x 500 nullable INT32/FLOAT columns, 30 % nulls, 100,000-value
         dictionaries (400 KB, larger than LDS); the row group's columns are split over the streams.

One step = one pass of the hot path over the rank's share: every page of every selected column
chunk decompressed and decoded into columnar buffers in HBM, compressed bytes already resident in
HBM (device-resident). `value` = decoded bytes of all ranks / max-over-ranks step time.
After the timed region (never inside it): bit-exact parity of the timed outputs against the CPU
oracle, the dominant kernel's isolated launch time (roofline), the end-to-end rate (pinned host
input -> H2D -> decode -> D2H into pinned host columns), and CPU baselines on the host cores.
The dominant kernel's HBM traffic comes from rocprofv3 --pmc passes run as child processes
before this process touches the GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload sf1|sf100|wide]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself (child
processes, before any GPU call). Prints ONE JSON line on rank 0.
"""
import argparse
import concurrent.futures as cf
import csv
import ctypes as C
import glob
import json
import os
import re
import shutil
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parquet-floor_amd"))

SF1_ROWS = 6001215
RG_ROWS = 1 << 20
SEED = 42
# PF_* switches act only on the diagnostics build (PFLOOR_LIB_PATH=parquet-floor_amd/diag/libpfloor_diag.so,
# PfOpts in pf_internal.h); the product library reads no environment.
_DIAG = "libpfloor_diag" in os.environ.get("PFLOOR_LIB_PATH", "")
# PF_DEBUG_SKIP (stage ablation, diagnostics build): skipped stages leave chunks failed by design
_SKIP = _DIAG and bool(os.environ.get("PF_DEBUG_SKIP"))
_EXEC = os.environ.get("PF_EXEC", "5")[:1] if _DIAG else "5"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PCIE_GBS = 63.0         # MI355X_MICROARCH.md: PCIe Gen5 x16 per direction
# kernels of each stage (rocprof names, pf_runtime.hip's launch order between the stage events), for
# the PMC traffic and the label of the roofline object
STAGE_KERNELS = {
    "snappy_parse": r"k_snappy_(head|litcopy|index|chain|repair|splits)$",
    "snappy_exec": r"k_snappy_(exec2|exec5|serial)$",
    "delta": r"k_(dbp_pos|dbp_blk|dbp_scan|delta)$",
    "levels": r"k_(runs|lvl|dlen)$",
    "count": r"k_(nest_lvl|count|count_flat|count_dict|count_seg|nest_scan|nest_ids|nest_chars|ba_[a-z]+)$",
    "scan": r"k_scan$",
    "flat": r"k_flat(_all|_fixed|_null|_fb)?$",
    "decode": r"k_(decode|decode_seg|dba_chars)$",
}
STAGE_LABEL = {"snappy_exec": "Snappy executor stage: k_snappy_exec%s (+ redo, serial fallback)" % _EXEC,
               "snappy_parse": "Snappy parse stage: k_snappy_head + index + chain + repair + splits",
               "delta": "DELTA_BINARY_PACKED stage: k_dbp_pos / k_dbp_blk / k_dbp_scan + k_delta",
               "levels": "level / id run stage: k_runs + k_lvl + k_dlen",
               "count": "count stage: k_nest_lvl, k_count[_flat|_seg], k_nest_scan / ids / chars, PLAIN BYTE_ARRAY k_ba_*",
               "scan": "k_scan", "flat": "flat stage: k_flat_null<4/8> + k_flat_fixed + k_flat_all (+ its fallback-queue workgroups)",
               "decode": "decode stage: k_decode + k_decode_seg + k_dba_chars"}
# the algorithmic bytes each stage is priced with (bench.stage_bytes)
STAGE_BYTES_DEF = {
    "snappy_parse": "compressed Snappy stream bytes read",
    "snappy_exec": "compressed Snappy stream bytes read + decompressed bytes written",
    "delta": "DELTA_BINARY_PACKED sections read + values written (4 or 8 B)",
    "levels": "page bodies (decompressed) of nullable / dictionary-encoded pages, read once",
    "count": "page bodies (decompressed) of BYTE_ARRAY and nested pages, read once",
    "scan": "none (prefix sums over page counts)",
    "flat": "page bodies (decompressed) read once + decoded column bytes written",
    "decode": "page bodies (decompressed) read once + decoded column bytes written",
}
ROOF_PASSES = 3         # isolated decodes of context 0's first batch for the roofline kernel time
E2E_PASSES = 2
E2E_STREAM_PASSES = 6   # E2E streamed: the file decoded this many times back to back (a reader over several files)
METRIC = "decoded GB/s + rows/s (node), lineitem-shape Snappy+dict, 1/2/4/8 GPUs"

WORKLOADS = {
    # physical file, logical row groups, row groups per decode batch
    # slice_mult 2: each column cut into twice as many row-group slices as its LPT share needs
    # (2.612-2.624 vs 2.634-2.653 ms at 1, 2.658-2.679 at 3; r05, gpurun_out/slices_sf1)
    "sf1": dict(rows=SF1_ROWS, rg_rows=RG_ROWS, seed=SEED, kind="lineitem", batch=0, slice_mult=2),
    "sf100": dict(rows=8_000_000, rg_rows=4_000_000, seed=43, kind="lineitem", batch=1, logical=150),
    "wide": dict(rows=1_000_000, rg_rows=1_000_000, seed=4, kind="wide", batch=1),
    # (configs[4]) l optional LIST<STRUCT<a INT64 (DELTA_BINARY_PACKED), b UTF8 (dictionary)>>, v2 pages
    # batch 0: the column split (as sf1): 0.84 vs 0.905 ms with one row group per batch (r04)
    "nested": dict(rows=1_000_000, rg_rows=250_000, seed=5, kind="nested", batch=0),
    # (configs[0]) INT64 / DOUBLE / nullable INT32 / dictionary UTF8, uncompressed
    # (batch 0: 0.278 vs 0.380 ms with one row group per batch, r04). string_weight 4: the string
    # column gets a stream of its own (its chain: value walk, runs, counts, scan, string gather):
    # 0.142-0.146 vs 0.181 ms at 1 (r05, gpurun_out/sw; 2: 0.182, 8: 0.204; config 5 is best at 1)
    "flat": dict(rows=1_000_000, rg_rows=250_000, seed=1, kind="flat", batch=0, string_weight=4.0),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def input_path(args):
    w = WORKLOADS[args.workload]
    pool = getattr(args, "pool", 100000)
    tag = f"_pool{pool}" if w["kind"] == "wide" and pool != 100000 else ""
    return os.path.join(args.data_dir, f"{w['kind']}_{w['rows']}_seed{w['seed']}_rg{w['rg_rows']}{tag}.parquet")


def make_input(args):
    path = input_path(args)
    if os.path.exists(path):
        return path
    import pyarrow.parquet as pq
    from pfloor import datagen
    w = WORKLOADS[args.workload]
    t0 = time.time()
    os.makedirs(args.data_dir, exist_ok=True)
    kw = dict(compression="snappy")
    if w["kind"] == "lineitem":
        # sf100's row groups are SF100-shaped (key ranges of the full 600M-row file)
        t = datagen.lineitem_table(w["rows"], seed=w["seed"], scale=100.0 if args.workload == "sf100" else None)
    elif w["kind"] == "nested":
        t = datagen.nested_table(w["rows"], seed=w["seed"])
        kw = dict(compression="snappy", data_page_version="2.0",
                  column_encoding={"l.list.element.a": "DELTA_BINARY_PACKED"}, use_dictionary=["l.list.element.b"])
    elif w["kind"] == "flat":
        t = datagen.flat_table(w["rows"], seed=w["seed"])
        kw = dict(compression="NONE")
    else:
        t = datagen.wide_table(w["rows"], seed=w["seed"], pool=getattr(args, "pool", 100000))
    tmp = path + f".tmp{os.getpid()}"
    pq.write_table(t, tmp, row_group_size=w["rg_rows"], **kw)
    os.replace(tmp, path)
    log(f"[bench] wrote {path} ({os.path.getsize(path) / 1e6:.1f} MB) in {time.time() - t0:.1f}s")
    return path


# --------------------------------------------------------------------------- work plan

def logical_row_groups(args, n_phys, world):
    w = WORKLOADS[args.workload]
    if args.workload == "sf1":
        return n_phys * world              # SF1 x N (weak scaling)
    return w.get("logical", n_phys)


def chunk_cost(pf, p, c, kind, row_cost=0.0):
    """LPT cost of one column chunk: its compressed bytes, or the decompressed bytes of its pages
    (what the Snappy executor and the value kernels walk: dense integer columns cost more per
    compressed byte than text), plus row_cost bytes per row (the flat stage's blocks scale with rows:
    a 1-bit dictionary column is a few hundred KB but as many blocks as any other column)."""
    extra = row_cost * pf.row_group_rows(p) if row_cost else 0.0
    if kind == "compressed":
        return pf.chunk_range(p, c)[1] + extra
    d = pf.chunk_desc(p, c, 0)
    return sum(d.pages[i].uncompressed_size for i in range(d.n_pages)) + extra


def wl_batch(args):
    """Row groups per decode batch: the workload's (0 = the column split over all row groups), or --rg-batch."""
    b = getattr(args, "rg_batch", None)
    return WORKLOADS[args.workload]["batch"] if b is None else b


def units_for_rank(args, pf, world, rank, S, batch=None):
    """This rank's work units (logical rg, physical rg, columns), dealt to S contexts, then grouped
    into decode batches: [[batch, ...] per context], batch = list of units."""
    from pfloor.shard import row_groups_for_rank
    n_phys = pf.num_row_groups
    n_log = logical_row_groups(args, n_phys, world)
    mine = row_groups_for_rank(n_log, rank, world)
    cols = list(range(pf.num_columns))
    if getattr(args, "columns", None):   # analysis: a column subset (not a bench line of BASELINE's config)
        cols = [int(c) for c in args.columns.split(",")]
    units = [(g, g % n_phys, cols) for g in mine]
    if args.workload == "wide" and units:   # one row group: split its columns over the contexts
        g, p, _ = units[0]
        k = max(1, min(S * (getattr(args, "wide_groups", None) or 1), len(cols)))   # column groups (batches)
        units = [(g, p, cols[i::k]) for i in range(k)] + units[1:]
    elif getattr(args, "split", "rowgroups") == "kinds" and units and S > 2 and batch is None and \
            wl_batch(args) <= 0:
        # A context's time is the sum of its stages' latencies, and every kind of page it holds adds
        # stages: BYTE_ARRAY columns add the value walk, the chars count and scan and the string
        # gather; fixed-width columns add the run tables and the fixed gather. Keep the kinds apart:
        # BYTE_ARRAY columns on `string_ctx` contexts, fixed-width columns on the others, each group
        # dealt as in "columns" (heavy columns cut into row-group slices, longest first).
        size = {(p, c): pf.chunk_range(p, c)[1] for _, p, _ in units for c in cols}
        strs = [c for c in cols if pf.columns[c].physical_type == 6]
        fixed = [c for c in cols if pf.columns[c].physical_type != 6]
        ks = max(1, min(S - 1, getattr(args, "string_ctx", 2))) if strs and fixed else (S if strs else 0)
        groups = [(strs, ks), (fixed, S - ks)]
        per = []
        for gcols, gS in groups:
            if not gcols or gS <= 0:
                continue
            cost = {c: sum(size[(p, c)] for _, p, _ in units) for c in gcols}
            share = sum(cost.values()) / gS
            slices = []
            for c in gcols:
                k = max(1, min(len(units), -(-cost[c] // max(1, int(share)))))
                for j in range(k):
                    us = units[j::k]
                    slices.append((sum(size[(p, c)] for _, p, _ in us), c, [(g, p) for g, p, _ in us]))
            load = [0] * gS
            gper = [dict() for _ in range(gS)]
            for cst, c, gps in sorted(slices, key=lambda t: -t[0]):
                k = min(range(gS), key=lambda k: load[k])
                load[k] += cst
                for gp in gps:
                    gper[k].setdefault(gp, []).append(c)
            per += gper
        return [[[(g, p, sorted(cs)) for (g, p), cs in sorted(d.items())]] for d in per if d], n_log, mine
    elif getattr(args, "split", "rowgroups") in ("columns", "kinds") and units and S > 1 and batch is None and \
            wl_batch(args) <= 0:
        # Each context decodes a few columns over the rank's row groups: a stage's latency is set by
        # its slowest item (a heavy column's Snappy pieces, string blocks) more than by how many items
        # it has, so heavy columns go to different contexts and their stage chains overlap instead
        # of adding up. A column heavier than a context's fair share is cut into that many slices of
        # its row groups; slices go longest-processing-time first (compressed bytes) to the least
        # loaded context.
        sw = getattr(args, "string_weight", None) or 1.0
        size = {(p, c): chunk_cost(pf, p, c, getattr(args, "lpt_cost", "compressed"), getattr(args, "row_cost", None) or 0.0) *
                (sw if pf.columns[c].physical_type == 6 else 1.0) for _, p, _ in units for c in cols}
        cost = {c: sum(size[(p, c)] for _, p, _ in units) for c in cols}
        share = sum(cost.values()) / S
        slices = []
        for c in cols:
            k = max(1, min(len(units), int(-(-cost[c] // max(1, int(share)))) * (getattr(args, "slice_mult", None) or 1)))
            for j in range(k):
                us = units[j::k]
                slices.append((sum(size[(p, c)] for _, p, _ in us), c, [(g, p) for g, p, _ in us]))
        load = [0] * S
        per = [dict() for _ in range(S)]          # context -> {(g, p): [columns]}
        for cst, c, gps in sorted(slices, key=lambda t: -t[0]):
            k = min(range(S), key=lambda k: load[k])
            load[k] += cst
            for gp in gps:
                per[k].setdefault(gp, []).append(c)
        return [[[(g, p, sorted(cs)) for (g, p), cs in sorted(d.items())]] for d in per if d], n_log, mine
    S = max(1, min(S, len(units)))
    per_ctx = [units[k::S] for k in range(S)]
    bsz = wl_batch(args) if batch is None else batch
    out = []
    for us in per_ctx:
        if bsz <= 0:
            out.append([us])                  # sf1: the context's row groups in one batch
        else:
            out.append([us[i:i + bsz] for i in range(0, len(us), bsz)])
    return out, n_log, mine


class BatchInput:
    """Chunk bytes of one batch (physical units) laid out back to back, 256-B aligned, with the
    descriptors pointing into that buffer; kept in a pinned host buffer and in HBM."""

    def __init__(self, pf, units, ctx):
        from pfloor.decoder import PinnedBuffer
        items = []
        off = 0
        for _g, p, cols in units:
            for c in cols:
                s, n = pf.chunk_range(p, c)
                items.append((p, c, s, n, off))
                off += (n + 255) // 256 * 256
        self.items = items
        self.nbytes = max(off, 1)
        self.host = PinnedBuffer(ctx, self.nbytes)
        for p, c, s, n, o in items:
            if n:
                pf.read_into(s, n, self.host.ptr.value + o)
        self.descs = [pf.chunk_desc(p, c, o) for p, c, _s, _n, o in items]
        from pfloor._native import ChunkDesc
        self.arr = (ChunkDesc * max(1, len(self.descs)))(*self.descs)   # built once: the timed decodes pass it as is
        self.dev = None

    def upload(self, dec):
        from pfloor import _native
        L = _native.lib()
        d = C.c_void_p()
        _native.check(L.pf_device_alloc(dec.h, self.nbytes, C.byref(d)), dec.h, "pf_device_alloc")
        _native.check(L.pf_memcpy_h2d(dec.h, d, self.host.ptr, self.nbytes), dec.h, "h2d")
        self.dev = d

    def free(self, dec):
        from pfloor import _native
        if self.dev:
            _native.lib().pf_device_free(dec.h, self.dev)
            self.dev = None
        self.host.free()


def page_stats(descs, cols=None):
    """Algorithmic byte counts from the page headers. cols: the chunks' column
    descriptors (same order), for the per-stage counts."""
    comp = uncomp = snappy_in = snappy_out = dbp_body = dbp_out = 0
    lvl_body = count_body = 0
    pages = 0
    for ci, d in enumerate(descs):
        col = cols[ci] if cols is not None else None
        for i in range(d.n_pages):
            p = d.pages[i]
            pages += 1
            comp += p.compressed_size
            uncomp += p.uncompressed_size
            lvl = (p.rep_bytes + p.def_bytes) if p.page_type == 3 else 0
            if d.codec == 1 and (p.page_type != 3 or p.is_compressed):
                snappy_in += p.compressed_size - lvl
                snappy_out += p.uncompressed_size - lvl
            if p.encoding == 5 and p.page_type in (0, 3):   # DELTA_BINARY_PACKED data page
                dbp_body += p.uncompressed_size - lvl
                dbp_out += p.num_values * (4 if d.physical_type == 1 else 8)
            if col is not None and p.page_type in (0, 3):
                if col.max_def > 0 or p.encoding in (2, 8):
                    lvl_body += p.uncompressed_size
                if col.physical_type == 6 or col.max_rep > 0:
                    count_body += p.uncompressed_size
    return dict(pages=pages, compressed=comp, uncompressed=uncomp, snappy_in=snappy_in, snappy_out=snappy_out,
                dbp_body=dbp_body, dbp_out=dbp_out, lvl_body=lvl_body, count_body=count_body)


def stage_bytes(st, dbytes):
    """Algorithmic bytes per stage (STAGE_BYTES_DEF) of one batch."""
    return {"snappy_exec": st["snappy_in"] + st["snappy_out"], "snappy_parse": st["snappy_in"],
            "delta": st["dbp_body"] + st["dbp_out"], "levels": st["lvl_body"], "count": st["count_body"],
            "flat": st["uncompressed"] + dbytes, "decode": st["uncompressed"] + dbytes}


def chunk_decoded_bytes(col, ci):
    b = ci.num_slots * ci.width
    if col.max_def > 0:
        b += (ci.num_slots + 7) // 8
    if col.physical_type == 6:
        b += 4 * (ci.num_slots + 1) + ci.num_chars
    if col.max_rep == 1:
        b += 4 * (ci.num_rows + 1) + (ci.num_rows + 7) // 8
    if col.max_rep > 0:
        b += 2 * ci.num_entries
    return b


# --------------------------------------------------------------------------- rocprofv3 PMC child

def pmc_child(args):
    """Runs under rocprofv3 --pmc: context 0's first batch decoded alone (1 stream), 1 + 3 times.
    ctypes only (no torch), so the profiled process is the decode and nothing else."""
    from pfloor.decoder import GpuDecoder, ParquetFile
    pf = ParquetFile(input_path(args))
    plan, _, _ = units_for_rank(args, pf, 1, 0, args.streams)
    dec = GpuDecoder(0)
    bi = BatchInput(pf, plan[0][0], dec.h)
    bi.upload(dec)
    for _ in range(1 + ROOF_PASSES):
        dec.decode(bi.descs, bi.dev.value, bi.nbytes, on_device=True)
        if dec.wait() != 0 and not _SKIP:
            raise RuntimeError(dec.error())
    bi.free(dec)
    dec.close()


def measure_pmc(args, kernel_re):
    """HBM traffic of the roofline kernels per launch: one rocprofv3 pass per counter (FETCH_SIZE and
    WRITE_SIZE cannot share a pass on gfx950), FETCH_SIZE doubled (MI355X_MICROARCH.md, HBM)."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return {"error": "rocprofv3 not found"}
    out = os.path.join(args.data_dir, f"pmc_{os.getpid()}")
    res = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, cnt)
        cmd = [prof, "--pmc", cnt, "--kernel-include-regex", kernel_re, "--output-format", "csv", "-d", d, "-o", "run",
               "--", sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", args.workload,
               "--data-dir", args.data_dir, "--streams", str(args.streams), "--split", args.split, "--pool", str(args.pool),
               "--string-ctx", str(args.string_ctx), "--lpt-cost", args.lpt_cost, "--string-weight", str(args.string_weight), "--slice-mult", str(args.slice_mult)] + \
              (["--rg-batch", str(args.rg_batch)] if args.rg_batch is not None else [])
        t0 = time.time()
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=240)
        log(f"[bench] rocprofv3 --pmc {cnt}: rc {r.returncode} in {time.time() - t0:.1f}s")
        if r.returncode != 0:
            return {"error": f"rocprofv3 {cnt} rc {r.returncode}: {r.stdout.decode(errors='replace')[-400:]}"}
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            return {"error": f"no counter_collection.csv for {cnt}"}
        per_launch = []
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                per_launch.append((int(row.get("Dispatch_Id", 0) or 0), row["Kernel_Name"].split("(")[0].replace("pf::", "").replace("void ", ""),
                                   float(row["Counter_Value"]) * 1024.0))   # KB -> bytes
        res[cnt] = sorted(per_launch)
    shutil.rmtree(out, ignore_errors=True)
    return res


def pmc_traffic_per_kernel(pmc):
    """{kernel: mean bytes per decode} over the last ROOF_PASSES decodes (the first is the warm-up)."""
    out = {}
    for cnt, rows in pmc.items():
        if not isinstance(rows, list):
            continue
        by = {}
        for _i, name, v in rows:
            by.setdefault(name, []).append(v)
        for name, vals in by.items():
            # every decode launches each kernel the same number of times
            per_decode = len(vals) // (1 + ROOF_PASSES) if len(vals) >= 1 + ROOF_PASSES else 0
            if per_decode == 0:
                continue
            tail = vals[per_decode:]
            mean = sum(tail) / ROOF_PASSES
            out.setdefault(name, {})[cnt] = mean * (2.0 if cnt == "FETCH_SIZE" else 1.0)
    return {k: {"fetch_bytes_x2": round(v.get("FETCH_SIZE", 0)), "write_bytes": round(v.get("WRITE_SIZE", 0)),
                "traffic_bytes": round(v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0))} for k, v in out.items()}


# --------------------------------------------------------------------------- CPU baselines

def _host_cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))   # the GPU box's CPU share is 16 cores per GPU


def cpu_baselines(path, pf, budget_s=8.0):
    """The Java reference cannot run (no JDK / parquet-mr jars on the box). Timed instead, on the
    whole file: the C oracle (oracle/pf_oracle.c, a plain-C port of parquet-mr's decode + Snappy) at
    1 core and at all host cores, and pyarrow.parquet.read_table at the same core counts."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    lib = os.path.join(ROOT, "oracle", "libpf_oracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle_binding import Oracle
    orc = Oracle(lib)
    cores = _host_cores()
    nrg, ncol = pf.num_row_groups, pf.num_columns
    rows = pf.num_rows
    work = [(g, c) for g in range(nrg) for c in range(ncol)]
    files = [orc.open(path) for _ in range(cores)]   # one handle per thread
    dec_bytes = 0
    for g, c in work:
        r = files[0].decode(g, c)
        assert r["status"] == 0, r["error"]
        dec_bytes += sum(r[k].nbytes for k in ("values", "validity", "offsets", "chars") if k in r)
    out = []

    def oracle_pass(threads):
        idx = [0]
        lock = threading.Lock()

        def run(t):
            of = files[t]
            while True:
                with lock:
                    if idx[0] >= len(work):
                        return
                    j = idx[0]
                    idx[0] += 1
                of.decode(*work[j])
        ts = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
        [t.start() for t in ts]
        [t.join() for t in ts]

    for threads in (1, cores):
        passes, t0 = 0, time.perf_counter()
        while True:
            oracle_pass(threads)
            passes += 1
            if time.perf_counter() - t0 > budget_s or passes >= 20:
                break
        dt = time.perf_counter() - t0
        out.append({"value": round(dec_bytes * passes / dt / 1e9, 4), "unit": "decoded GB/s",
                    "rows_per_s": round(rows * passes / dt, 1), "cores": threads, "kind": "port",
                    "sample": f"whole file ({nrg} row groups x {ncol} chunks, {rows} rows), {passes} passes, "
                              f"{threads} thread(s), oracle/pf_oracle.c (C port of parquet-mr 1.12.2 + Snappy)"})
    for of in files:
        of.close()
    try:
        import pyarrow as pa
        import pyarrow.parquet as pq
        for threads in (1, cores):
            pa.set_cpu_count(threads)
            passes, t0 = 0, time.perf_counter()
            while True:
                pq.read_table(path, use_threads=threads > 1)
                passes += 1
                if time.perf_counter() - t0 > budget_s or passes >= 20:
                    break
            dt = time.perf_counter() - t0
            out.append({"value": round(dec_bytes * passes / dt / 1e9, 4), "unit": "decoded GB/s (same byte count)",
                        "rows_per_s": round(rows * passes / dt, 1), "cores": threads, "kind": "pyarrow",
                        "sample": f"pyarrow {pa.__version__} parquet.read_table of the whole file, {passes} passes, "
                                  f"{threads} thread(s) (Arrow C++ reader, not the reference)"})
    except Exception as e:   # reported, never fatal
        out.append({"kind": "pyarrow", "error": repr(e)})
    best = out[1]
    return dict(best, variants=out, note="Java reference CPU baseline unavailable (no JDK / parquet-mr jars on "
                                         "the box); the oracle port and pyarrow are timed instead")


# --------------------------------------------------------------------------- parity of the timed outputs

def check_parity(path, pf, decs, last_batches, budget_threads):
    """Bit-exact comparison of every chunk of every context's last timed batch (still resident on
    the device) with the CPU oracle; physical row groups the timed batches did not cover are decoded
    once more and compared too. Oracle decodes run in a thread pool (outside any timing)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import assert_chunk_equal
    from oracle_binding import Oracle
    orc = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
    handles = threading.local()

    def oracle_decode(key):
        if not hasattr(handles, "f"):
            handles.f = orc.open(path)
        return handles.f.decode(*key)

    todo = []
    for dec, bi in zip(decs, last_batches):
        for i, (p, c, *_r) in enumerate(bi.items):
            col = pf.columns[c]
            todo.append(((p, c), dec.fetch(i, col.physical_type, col.max_def, col.max_rep)))
    checked = {k for k, _ in todo}
    n_ok, bad = 0, []
    with cf.ThreadPoolExecutor(budget_threads) as ex:
        futs = {ex.submit(oracle_decode, k): (k, g) for k, g in todo}
        for fu in cf.as_completed(futs):
            k, g = futs[fu]
            try:
                assert g["status"] == 0, f"status {g['status']}"
                assert_chunk_equal(g, fu.result(), f"rg{k[0]} c{k[1]}")
                n_ok += 1
            except AssertionError as e:
                bad.append(str(e)[:200])
    return {"chunks": len(todo), "bit_exact": not bad and n_ok == len(todo), "row_groups": sorted({k[0] for k in checked}),
            "mismatches": bad[:5], "against": "oracle/pf_oracle.c (CPU restatement, pinned to pyarrow golden vectors)"}


# --------------------------------------------------------------------------- main

def spawn_ranks(args, argv):
    """--gpus N without a launcher: start N ranks as child processes (no GPU call happens here)."""
    make_input(args)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


class ContextPool:
    """One persistent host thread per decode stream (ctypes releases the GIL, so the host-side
    planning of one stream overlaps the GPU work of the others). The threads are started once and
    parked on a condition between runs, so run(k) costs no thread start / join: it hands every
    stream "decode your batches k times in order" and returns when all are done.

    pipelined=True (the timed steps): each stream has two contexts sharing its HIP stream
    (pf_ctx_create_shared); batch i+1 is planned and enqueued on one while batch i still decodes on
    the other, then batch i is waited for — the way a reader prefetches the next row group, so the
    host planning (~0.3 ms per batch) is off the stream's critical path. Stage timing is off
    (its events are markers between kernels). pipelined=False: decode -> pf_wait per batch on the
    first context, stage events on; context 0's per-stage HIP-event times are accumulated."""

    def __init__(self, decs, batches, on_device=True, twins=None):
        self.decs, self.batches, self.on_device = decs, batches, on_device
        self.twins = twins
        self.last = list(decs)           # per stream: the context holding its last decoded batch
        self.stage_acc, self.host_s, self.host_calls = {}, 0.0, 0
        self._lock = threading.Lock()
        self._cv = threading.Condition()
        self._gen, self._job, self._done, self._errs, self._stop = 0, None, 0, [], False
        self._threads = [threading.Thread(target=self._loop, args=(i,), daemon=True) for i in range(len(decs))]
        for t in self._threads:
            t.start()

    def _decode(self, d, bi):
        t0 = time.perf_counter()
        d.decode(bi.arr, (bi.dev if self.on_device else bi.host.ptr).value, bi.nbytes, on_device=self.on_device)
        t1 = time.perf_counter()
        with self._lock:
            self.host_s += t1 - t0
            self.host_calls += 1

    @staticmethod
    def _wait(d):
        # PF_DEBUG_SKIP (stage ablation, pf_runtime.hip): skipped stages leave chunks failed by design
        if d.wait() != 0 and not _SKIP:
            raise RuntimeError(d.error())

    def _work(self, i, passes, pipelined):
        d, bl = self.decs[i], self.batches[i]
        if pipelined:
            pair = (d, self.twins[i])
            seq = [bi for _ in range(passes) for bi in bl]
            for k, bi in enumerate(seq):
                self._decode(pair[k % 2], bi)
                if k > 0:
                    self._wait(pair[(k - 1) % 2])
            if seq:
                self._wait(pair[(len(seq) - 1) % 2])
                self.last[i] = pair[(len(seq) - 1) % 2]
            return
        for _ in range(passes):
            for bi in bl:
                self._decode(d, bi)
                self._wait(d)
                if i == 0:
                    for k, v in d.timing().items():
                        self.stage_acc[k] = self.stage_acc.get(k, 0.0) + v
        self.last[i] = d

    def _loop(self, i):
        seen = 0
        while True:
            with self._cv:
                self._cv.wait_for(lambda: self._stop or self._gen != seen)
                if self._stop:
                    return
                seen, job = self._gen, self._job
            try:
                self._work(i, *job)
            except Exception as e:
                self._errs.append(e)
            with self._cv:
                self._done += 1
                self._cv.notify_all()

    def set_timing(self, on):
        for d in self.decs + (self.twins or []):
            d.set_timing(on)

    def run(self, passes, pipelined=False):
        self.set_timing(not pipelined)
        with self._cv:
            self._errs, self._done, self._job = [], 0, (passes, pipelined)
            self._gen += 1
            self._cv.notify_all()
            self._cv.wait_for(lambda: self._done == len(self._threads))
        if self._errs:
            raise self._errs[0]

    def warm(self, passes, min_s, pipelined=True):
        """Untimed warmup: `passes` passes, then more until at least min_s seconds of identical work
        have run (clocks and caches settle; a 5-pass warmup is ~16 ms). Returns the passes run."""
        t0 = time.perf_counter()
        n = 0
        if passes > 0:
            self.run(passes, pipelined)
            n = passes
        while time.perf_counter() - t0 < min_s:
            k = max(1, n)   # doubling chunks: few run() calls
            self.run(k, pipelined)
            n += k
        return n

    def reset(self):
        self.stage_acc, self.host_s, self.host_calls = {}, 0.0, 0

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for t in self._threads:
            t.join()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)   # ~1.2 s timed: long enough for an SMI sampler to see the GPU busy
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-s", type=float, default=0.3,
                    help="untimed warmup runs at least --warmup passes and at least this many seconds of them")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="sf1")
    ap.add_argument("--data-dir", default=os.environ.get("PF_BENCH_DIR", "/tmp/pfloor_bench"))
    ap.add_argument("--streams", type=int, default=4,
                    help="decode contexts (HIP streams) per GPU; work units are dealt round-robin to them")
    ap.add_argument("--rg-batch", type=int, default=None,
                    help="row groups per decode batch (default: the workload's; 0 = each context decodes a few columns over all row groups)")
    ap.add_argument("--split", choices=("columns", "kinds", "rowgroups"), default="columns",
                    help="sf1: give each context all row groups of a column subset (default), the same with "
                         "BYTE_ARRAY and fixed-width columns on separate contexts (kinds), or whole row groups")
    ap.add_argument("--string-ctx", type=int, default=2, help="--split kinds: contexts for the BYTE_ARRAY columns")
    ap.add_argument("--string-weight", type=float, default=None,
                    help="--split columns: LPT cost multiplier of BYTE_ARRAY chunks (their value walk, chars count and "
                         "copy); default: the workload's (flat 4, others 1)")
    ap.add_argument("--wide-groups", type=int, default=None, help=argparse.SUPPRESS)   # analysis: wide column batches per stream
    ap.add_argument("--row-cost", type=float, default=None, help=argparse.SUPPRESS)   # analysis: LPT bytes per row of a chunk
    ap.add_argument("--slice-mult", type=int, default=None,
                    help="--split columns: row-group slices per column x this (default: the workload's; sf1 2, others 1)")
    ap.add_argument("--lpt-cost", choices=("decompressed", "compressed"), default="compressed",
                    help="sf1 --split columns: the per-chunk cost the column slices are dealt by")
    ap.add_argument("--columns", default=None, help=argparse.SUPPRESS)   # analysis only: comma-separated column subset
    ap.add_argument("--pool", type=int, default=100000,
                    help="wide: distinct values per column (SURVEY 8(d) sweep: 1K, 16K, 32K, 64K, 100K)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-write", action="store_true", help="skip the write-path leg")
    ap.add_argument("--e2e-split", type=int, default=1, help="E2E: batches per row group (column subsets)")
    ap.add_argument("--e2e-streams", type=int, default=2,
                    help="E2E: decode streams (each with its twin context and the library's copy stream: the "
                         "box has 4 hardware queues)")
    ap.add_argument("--e2e-last", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e-rg-batch", type=int, default=0,
                    help="E2E: row groups per decode batch (batches alternate between a stream's twin contexts)")
    ap.add_argument("--e2e-copy", choices=("batch", "chunks"), default="batch",
                    help="E2E D2H: one copy per output arena (batch) or per chunk array (chunks)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="timed steps decode -> wait per batch on one context per stream (A/B of the pipelined default)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args, _ = ap.parse_known_args()
    if args.string_weight is None:
        args.string_weight = WORKLOADS[args.workload].get("string_weight", 1.0)
    if args.slice_mult is None:
        args.slice_mult = WORKLOADS[args.workload].get("slice_mult", 1)
    if args.pmc_child:
        return pmc_child(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args, sys.argv[1:])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)   # barriers + max-over-ranks time only
    if rank == 0:
        make_input(args)
    if dist:
        dist.barrier()
    path = input_path(args)

    # HBM traffic of the roofline kernels: rocprofv3 child processes, before this process touches the GPU
    pmc = None
    # never start rocprofv3 from a process that is itself being profiled: the profiler's preload has
    # already initialised the GPU here, and a GPU-initialised process must not exec another program
    profiled = any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", "")
    if profiled:
        pmc = {"error": "skipped: bench.py is running under a profiler"}
    elif world == 1 and not args.no_pmc:
        try:
            pmc = measure_pmc(args, "k_snappy|k_flat|k_decode|k_delta|k_dbp|k_count|k_runs|k_lvl|k_dlen|k_nest|k_ba_|k_scan|k_dba")
        except Exception as e:
            pmc = {"error": repr(e)}

    import torch
    from pfloor import _native
    from pfloor.decoder import GpuDecoder, ParquetFile

    device = local_rank
    torch.cuda.set_device(device)
    pf = ParquetFile(path)
    plan, n_log, mine = units_for_rank(args, pf, world, rank, args.streams)
    S = len(plan)
    decs = [GpuDecoder(device) for _ in range(S)]
    twins = [GpuDecoder(share=d) for d in decs]   # second context per stream (pipelined steps)
    # batch inputs, cached by physical content (sf100 replicas share one device copy)
    cache = {}
    batches = []
    for k, bl in enumerate(plan):
        row = []
        for units in bl:
            key = tuple((p, tuple(cols)) for _g, p, cols in units)
            if key not in cache:
                bi = BatchInput(pf, units, decs[0].h)
                bi.upload(decs[0])
                cache[key] = bi
            row.append(cache[key])
        batches.append(row)
    _native.check(_native.lib().pf_sync(decs[0].h), decs[0].h, "pf_sync")   # uploads done before any context reads them

    pool = ContextPool(decs, batches, True, twins)
    t_w = time.perf_counter()
    warm_passes = pool.warm(args.warmup, args.warmup_s, pipelined=not args.no_pipeline)
    warm_s = time.perf_counter() - t_w
    # decoded bytes of one step (every batch's result is identical each step)
    dbytes = 0
    for d, bl in zip(decs, batches):
        for bi in bl:
            d.decode(bi.descs, bi.dev.value, bi.nbytes, on_device=True)
            if d.wait() != 0 and not _SKIP:
                raise RuntimeError(d.error())
            for i, (p, c, *_r) in enumerate(bi.items):
                dbytes += chunk_decoded_bytes(pf.columns[c], d.info(i))
    rows = sum(pf.row_group_rows(g % pf.num_row_groups) for g in mine) if args.workload != "wide" else \
        pf.row_group_rows(0)
    pool.reset()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    pool.run(args.steps, pipelined=not args.no_pipeline)   # K passes over the rank's share; streams run independently
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    host_plan_ms = pool.host_s / max(1, pool.host_calls) * 1e3
    timed_last = list(pool.last)
    tot = np.array([dbytes, rows], dtype=np.float64)
    if dist:
        import torch as _t
        t = _t.tensor([dt], dtype=_t.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tt = _t.tensor(tot)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        tot = tt.numpy()
    n_b0 = max(1, len(batches[0]))
    ms_per_step = dt / args.steps * 1e3
    value = float(tot[0]) * args.steps / dt / 1e9

    # ---- parity of the timed outputs (each context's last batch is still resident) ----
    parity = None
    if not args.no_parity:
        t1 = time.time()
        try:
            parity = check_parity(path, pf, timed_last, [bl[-1] for bl in batches], _host_cores())
        except Exception as e:
            parity = {"bit_exact": False, "error": repr(e)}
        log(f"[bench] parity {parity.get('chunks')} chunks bit_exact={parity.get('bit_exact')} in {time.time() - t1:.1f}s")

    # ---- per-stage times: separate untimed passes, all streams decoding, stage events on ----
    pool.reset()
    stage_passes = min(args.steps, 10)
    pool.run(stage_passes, pipelined=False)
    stage_ms = {k: v / (stage_passes * n_b0) for k, v in pool.stage_acc.items()}

    # ---- roofline of the dominant stage: context 0's first batch decoded alone ----
    b0 = batches[0][0]
    st0 = page_stats(b0.descs, [pf.columns[c] for (_p, c, *_r) in b0.items])
    dbytes0 = 0
    iso = {}
    dec = decs[0]
    for r in range(ROOF_PASSES):
        dec.decode(b0.descs, b0.dev.value, b0.nbytes, on_device=True)
        if dec.wait() != 0 and not _SKIP:
            raise RuntimeError(dec.error())
        for k, v in dec.timing().items():
            iso[k] = iso.get(k, 0.0) + v / ROOF_PASSES
    for i, (p, c, *_r) in enumerate(b0.items):
        dbytes0 += chunk_decoded_bytes(pf.columns[c], dec.info(i))
    kern_bytes = stage_bytes(st0, dbytes0)
    dom = max((k for k in iso if k in kern_bytes), key=lambda k: iso.get(k, 0.0))
    dom_ms = iso.get(dom, 0.0)
    dom_bytes = kern_bytes[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else None
    traffic, traffic_detail, traffic_names = None, None, None
    if pmc and "error" not in pmc:
        traffic_detail = pmc_traffic_per_kernel(pmc)
        names = [n for n in traffic_detail if STAGE_KERNELS.get(dom) and re.match(STAGE_KERNELS[dom], n.split("<")[0])]
        if names:
            traffic = sum(traffic_detail[n]["traffic_bytes"] for n in names)
            traffic_names = sorted(names)
    b_alg_step = None
    descs_all = [d for bl in batches for bi in bl for d in bi.descs]
    st_all = page_stats(descs_all)
    b_alg_step = st_all["compressed"] + dbytes

    # ---- end to end: pinned host input -> H2D -> decode -> D2H into pinned host columns ----
    e2e = None
    if not args.no_e2e:
        try:
            # whole row groups dealt round-robin to the contexts (one context's H2D, another's
            # kernels and a third's D2H overlap; the link is full duplex). Measured: 37-39 GB/s with
            # this plan, 35 with one row group per batch, 26 with the column split.
            e2e_plan, _, _ = units_for_rank(argparse.Namespace(**{**vars(args), "split": "rowgroups"}), pf, world, rank,
                                            min(args.e2e_streams, len(decs)), batch=args.e2e_rg_batch)
            if args.e2e_split > 1:   # each row group's columns in e2e_split batches (earlier first D2H)
                k = args.e2e_split
                e2e_plan = [[[(g, p, cs[i::k]) for g, p, cs in units] for units in bl for i in range(k)]
                            for bl in e2e_plan]
            e2e_batches = [[BatchInput(pf, units, decs[0].h) for units in bl] for bl in e2e_plan]
            # --e2e-last: the last contexts instead of the first (analysis: which hardware queues the library's
            # copy streams share with the decode streams)
            ke = len(e2e_batches)
            sel = slice(-ke, None) if args.e2e_last else slice(0, ke)
            e2e = measure_e2e(decs[sel], e2e_batches, pf, st_all, args.e2e_copy,
                              barrier=dist.barrier if dist else None, twins=twins[sel])
            for bl in e2e_batches:
                for bi in bl:
                    bi.host.free()
        except Exception as e:
            e2e = {"error": repr(e)}
        if dist:   # node E2E: bytes of all ranks / slowest rank's pass (barrier-aligned passes)
            import torch as _t
            ok = e2e is not None and "ms_per_pass" in e2e
            v = _t.tensor([e2e["ms_per_pass"] if ok else 0.0, e2e["decoded_bytes"] if ok else 0.0, 1.0 if ok else 0.0],
                          dtype=_t.float64)
            mx = v.clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(v, op=dist.ReduceOp.SUM)
            if ok and int(v[2].item()) == world:
                e2e["node"] = {"value": round(float(v[1].item()) / (float(mx[0].item()) * 1e-3) / 1e9, 3),
                               "unit": "decoded GB/s, all ranks (sum of decoded bytes / max pass time)",
                               "n_gpus": world, "ms_per_pass_max": round(float(mx[0].item()), 3),
                               "pcie_bound_gbs_node": PCIE_GBS * world}

    # ---- write path: row group 0 re-encoded on the GPU and read back ----
    write = None
    if not args.no_write and rank == 0:
        try:
            for d in decs:
                d.set_timing(True)
            write = measure_write(path, pf, decs[0], decs=decs)
        except Exception as e:
            write = {"error": repr(e)}

    w = WORKLOADS[args.workload]
    if args.workload == "sf1":
        wl = (f"lineitem SF1 x{world} ({w['rows']} rows x {world}, 16 cols, {pf.num_row_groups * world} row groups of 1Mi rows), "
              "Snappy + dictionary, device-resident")
        scaling = "weak"
    elif args.workload == "sf100":
        wl = (f"lineitem SF100-shaped ({n_log} row groups of {w['rg_rows']} rows = {n_log * w['rg_rows']} rows; the "
              f"{pf.num_row_groups} distinct synthetic row groups stand for the {n_log}), Snappy + dictionary, device-resident")
        scaling = "strong"
    elif args.workload == "nested":
        wl = (f"nested: {w['rows']} rows of l optional LIST<STRUCT<a INT64 DELTA_BINARY_PACKED, b UTF8 dictionary>> "
              f"(lengths 0-4, 10% null lists, 5% null elements / leaves), v2 pages, Snappy, {pf.num_row_groups} row groups, "
              "device-resident")
        scaling = "strong"
    elif args.workload == "flat":
        wl = (f"flat: {w['rows']} rows (id INT64, x DOUBLE, n nullable INT32, s dictionary UTF8), uncompressed, "
              f"{pf.num_row_groups} row groups, device-resident")
        scaling = "strong"
    else:
        wl = (f"wide: {w['rows']} rows x {pf.num_columns} nullable INT32/FLOAT columns, 30% nulls, {args.pool}-value dictionaries, "
              "Snappy, device-resident")
        scaling = "strong"
    step_frac = round(b_alg_step / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
    out = {
        "metric": METRIC,
        "value": round(value, 3), "unit": "decoded GB/s",
        # headline efficiency: the whole step's algorithmic HBM bytes / step time /
        # HBM peak, with the dominant kernel's own fraction beside it (details: pipeline_roofline, roofline)
        "step_frac": step_frac,
        "dominant_kernel_frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
        "rows_per_s": round(float(tot[1]) * args.steps / dt, 1),
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "warmup_policy": {"passes_run": warm_passes, "seconds": round(warm_s, 3),
                          "rule": f"max(--warmup passes, passes filling {args.warmup_s} s), untimed, same work as a step"},
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": "u8", "data": f"synthetic (pyarrow-written {w['kind']}-shaped file, seed {w['seed']})",
        "config": {"workload": wl, "rows_per_step": int(tot[1]),
                   "row_groups_per_rank": len(mine), "decoded_bytes_per_step": int(tot[0]),
                   "compressed_page_bytes_rank0": st_all["compressed"],
                   "parallelism": f"row groups sharded round-robin over {world} GPU(s) (pfloor.shard, no collective), "
                                  f"{S} decode streams per GPU" +
                                  (f", each stream a column subset (column slices dealt LPT on {args.lpt_cost} bytes"
                                   + (f", BYTE_ARRAY chunks weighted x{args.string_weight:g}" if args.string_weight != 1.0 else "")
                                   + (f", x{args.slice_mult} row-group slices per column" if args.slice_mult != 1 else "")
                                   + ")" if args.split == "columns" and S > 1 and wl_batch(args) <= 0 else "")},
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "stage_ms_source": "context 0's per-stage HIP events, separate untimed passes (all streams decoding, "
                           "not pipelined); the timed steps run with the events off",
        "pipelined": not args.no_pipeline,
        "host_enqueue_ms_per_batch": round(host_plan_ms, 4),
        "roofline": {"bound": "hbm", "kernel": STAGE_LABEL.get(dom, dom), "achieved": round(achieved, 2) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None, "traffic": traffic,
                     "traffic_source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch, measured in "
                                       "this run (child processes, same batch, 1 stream)" if traffic else
                                       (pmc or {}).get("error"),
                     "algorithmic_bytes_per_launch": dom_bytes, "algorithmic_bytes_def": STAGE_BYTES_DEF.get(dom),
                     "traffic_kernels": traffic_names, "launch_ms": round(dom_ms, 4),
                     "launch_ms_source": f"HIP events on context 0's stream, its first batch decoded alone x{ROOF_PASSES} "
                                         "after the timed region",
                     "stage_ms_overlapped": round(stage_ms.get(dom, 0.0), 4)},
        "pipeline_roofline": {"b_alg_per_step_rank0": b_alg_step, "ms_per_step": round(ms_per_step, 4),
                              "achieved": round(b_alg_step / (ms_per_step * 1e-3) / 1e9, 2),
                              "frac": step_frac},
    }
    if traffic_detail:
        out["pmc_traffic_per_launch"] = traffic_detail
    if parity is not None:
        out["parity"] = parity
    if e2e is not None:
        out["e2e"] = e2e
    if write is not None:
        out["write"] = write
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baselines(path, pf)
        except Exception as e:   # reported, never fatal
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    pool.close()
    for bi in cache.values():
        bi.free(decs[0])
    for d in twins + decs:
        d.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if parity is not None and not parity.get("bit_exact"):
        log("[bench] PARITY FAILURE")
        return 3
    return 0


def measure_write(path, pf, dec, passes=3, decs=None):
    """Write path (ParquetWriter.java:61-165 settings): row group 0 of the input, decoded on the
    GPU to host columns, is written WRITE passes times as a one-row-group file by pfloor.writer
    (per column: H2D, dictionary encode, pages, Snappy on the GPU, headers + file on the host);
    the best pass is reported as input bytes / wall time. The last file is then decoded on the GPU
    and compared bit-exactly with the source columns."""
    import tempfile
    from pfloor import writer as W
    from pfloor.decoder import decode_file
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import assert_chunk_equal
    src = decode_file(path, row_groups=[0], decoder=dec)
    if src["_status"] != 0:
        raise RuntimeError(src["_error"])
    n = pf.row_group_rows(0)
    fields, cols, in_bytes = [], {}, 0
    dt = {1: np.int32, 2: np.int64, 4: np.float32, 5: np.float64, 0: np.uint8}
    for c, col in enumerate(pf.columns):
        g = src[(0, c)]
        name = ".".join(col.path)
        f = W.Field(name, col.physical_type, col.max_def > 0, col.physical_type == 6)
        fields.append(f)
        if col.physical_type == 6:
            d = (g["offsets"], g["chars"])
            in_bytes += g["offsets"].nbytes + g["chars"].nbytes
        else:
            d = g["values"].view(dt[col.physical_type])
            in_bytes += d.nbytes
        if col.max_def > 0:
            d = (*d, g["validity"]) if isinstance(d, tuple) else (d, g["validity"])
            in_bytes += g["validity"].nbytes
        cols[name] = d
    schema = W.MessageType("lineitem", *fields)
    out_path = os.path.join(tempfile.gettempdir(), f"pfloor_write_{os.getpid()}.parquet")
    times, encs, kms = [], None, None
    for _ in range(passes):
        t0 = time.perf_counter()
        wr = W.ParquetWriter(schema, out_path, None, decoder=None if decs else dec, decoders=decs)
        wr.write_columns(cols, n)
        wr.close()
        times.append(time.perf_counter() - t0)
        encs = list(wr.last_chunks)
        kms = dict(wr.kernel_ms)
    size = os.path.getsize(out_path)
    back = decode_file(out_path, decoder=dec)
    bad = []
    for c in range(len(fields)):
        try:
            assert_chunk_equal(back[(0, c)], src[(0, c)], f"write c{c}")
        except AssertionError as e:
            bad.append(str(e)[:160])
    os.remove(out_path)
    best = min(times)
    return {"value": round(in_bytes / best / 1e9, 3), "unit": "GB/s of column bytes in (host) -> Parquet file",
            "ms_per_row_group": round(best * 1e3, 2), "rows": n, "columns": len(fields), "input_bytes": in_bytes,
            "file_bytes": size, "dictionary_columns": sum(1 for e in encs if e[1] == 8),
            "plain_fallbacks": sum(1 for e in encs if e[2] in (1, 2)),
            "parity": {"chunks": len(fields), "bit_exact": not bad, "mismatches": bad[:3],
                       "against": "the source columns, read back by the GPU read path"},
            "contexts": len(decs) if decs else 1,
            "roofline": {"bound": "hbm", "kernel": "k_snappy_compress (all 16 columns' launches, summed)",
                         "algorithmic_bytes": kms["snappy_in"] + kms["snappy_out"], "kernel_ms": round(kms["snappy"], 3),
                         "achieved": round((kms["snappy_in"] + kms["snappy_out"]) / (kms["snappy"] * 1e-3) / 1e9, 2)
                         if kms["snappy"] > 0 else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round((kms["snappy_in"] + kms["snappy_out"]) / (kms["snappy"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                         if kms["snappy"] > 0 else None,
                         "source": "HIP events around each k_snappy_compress launch (pf_encoded_chunk.snappy_ms), "
                                   "launches on up to 4 streams may overlap"},
            "encode_kernels_ms": round(kms["encode"], 3),
            "passes": passes}


def measure_e2e(decs, batches, pf, st_all, copy_mode="batch", barrier=None, twins=None):
    """Whole rank share, E2E_PASSES times: per context, per batch: pinned H2D of the batch's chunk
    bytes (inside pf_decode_row_group), decode, pf_wait, then the D2H of the decoded columns into
    pinned host memory — copy_mode "batch": pf_copy_batch_async, one copy per output arena (3 per
    batch); "chunks": pf_copy_columns_async, one copy per array of every chunk (up to 8 per chunk).
    The next batch on that context is ordered after those copies."""
    from pfloor import _native
    from pfloor.decoder import PinnedBuffer
    from pfloor._native import ColumnOut
    L = _native.lib()
    # output layout per batch from one decode (sizes are the same every pass)
    layouts = []
    d2h = 0
    for d, bl in zip(decs, batches):
        row = []
        for bi in bl:
            d.decode(bi.descs, bi.host.ptr.value, bi.nbytes, on_device=False)
            if d.wait() != 0 and not _SKIP:
                raise RuntimeError(d.error())
            infos = [d.info(i) for i in range(len(bi.items))]
            row.append(infos)
        layouts.append(row)
    if copy_mode == "batch":
        return _e2e_batch(decs, batches, layouts, pf, barrier, twins)
    # pinned output buffers: one per context, sized for its largest batch
    outs = []
    for ctx_i, (d, bl) in enumerate(zip(decs, batches)):
        per_batch = []
        need_max = 0
        for bj, bi in enumerate(bl):
            fields = []
            off = 0
            for i, (p, c, *_r) in enumerate(bi.items):
                ci = layouts[ctx_i][bj][i]
                col = pf.columns[c]
                f = {}

                def take(name, n):
                    nonlocal off
                    f[name] = (off, n)
                    off += (n + 255) // 256 * 256
                if col.physical_type == 6:
                    take("offsets", 4 * (ci.num_slots + 1))
                    take("chars", ci.num_chars)
                else:
                    take("values", ci.num_slots * ci.width)
                if col.max_def > 0:
                    take("validity", (ci.num_slots + 7) // 8)
                if col.max_rep == 1:
                    take("list_offsets", 4 * (ci.num_rows + 1))
                    take("list_validity", (ci.num_rows + 7) // 8)
                if col.max_rep > 0:
                    take("def_levels", ci.num_entries)
                    take("rep_levels", ci.num_entries)
                fields.append(f)
            per_batch.append(fields)
            need_max = max(need_max, off)
        buf = PinnedBuffer(d.h, need_max)
        arrs = []
        for fields in per_batch:
            arr = (ColumnOut * max(1, len(fields)))()
            for i, f in enumerate(fields):
                for name, (o, n) in f.items():
                    setattr(arr[i], name, buf.ptr.value + o if n else None)
                    setattr(arr[i], name + "_cap", n)
                    d2h += n
            idx = (C.c_int * max(1, len(fields)))(*range(len(fields)))
            arrs.append((arr, idx, len(fields)))
        outs.append((buf, arrs))
    d2h_per_pass = d2h
    h2d_per_pass = sum(bi.nbytes for bl in batches for bi in bl)
    errs = []

    def worker(ci, d, bl):
        try:
            for bj, bi in enumerate(bl):
                d.decode(bi.descs, bi.host.ptr.value, bi.nbytes, on_device=False)
                if d.wait() != 0 and not _SKIP:
                    raise RuntimeError(d.error())
                arr, idx, n = outs[ci][1][bj]
                _native.check(L.pf_copy_columns_async(d.h, n, idx, arr), d.h, "pf_copy_columns_async")
            _native.check(L.pf_sync(d.h), d.h, "pf_sync")
        except Exception as e:
            errs.append(e)

    def one_pass():
        ts = [threading.Thread(target=worker, args=(i, d, bl)) for i, (d, bl) in enumerate(zip(decs, batches))]
        [t.start() for t in ts]
        [t.join() for t in ts]
        if errs:
            raise errs[0]
    one_pass()   # warm-up (first touch of the pinned outputs)
    t0 = time.perf_counter()
    for _ in range(E2E_PASSES):
        one_pass()
    dt = (time.perf_counter() - t0) / E2E_PASSES
    for buf, _ in outs:
        buf.free()
    decoded = d2h_per_pass
    t_link = max(h2d_per_pass, d2h_per_pass) / (PCIE_GBS * 1e9)
    return {"value": round(decoded / dt / 1e9, 3), "unit": "decoded GB/s (pinned host in -> host columns out)",
            "ms_per_pass": round(dt * 1e3, 3), "h2d_bytes": h2d_per_pass, "d2h_bytes": d2h_per_pass,
            "pcie_bound_gbs": PCIE_GBS, "frac": round(t_link / dt, 4),
            "frac_definition": "max(H2D, D2H bytes) / 63 GB/s divided by the measured pass time",
            "passes": E2E_PASSES, "d2h_copies": "per chunk array (pf_copy_columns_async)"}


def measure_link(nbytes, reps=3):
    """Raw PCIe rates on this box: one pinned-host <-> HBM copy of nbytes each way (torch), best of reps."""
    try:
        import torch
        n = int(nbytes)
        dev = torch.empty(n, dtype=torch.uint8, device="cuda")
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        out = {}
        for name, dst, src in (("d2h_gbs", host, dev), ("h2d_gbs", dev, host)):
            best = None
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dst.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
                t = time.perf_counter() - t0
                best = t if best is None else min(best, t)
            out[name] = round(n / best / 1e9, 2)
        out["bytes"] = n
        del dev, host
        return out
    except Exception as e:
        return {"error": repr(e)}


def _e2e_batch(decs, batches, layouts, pf, barrier=None, twins=None):
    """measure_e2e with pf_copy_batch_async: per stream, batches alternate between the context and its
    twin (own arenas, own pinned output buffer sized for the stream's largest batch), so batch j's
    download (the library's copy stream) runs under batch j + 1's H2D and kernels.
    barrier (N > 1): aligns the ranks' timed passes, so the node rate is sum(bytes) / max(time)."""
    from pfloor import _native
    from pfloor.decoder import PinnedBuffer
    L = _native.lib()
    d2h_arrays = 0
    for row, bl in zip(layouts, batches):
        for infos, bi in zip(row, bl):
            for ci, (p, c, *_r) in zip(infos, bi.items):
                d2h_arrays += chunk_decoded_bytes(pf.columns[c], ci)
    bufs, copied = [], 0
    for d, bl in zip(decs, batches):
        need = 0
        for bi in bl:   # batch sizes from one decode of each batch
            d.decode(bi.descs, bi.host.ptr.value, bi.nbytes, on_device=False)
            if d.wait() != 0 and not _SKIP:
                raise RuntimeError(d.error())
            n = C.c_size_t()
            _native.check(L.pf_batch_bytes(d.h, C.byref(n)), d.h, "pf_batch_bytes")
            need = max(need, n.value)
            copied += n.value
        bufs.append([PinnedBuffer(d.h, max(need, 1)) for _ in range(2 if twins else 1)])
    h2d_per_pass = sum(bi.nbytes for bl in batches for bi in bl)
    errs = []

    def worker(ci, d, bl, passes=1):
        try:
            pair = (d, twins[ci]) if twins else (d,)
            for j, bi in enumerate(list(bl) * passes):
                dj, buf = pair[j % len(pair)], bufs[ci][j % len(pair)]
                dj.decode(bi.descs, bi.host.ptr.value, bi.nbytes, on_device=False)
                if dj.wait() != 0 and not _SKIP:
                    raise RuntimeError(dj.error())
                _native.check(L.pf_copy_batch_async(dj.h, buf.ptr, buf.nbytes), dj.h, "pf_copy_batch_async")
            for dj in pair:
                _native.check(L.pf_sync(dj.h), dj.h, "pf_sync")
        except Exception as e:
            errs.append(e)

    def one_pass(passes=1):
        ts = [threading.Thread(target=worker, args=(i, d, bl, passes)) for i, (d, bl) in enumerate(zip(decs, batches))]
        [t.start() for t in ts]
        [t.join() for t in ts]
        if errs:
            raise errs[0]
    one_pass()
    if barrier:
        barrier()
    t0 = time.perf_counter()
    for _ in range(E2E_PASSES):
        one_pass()
    if barrier:
        barrier()
    dt_file = (time.perf_counter() - t0) / E2E_PASSES
    # streamed: the passes back to back in each stream's worker (no join between files), so one file's
    # first H2D and decode run under the previous file's last downloads
    t0 = time.perf_counter()
    one_pass(E2E_STREAM_PASSES)
    if barrier:
        barrier()
    dt = (time.perf_counter() - t0) / E2E_STREAM_PASSES
    for bb in bufs:
        for b in bb:
            b.free()
    t_link = max(h2d_per_pass, copied) / (PCIE_GBS * 1e9)
    link = measure_link(copied)
    return {"value": round(d2h_arrays / dt / 1e9, 3), "unit": "decoded GB/s (pinned host in -> host columns out)",
            "link_measured": link, "frac_of_measured_d2h": round(copied / link["d2h_gbs"] / 1e9 / dt, 4) if "d2h_gbs" in link else None,
            "ms_per_pass": round(dt * 1e3, 3), "streamed_passes": E2E_STREAM_PASSES,
            "file": {"ms_per_pass": round(dt_file * 1e3, 3), "value": round(d2h_arrays / dt_file / 1e9, 3),
                     "what": "one file per pass, the streams joined at its end (pipeline fill and drain in every pass)"},
            "h2d_bytes": h2d_per_pass, "d2h_bytes": copied,
            "decoded_bytes": d2h_arrays, "pcie_bound_gbs": PCIE_GBS, "frac": round(t_link / dt, 4),
            "frac_definition": "max(H2D, D2H bytes) / 63 GB/s divided by the measured pass time",
            "passes": E2E_PASSES, "streams": len(decs), "twins": bool(twins),
            "d2h_copies": "one per batch (pf_copy_batch_async: k_download writes the pinned pages on the library's copy stream)"}


if __name__ == "__main__":
    sys.exit(main() or 0)
