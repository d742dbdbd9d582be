"""Diagnostic: compare the GPU Snappy index tables (windows, lane outs, token bitmap, 64 KiB
splits) of one stream against the true token chain computed on the host."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from oracle_binding import Oracle  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor.decoder import GpuDecoder  # noqa: E402
from snappy_stats import tokens  # noqa: E402
import test_gpu_snappy as T  # noqa: E402


def main():
    seed, name = int(sys.argv[1]), sys.argv[2]
    o = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
    comp = None
    if name.startswith("page:"):   # page:<column>:<page index> of a lineitem-shaped file (seed = rows)
        import pyarrow.parquet as pq
        from pfloor import datagen
        from pfloor.decoder import ParquetFile
        _, col, pidx = name.split(":")
        path = f"/tmp/probe_lineitem_{seed}.parquet"
        if not os.path.exists(path):
            pq.write_table(datagen.lineitem_table(seed, seed=42), path, compression="snappy", row_group_size=1 << 20)
        with ParquetFile(path) as pf:
            c = [i for i, cc in enumerate(pf.columns) if cc.path[0] == col][0]
            st, nn = pf.chunk_range(0, c)
            buf = np.zeros(nn, np.uint8)
            pf.read_into(st, nn, buf.ctypes.data)
            d = pf.chunk_desc(0, c, 0)
            pg = d.pages[int(pidx)]
            comp = buf[pg.offset:pg.offset + pg.compressed_size].tobytes()
        data = o.snappy_uncompress(comp)
    elif name.startswith("boundary"):
        data = dict(T._boundary_streams(seed))[int(name.split(":")[1])]
    else:
        data = T._payloads(np.random.default_rng(seed))[name]
    if comp is None:
        comp = o.snappy_compress(data, mode=0)
    dec = GpuDecoder(0)
    L = _native.lib()
    trace = getattr(L, "pf_debug_trace", None) if os.environ.get("PFLOOR_LIB_PATH") else None
    tbuf = np.zeros(8192, np.uint32)
    if trace:
        trace.argtypes = [C.c_void_p, C.c_int, C.c_int]
    for rep in range(20):
        if trace:
            trace(tbuf.ctypes.data, 8192, 1)
        got, fb = dec.snappy_decompress(comp)
        if got != data:
            break
    if trace:
        trace(tbuf.ctypes.data, 8192, 0)
        i, lines = 0, 0
        while i < 8192 and tbuf[i] and lines < 400:
            t = int(tbuf[i]) >> 16
            w = {0xAAAA: 5, 0xBBBB: 8, 0xCCCC: 5, 0xDDDD: 5, 0xEEEE: 6, 0xFFFF: 5, 0x9999: 5}.get(t, 1)
            print("trace", hex(int(tbuf[i])), list(map(int, tbuf[i + 1:i + w])))
            i += w; lines += 1
    print("failing rep", rep)
    n, ulen = len(comp), len(data)
    print("got == data:", got == data)
    nw, npc = max(1, -(-n // 8192)), max(1, -(-ulen // 65536))
    f = L.pf_debug_snappy_tables
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    sp = np.zeros(npc, np.uint32); wn = np.zeros((nw, 4), np.uint32); lo = np.zeros((nw, 64), np.uint32)
    tm = np.zeros(nw * 256, np.uint32)
    assert f(dec.h, sp.ctypes.data, npc, wn.ctypes.data, nw, lo.ctypes.data, tm.ctypes.data) == 0
    toks = tokens(comp)
    starts = np.array([t[0] for t in toks]); outs = np.array([t[2] for t in toks])
    cum = np.concatenate([[0], np.cumsum(outs)])
    print(f"n={n} ulen={ulen} windows={nw} pieces={npc} fb={fb} match={got == data}")
    if isinstance(got, bytes) and got != data:
        a = np.frombuffer(got, np.uint8); b = np.frombuffer(data, np.uint8)
        m = min(len(a), len(b))
        dif = np.nonzero(a[:m] != b[:m])[0]
        print("diffs:", len(dif), "len got/exp", len(a), len(b))
        runs, st = [], dif[0]
        for x, y in zip(dif[:-1], dif[1:]):
            if y != x + 1:
                runs.append((int(st), int(x))); st = y
        runs.append((int(st), int(dif[-1])))
        print("diff ranges:", runs[:20])
        r0, r1 = runs[0][0], runs[-1][1] + 1
        seg = a[r0:r1]
        best = []
        for dlt in range(-70000, 70000):
            lo_, hi_ = r0 + dlt, r1 + dlt
            if lo_ < 0 or hi_ > len(b):
                continue
            eq = int((b[lo_:hi_] == seg).sum())
            best.append((eq, dlt))
        best.sort(reverse=True)
        print("best shifts (matches, delta) of the wrong range:", best[:5], "of", r1 - r0)
        for r0, r1 in runs[:3]:
            print(" got", a[r0:r0 + 16], "exp", b[r0:r0 + 16])
        ti = int(np.searchsorted(cum, dif[0], side="right") - 1)
        for t in range(max(0, ti - 3), min(len(toks), ti + 40)):
            p, kind, ol, off, tl = toks[t]
            o0 = int(cum[t])
            print(f"  tok {t} in {p} kind {'lit' if kind == 0 else 'copy'} out {o0} len {ol} off {off} "
                  f"exp {b[o0:o0 + min(ol, 6)]} got {a[o0:o0 + min(ol, 6)]} raw {list(comp[p:p + 4])}")
    bits = np.unpackbits(tm.view(np.uint8), bitorder="little")[:n].astype(bool)
    true_bits = np.zeros(n, bool); true_bits[starts] = True
    bad = np.nonzero(bits != true_bits)[0]
    print("bitmap mismatches:", len(bad), bad[:20])
    for w in range(nw):
        a, b = w * 8192, min((w + 1) * 8192, n)
        sel = (starts >= a) & (starts < b)
        tout = int(outs[sel].sum())
        ex = starts[np.searchsorted(starts, b)] if np.searchsorted(starts, b) < len(starts) else n
        rl = [int(outs[(starts >= a + 128 * l) & (starts < min(a + 128 * (l + 1), b))].sum()) for l in range(64)]
        flag = "" if (wn[w, 2] == tout and wn[w, 1] == ex and list(lo[w]) == rl) else "  <-- MISMATCH"
        print(f"win {w}: entry {wn[w,0]} exit {wn[w,1]} (true {ex}) out {wn[w,2]} (true {tout}) flags {wn[w,3]}"
              f" laneouts_ok {list(lo[w]) == rl}{flag}")
    for k in range(1, npc):
        i = np.searchsorted(cum, k * 65536)
        tsp = starts[i] if i < len(starts) and cum[i] == k * 65536 else 0xffffffff
        print(f"split {k}: gpu {sp[k]} true {tsp}{'' if sp[k] == tsp else '  <-- MISMATCH'}")


if __name__ == "__main__":
    main()
