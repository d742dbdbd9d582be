"""Diagnostic (design input for a token-level Snappy executor): per batch of a piece (2 KiB of input),
how many copy tokens read a source that lies inside the batch's own output, whether that source lies
inside ONE earlier token (so the copy can be rewritten as a copy of that token's source: composition),
whether the periodic (self-overlapping) cases compose without a wrap, and the chain depth in tokens.

    python tools/exec_compose.py [rows]
"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tools")]
import pyarrow.parquet as pq  # noqa: E402

from pfloor import datagen  # noqa: E402
from pfloor.decoder import ParquetFile  # noqa: E402
from snappy_stats import tokens  # noqa: E402

INF = 1 << 30


def batch_stats(tl, st):
    """tl: tokens of one batch [(o, kind, ol, off)] (piece-relative o), window start o0 = tl[0][0]."""
    o0 = tl[0][0]
    starts = np.array([t[0] for t in tl])
    # per token mapping state: None = literal / final, else (u, delta, period)
    depth = {}
    res = {}   # token index -> ("fin") or ("hard")
    for i, (o, kind, ol, off) in enumerate(tl):
        if kind == 0:
            res[i] = ("fin", 0)
            continue
        s = o - off
        per = off if off < ol else INF
        need = min(ol, off)            # bytes of the source the copy reads (the rest repeat)
        if s + need <= o0:
            res[i] = ("fin", 0)
            st["pre"] += 1
            continue
        st["inwin"] += 1
        u = int(np.searchsorted(starts, s, side="right") - 1)
        uo, uk, uol, uoff = tl[max(u, 0)]
        if u < 0 or s + need > uo + uol:
            res[i] = ("hard", 0)
            st["span"] += 1
            continue
        d = s - uo
        # compose along u's chain
        r = res[u]
        if r[0] == "hard":
            res[i] = ("hard", 0)
            st["hard_src"] += 1
            continue
        if r[0] == "fin" and uk == 0:
            res[i] = ("fin", 1)
            st["lit"] += 1
            continue
        # u is a copy resolved to a final source with period pu and depth r[1]
        upu = uoff if uoff < uol else INF
        if upu != INF and (d % upu) + min(per, ol) > upu:
            res[i] = ("hard", 0)
            st["wrap"] += 1
            continue
        res[i] = ("fin", r[1] + 1)
        st["ok"] += 1
        st["depth_max"] = max(st["depth_max"], r[1] + 1)
        st["depth_sum"] += r[1] + 1


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    path = f"/tmp/probe_lineitem_{rows}.parquet"
    if not os.path.exists(path):
        pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
    with ParquetFile(path) as pf:
        for col in range(pf.num_columns):
            s, n = pf.chunk_range(0, col)
            buf = np.zeros(n, np.uint8)
            pf.read_into(s, n, buf.ctypes.data)
            d = pf.chunk_desc(0, col, 0)
            st = collections.Counter()
            npages = 0
            for i in range(d.n_pages):
                pg = d.pages[i]
                if pg.compressed_size >= pg.uncompressed_size:
                    continue
                b = buf[pg.offset:pg.offset + pg.compressed_size].tobytes()
                toks = tokens(b)
                if len(toks) <= 1:
                    continue
                npages += 1
                if npages > 12:
                    break
                out = 0
                pieces = collections.defaultdict(list)
                for (p, kind, ol, off, tln) in toks:
                    pieces[out >> 16].append((p, out & 0xffff, kind, ol, off))
                    out += ol
                for k, tl in pieces.items():
                    # batches: 2 KiB of input, at most 4 KiB of output
                    i0 = 0
                    while i0 < len(tl):
                        p0, o0 = tl[i0][0], tl[i0][1]
                        i1 = i0
                        while i1 < len(tl) and tl[i1][0] < (p0 & ~15) + 2048 and tl[i1][1] + tl[i1][3] - (o0 & ~15) <= 4096:
                            i1 += 1
                        i1 = max(i1, i0 + 1)
                        batch_stats([(t[1], t[2], t[3], t[4]) for t in tl[i0:i1]], st)
                        st["batches"] += 1
                        st["tokens"] += i1 - i0
                        i0 = i1
            if not st["batches"]:
                continue
            inw = max(st["inwin"], 1)
            print(f"col {col:2d}: batches {st['batches']} tok/batch {st['tokens'] / st['batches']:.0f} "
                  f"in-window copies {st['inwin'] / st['tokens'] * 100:.1f}% of tokens: from literal {st['lit'] / inw * 100:.1f}% "
                  f"composed {st['ok'] / inw * 100:.1f}% span {st['span'] / inw * 100:.1f}% wrap {st['wrap'] / inw * 100:.1f}% "
                  f"hard-src {st['hard_src'] / inw * 100:.1f}% | depth mean {st['depth_sum'] / max(st['ok'], 1):.1f} max {st['depth_max']}",
                  flush=True)


if __name__ == "__main__":
    main()
