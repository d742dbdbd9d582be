"""Diagnostic (design input for the LDS-image Snappy executor): per 64 KiB piece of the pages the
executor decodes (compressed, not a single literal), the tokens, the copy offsets and the number of
pointer-doubling rounds a byte-level resolution needs when the piece is resolved in windows of W
output bytes whose preceding bytes are final.

    python tools/exec_depth.py [rows]
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


def piece_rounds(src, lit, W):
    """Rounds of pointer doubling until every byte's pointer is a literal byte or precedes its window."""
    n = len(src)
    ws = (np.arange(n) // W) * W
    p = src.copy()
    done = lit | (p < ws)
    r = 0
    while not done.all() and r < 24:
        p = np.where(done, p, p[p])
        done = done | lit[p] | (p < ws)
        r += 1
    return r


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    path = f"/tmp/probe_lineitem_{rows}.parquet"
    if not os.path.exists(path):
        pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
    Ws = (256, 1024, 2048, 4096, 8192)
    with ParquetFile(path) as pf:
        names = [pf.columns[c].path[0] if hasattr(pf, "columns") else str(c) for c in range(pf.num_columns)]
        for col in range(pf.num_columns):
            s, n = pf.chunk_range(0, col)
            buf = np.zeros(n, np.uint8)
            pf.read_into(s, n, buf.ctypes.data)
            d = pf.chunk_desc(0, col, 0)
            stats = collections.defaultdict(list)
            far = [0, 0]
            for i in range(d.n_pages):
                pg = d.pages[i]
                if pg.compressed_size >= pg.uncompressed_size:
                    continue
                b = buf[pg.offset:pg.offset + pg.compressed_size].tobytes()
                toks = tokens(b)
                if len(toks) <= 1:
                    continue
                out = 0
                pieces = collections.defaultdict(list)
                for (p, kind, ol, off, tl) in toks:
                    pieces[out >> 16].append((out & 0xffff, kind, ol, off))
                    out += ol
                for k, tl in pieces.items():
                    P = sum(t[2] for t in tl)
                    src = np.zeros(P, np.int64)
                    lit = np.zeros(P, bool)
                    for (o, kind, ol, off) in tl:
                        if kind == 0:
                            lit[o:o + ol] = True
                            src[o:o + ol] = np.arange(o, o + ol)
                        else:
                            src[o:o + ol] = np.arange(o, o + ol) - off
                            far[0] += 1
                            far[1] += off > 32768
                    stats["tokens"].append(len(tl))
                    stats["bytes"].append(P)
                    for W in Ws:
                        stats[W].append(piece_rounds(src, lit, W))
            if not stats["tokens"]:
                print(f"col {col}: no executor pages")
                continue
            t = np.array(stats["tokens"])
            msg = f"col {col:2d}: pieces {len(t):4d} tokens/piece mean {t.mean():7.0f} max {t.max():6d}; " \
                  f"copies {far[0]} off>32K {far[1]}; rounds(W) " + \
                  " ".join(f"{W}:{np.mean(stats[W]):.1f}/{np.max(stats[W])}" for W in Ws)
            print(msg, flush=True)


if __name__ == "__main__":
    main()
