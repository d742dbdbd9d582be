"""Diagnostic (VERDICT r05 item 1(b) input): per SF1 column, the share of Snappy output bytes that sit in
k_snappy_exec5 consumer windows with no pending byte -- windows whose bytes are all literal bytes or copy
bytes whose source lies before the window, which a token-granular fast path could move without pointer
jumping. Batches are rebuilt as the producer cuts them (at most X5_BATCH output bytes and 128 tokens,
a literal longer than 64 bytes alone), windows are 256 bytes from the batch's 4-byte aligned base, and a
copy byte is pending when its source (x - off * (1 + j // off)) is at or past the window start.

    python tools/exec_depfree.py [rows]
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

X5_BATCH, TOKS = 764, 128


def batches(toks):
    """Producer batches of one 64 KiB piece: lists of (out, kind, ol, off); long literals alone."""
    i = 0
    while i < len(toks):
        o, kind, ol, off = toks[i]
        if kind == 0 and ol > 64:
            yield "long", [toks[i]]
            i += 1
            continue
        j, tot = i, 0
        while j < len(toks) and j - i < TOKS:
            k2, ol2 = toks[j][1], toks[j][2]
            if (k2 == 0 and ol2 > 64) or tot + ol2 > X5_BATCH:
                break
            tot += ol2
            j += 1
        yield "normal", toks[i:j]
        i = j


def window_stats(tl, st):
    s0 = tl[0][0]
    Sb = s0 & ~3
    end = tl[-1][0] + tl[-1][2]
    # per output byte: pending flag
    n = end - Sb
    pend = np.zeros(n, bool)
    for (o, kind, ol, off) in tl:
        if kind == 0:
            continue
        x = np.arange(o - Sb, o - Sb + ol)
        j = x - (o - Sb)
        y = x - off * (1 + j // off)
        ws = np.where(x < 256, s0 - Sb, (x // 256) * 256)
        pend[o - Sb:o - Sb + ol] = y >= ws
    for w0 in range(0, n, 256):
        lo = max(w0, s0 - Sb)
        hi = min(w0 + 256, n)
        if hi <= lo:
            continue
        b = hi - lo
        st["bytes"] += b
        st["windows"] += 1
        npend = int(pend[lo:hi].sum())
        st["pend_bytes"] += npend
        if npend == 0:
            st["free_bytes"] += b
            st["free_windows"] += 1


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    path = f"/tmp/probe_lineitem_{rows}.parquet"
    if not os.path.exists(path):
        pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
    tot = collections.Counter()
    with ParquetFile(path) as pf:
        names = [f.name for f in pq.ParquetFile(path).schema_arrow]
        for col in range(pf.num_columns):
            s, n = pf.chunk_range(0, col)
            buf = np.zeros(n, np.uint8)
            pf.read_into(s, n, buf.ctypes.data)
            d = pf.chunk_desc(0, col, 0)
            st = collections.Counter()
            for i in range(d.n_pages):
                pg = d.pages[i]
                if pg.compressed_size >= pg.uncompressed_size:
                    continue
                toks = tokens(buf[pg.offset:pg.offset + pg.compressed_size].tobytes())
                if len(toks) <= 1:   # one literal: read in place, no executor
                    continue
                out = 0
                pieces = collections.defaultdict(list)
                for (p, kind, ol, off, tln) in toks:
                    pieces[out >> 16].append((out, kind, ol, off))
                    out += ol
                for tl in pieces.values():
                    for kind, bt in batches(tl):
                        if kind == "long":
                            st["long_bytes"] += bt[0][2]
                        else:
                            window_stats(bt, st)
            allb = st["bytes"] + st["long_bytes"]
            if not allb:
                continue
            tot.update(st)
            print(f"{names[col]:16s} out {allb / 1e6:7.2f} MB | long literals {st['long_bytes'] / allb * 100:5.1f}% | "
                  f"windows {st['windows']:6d}: dependency-free {st['free_windows'] / max(st['windows'], 1) * 100:5.1f}% "
                  f"holding {st['free_bytes'] / max(st['bytes'], 1) * 100:5.1f}% of window bytes | pending bytes "
                  f"{st['pend_bytes'] / max(st['bytes'], 1) * 100:5.1f}%", flush=True)
    allb = tot["bytes"] + tot["long_bytes"]
    print(f"{'all':16s} out {allb / 1e6:7.2f} MB | long literals {tot['long_bytes'] / allb * 100:5.1f}% | "
          f"windows {tot['windows']:6d}: dependency-free {tot['free_windows'] / max(tot['windows'], 1) * 100:5.1f}% "
          f"holding {tot['free_bytes'] / max(tot['bytes'], 1) * 100:5.1f}% of window bytes | pending bytes "
          f"{tot['pend_bytes'] / max(tot['bytes'], 1) * 100:5.1f}%")


if __name__ == "__main__":
    main()
