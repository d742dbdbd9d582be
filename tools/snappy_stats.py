"""Diagnostic: token statistics of the Snappy page bodies of a lineitem-shaped file (design input
for the GPU decompressor): copy-offset distribution, literal lengths, and how quickly a token walk
started at an arbitrary region boundary synchronises with the true token chain."""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402

from pfloor import datagen  # noqa: E402
from pfloor.decoder import ParquetFile  # noqa: E402


def tokens(b):
    """(pos, kind, out_len, offset) per token; kind 0 literal, 1 copy."""
    p, n, sh = 0, 0, 0
    while True:
        c = b[p]; p += 1
        n |= (c & 0x7F) << sh; sh += 7
        if c < 0x80:
            break
    out = []
    while p < len(b):
        t = b[p]
        ty = t & 3
        if ty == 0:
            L = t >> 2
            if L < 60:
                ln, il = L + 1, 1
            else:
                nb = L - 59
                ln = int.from_bytes(b[p + 1:p + 1 + nb], "little") + 1
                il = 1 + nb
            out.append((p, 0, ln, 0, il + ln))
            p += il + ln
        elif ty == 1:
            out.append((p, 1, 4 + ((t >> 2) & 7), ((t >> 5) << 8) | b[p + 1], 2))
            p += 2
        elif ty == 2:
            out.append((p, 1, (t >> 2) + 1, b[p + 1] | (b[p + 2] << 8), 3))
            p += 3
        else:
            out.append((p, 1, (t >> 2) + 1, int.from_bytes(b[p + 1:p + 5], "little"), 5))
            p += 5
    return out


def tok_len(b, p):
    t = b[p]
    ty = t & 3
    if ty == 0:
        L = t >> 2
        if L < 60:
            return L + 2
        nb = L - 59
        return 1 + nb + int.from_bytes(b[p + 1:p + 1 + nb], "little") + 1
    return (2, 3, 5)[ty - 1]


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
    path = f"/tmp/probe_lineitem_{rows}.parquet"
    if not os.path.exists(path):
        pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
    offs, copy_lens, lit_lens = [], [], []
    per_kind = collections.defaultdict(lambda: [0, 0, 0, 0])   # pages, tokens, in, out
    sync = collections.defaultdict(lambda: [0, 0, 0])          # regions, consistent-first-try, spec tokens before sync
    with ParquetFile(path) as pf:
        for col in range(pf.num_columns):
            s, n = pf.chunk_range(0, col)
            buf = np.zeros(n, np.uint8)
            pf.read_into(s, n, buf.ctypes.data)
            d = pf.chunk_desc(0, col, 0)
            for i in range(d.n_pages):
                pg = d.pages[i]
                b = buf[pg.offset:pg.offset + pg.compressed_size].tobytes()
                kind = "dict" if pg.page_type == 2 else ("dictids" if pg.encoding in (2, 8) else "plain")
                toks = tokens(b)
                k = per_kind[kind]
                k[0] += 1; k[1] += len(toks); k[2] += len(b); k[3] += sum(t[2] for t in toks)
                for t in toks:
                    if t[1]:
                        offs.append(t[3]); copy_lens.append(t[2])
                    else:
                        lit_lens.append(t[2])
                starts = np.array([t[0] for t in toks], np.int64)
                isstart = np.zeros(len(b) + 8, bool)
                isstart[starts] = True
                for RB in (256,):
                    for r0 in range(RB, len(b), RB):
                        # true entry: first true token start >= r0
                        j = np.searchsorted(starts, r0)
                        if j >= len(starts):
                            continue
                        e = starts[j]
                        if e >= r0 + RB:
                            continue
                        q, cnt = r0, 0
                        while q < e:
                            q += tok_len(b + b"\0" * 8, q); cnt += 1
                        sy = sync[(kind, RB)]
                        sy[0] += 1; sy[1] += int(q == e); sy[2] += cnt
    offs = np.array(offs); lit = np.array(lit_lens); cl = np.array(copy_lens)
    print("kinds:", {k: v for k, v in per_kind.items()})
    print(f"copies {len(offs)} literals {len(lit)}; copy bytes {cl.sum()} literal bytes {lit.sum()}")
    for th in (1024, 2048, 4096, 8192, 16384, 32768):
        m = offs > th
        print(f"  offset > {th:6d}: {m.mean() * 100:5.1f}% of copies, {cl[m].sum() / cl.sum() * 100:5.1f}% of copy bytes")
    m = offs < cl
    print(f"  overlapping (offset < len): {m.mean() * 100:.1f}%")
    print("  literal len pct 50/90/99:", np.percentile(lit, [50, 90, 99]))
    print("  copy len pct 50/90/99:", np.percentile(cl, [50, 90, 99]))
    for k, v in sync.items():
        print(f"sync {k}: regions {v[0]} consistent {v[1] / max(v[0], 1) * 100:.1f}% spec tokens before entry {v[2] / max(v[0], 1):.2f}")


if __name__ == "__main__":
    main()
