"""Design probe for a token-granular Snappy executor (r04): per column of a lineitem-shaped row
group, the page streams' tokens are cut into batches of B tokens (<= C output bytes, within 64 KiB
pieces) and every copy classified by where its source [a, a + min(len, off)) lies:
  pre    before the batch (already in the ring / HBM),
  lit    inside one in-batch literal,
  one    inside one in-batch copy (token-level pointer jumping can redirect it),
  multi  spanning several in-batch tokens (needs byte-level resolution or a batch cut).
Also the redirect-chain depth of 'one' copies."""
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


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    C = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
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
            depth = collections.Counter()
            nb = 0
            ntok = 0
            outb = 0
            for i in range(d.n_pages):
                pg = d.pages[i]
                b = buf[pg.offset:pg.offset + pg.compressed_size].tobytes()
                toks = tokens(b)
                if len(toks) <= 1:
                    continue
                T = np.array([(t[1], t[2], t[3]) for t in toks], np.int64)
                k, ol, off = T[:, 0], T[:, 1], T[:, 2]
                o = np.concatenate([[0], np.cumsum(ol)[:-1]])
                ntok += len(T); outb += int(ol.sum())
                # batch start index per token (B tokens, <= C output bytes, within a 64 KiB piece)
                bs = np.empty(len(T), np.int64)
                j = 0
                ol_l, o_l = ol.tolist(), o.tolist()
                while j < len(T):
                    e, O0, pc = j, o_l[j], o_l[j] >> 16
                    while e < len(T) and e - j < B and (o_l[e] >> 16) == pc and o_l[e] + ol_l[e] - O0 <= C:
                        e += 1
                    e = max(e, j + 1)
                    bs[j:e] = j
                    nb += 1
                    j = e
                cp = k != 0
                a = o - off
                m = np.minimum(ol, off)
                O0 = o[bs]
                pre = cp & (a + m <= O0)
                u = np.searchsorted(o, a, side="right") - 1
                u = np.clip(u, 0, len(T) - 1)
                inside = cp & ~pre & (u >= bs) & (a + m <= o[u] + ol[u]) & (u != np.arange(len(T)))
                lit = inside & (k[u] == 0)
                one = inside & (k[u] != 0)
                multi = cp & ~pre & ~inside
                st["pre"] += int(pre.sum()); st["lit"] += int(lit.sum()); st["one"] += int(one.sum()); st["multi"] += int(multi.sum())
                # redirect depth of 'one' copies: hops until pre / literal
                h = np.where(pre, 0, np.where(lit, 1, np.where(one, -1, 999)))
                h[~cp] = 0
                for _ in range(70):
                    und = h < 0
                    if not und.any():
                        break
                    hu = h[u]
                    h = np.where(und & (hu >= 0), np.where(hu >= 999, 999, hu + 1), h)
                for hv, c in zip(*np.unique(h[one], return_counts=True)):
                    depth[int(min(hv, 999))] += int(c)
            tot = sum(st.values())
            nm = pf.columns[col].path[0]
            if tot == 0:
                print(f"{nm}: no copies ({ntok} tokens)")
                continue
            dd = sorted(depth.items())
            mx = max((h for h, _ in dd), default=0)
            print(f"{nm}: tokens {ntok} out {outb} B/tok {outb / max(ntok, 1):.1f} batches {nb} ({outb / max(nb, 1):.0f} B/batch) copies {tot}: "
                  + " ".join(f"{k} {v / tot * 100:.1f}%" for k, v in sorted(st.items())) + f"  depth max {mx}, p50 "
                  + str(np.percentile(np.repeat([h for h, _ in dd], [c for _, c in dd]), 50) if dd else "-"))


if __name__ == "__main__":
    main()
