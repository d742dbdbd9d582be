"""Diagnostic: decode one row group of a file on the GPU (whole row group, then each failing chunk
alone) and report every chunk's mismatches against the oracle as contiguous ranges, with the
chunk's page table.  python tools/debug_rg.py FILE RG [gen8m]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]
from oracle_binding import Oracle  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile, decode_file  # noqa: E402


def ranges(bad):
    out = []
    if len(bad) == 0:
        return out
    s = p = int(bad[0])
    for b in bad[1:]:
        b = int(b)
        if b != p + 1:
            out.append((s, p))
            s = b
        p = b
    out.append((s, p))
    return out


def diff(g, e):
    rep = {}
    for k in ("num_entries", "num_slots", "num_values", "num_rows", "num_chars"):
        if k in e and int(g.get(k, -1)) != int(e[k]):
            rep[k] = (int(g.get(k, -1)), int(e[k]))
    for a in ("values", "validity", "offsets", "chars", "list_offsets", "def_levels", "rep_levels"):
        if a not in e or a not in g:
            continue
        x, y = np.asarray(g[a]), np.asarray(e[a])
        if a == "validity":
            n = int(e["num_slots"])
            x = np.unpackbits(x.view(np.uint8), bitorder="little")[:n]
            y = np.unpackbits(y.view(np.uint8), bitorder="little")[:n]
        if x.shape != y.shape:
            rep[a] = f"shape {x.shape} vs {y.shape}"
            m = min(len(x), len(y))
            x, y = x[:m], y[:m]
        bad = np.flatnonzero(x != y)
        if len(bad):
            rep[a + "_bad"] = (len(bad), ranges(bad)[:8])
    return rep


def main():
    path, rg = sys.argv[1], int(sys.argv[2])
    if len(sys.argv) > 3 and sys.argv[3] == "gen8m" and not os.path.exists(path):
        import pyarrow.parquet as pq
        from pfloor import datagen
        pq.write_table(datagen.lineitem_table(8_000_000, seed=43, scale=100.0), path, compression="snappy",
                       row_group_size=4_000_000)
    orc = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
    dec = GpuDecoder(0)
    with ParquetFile(path) as pf, orc.open(path) as of:
        ncol = pf.num_columns
        got = decode_file(path, row_groups=[rg], decoder=dec)
        print("whole rg status", got["_status"], got["_error"], flush=True)
        failing = []
        for c in range(ncol):
            e = of.decode(rg, c)
            r = diff(got[(rg, c)], e)
            print(f"c{c:2d} {pf.columns[c].path[0]:16s} {'OK' if not r else r}", flush=True)
            if r:
                failing.append(c)
        for c in failing:
            d = pf.chunk_desc(rg, c, 0)
            ents, pages = 0, []
            for i in range(d.n_pages):
                p = d.pages[i]
                pages.append((p.page_type, p.encoding, ents, p.num_values, p.compressed_size, p.uncompressed_size))
                if p.page_type != 2:
                    ents += p.num_values
            print(f"c{c} pages (type, enc, first_entry, n, comp, uncomp):", pages[:12], "...", len(pages), flush=True)
            alone = decode_file(path, row_groups=[rg], columns=[c], decoder=dec)
            print(f"c{c} alone:", diff(alone[(rg, c)], of.decode(rg, c)) or "OK", flush=True)
    dec.close()


if __name__ == "__main__":
    main()
