"""Diagnostic: decode config 4's wide file (bench --workload wide) column subsets in one batch and
report failing chunks / pages (PF_PAGE_NULL=0 exercises k_lvl + k_flat_null alone)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile, decode_file  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
path = f"/tmp/probe_wide_{rows}.parquet"
if not os.path.exists(path):
    pq.write_table(datagen.wide_table(rows, seed=4, pool=100000), path, compression="snappy", row_group_size=rows)
with ParquetFile(path) as pf:
    ncol = pf.num_columns
    dec = GpuDecoder(0)   # one context, reused: batches after the first see its arenas' old contents
    for rep in range(3):
      for k in range(4):
        cols = list(range(k, ncol, 4))
        got = decode_file(path, row_groups=[0], columns=cols, decoder=dec)
        print(f"rep {rep} subset {k}: status {got['_status']} {got['_error']}", flush=True)
        if got["_status"]:
            err = got["_error"]
            if "chunk" in err:
                ci = int(err.split("chunk")[1].split(":")[0])
                c = cols[ci]
                d = pf.chunk_desc(0, c, 0)
                pg = int(err.split("page")[1].strip(" )"))
                print(f"  column {c} type {pf.columns[c].physical_type} pages {d.n_pages}")
                for i in range(d.n_pages):
                    p = d.pages[i]
                    print(f"   page {i} type {p.page_type} enc {p.encoding} nv {p.num_values} comp {p.compressed_size} unc {p.uncompressed_size}")
