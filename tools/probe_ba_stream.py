"""k_ba_tile traffic check (run under rocprofv3 --pmc, tools/gpu_pmc_ba.sh): decodes l_comment of one
lineitem row group (PLAIN pages after the dictionary overflow) REPS times and prints the walk's stream
bytes per decode (the data pages' uncompressed value bytes), so FETCH_SIZE per k_ba_tile launch can be
set against the bytes the kernel must read."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, ParquetFile, decode_file  # noqa: E402

rows = 1048576
path = os.path.join(ROOT, "gpurun_out", f"probe_lineitem_{rows}.parquet")
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
with ParquetFile(path) as pf:
    col = [c.path[0] for c in pf.columns].index("l_comment")
md = pq.ParquetFile(path).metadata.row_group(0).column(col)
print(f"l_comment rg0: compressed {md.total_compressed_size} uncompressed {md.total_uncompressed_size} "
      f"encodings {md.encodings} dictionary page offset {md.dictionary_page_offset}", flush=True)
with GpuDecoder(0) as dec:
    for _ in range(reps):
        got = decode_file(path, row_groups=[0], columns=[col], decoder=dec)
        assert got["_status"] == 0
print("decodes", reps, flush=True)
