"""Decode one lineitem row group (all 16 columns) REPS times -- a fixed workload for rocprofv3 --pmc
surveys (tools/gpu_pmc_all.sh); prints the row group's compressed / uncompressed bytes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd")]
import pyarrow.parquet as pq  # noqa: E402
from pfloor import datagen  # noqa: E402
from pfloor.decoder import GpuDecoder, decode_file  # noqa: E402

rows = 1048576
path = os.path.join(ROOT, "gpurun_out", f"probe_lineitem_{rows}.parquet")
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pq.write_table(datagen.lineitem_table(rows, seed=42), path, compression="snappy", row_group_size=1 << 20)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rg = pq.ParquetFile(path).metadata.row_group(0)
print("compressed", sum(rg.column(c).total_compressed_size for c in range(rg.num_columns)),
      "uncompressed", sum(rg.column(c).total_uncompressed_size for c in range(rg.num_columns)), flush=True)
with GpuDecoder(0) as dec:
    for _ in range(reps):
        got = decode_file(path, row_groups=[0], decoder=dec)
        assert got["_status"] == 0
