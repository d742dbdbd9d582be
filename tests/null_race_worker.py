"""Worker for test_gpu_page_null.py::test_null_blocks_concurrent (runs in its own process: with
PF_PAGE_NULL=1 it decodes on the diagnostics build, where that switch is read at pf_ctx_create; with 0,
the default, on the product library). Two threads, each with its own
decode context (HIP stream), decode halves of a wide nullable file together, three times; every
chunk is compared with the oracle. Under that contention k_flat_null's blocks of one page start at
different times, which is what the r04 race needed (a block skipping its page once a sibling block
had finished)."""
import contextlib
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402

from golden_util import assert_chunk_equal  # noqa: E402
from oracle_binding import Oracle  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor.decoder import GpuDecoder, decode_file  # noqa: E402


def main(path):
    rng = np.random.default_rng(11)
    n, ncol = 400_000, 48
    cols = {}
    for c in range(ncol):
        pool = rng.integers(-2**31, 2**31 - 1, 100_000).astype(np.int32 if c % 2 else np.int64)
        cols[f"c{c}"] = pa.array(pool[rng.integers(0, len(pool), n)], mask=rng.random(n) < 0.3)
    pq.write_table(pa.table(cols), path, compression="snappy", row_group_size=n)
    want = {}
    with Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so")).open(path) as of:
        for c in range(ncol):
            want[c] = of.decode(0, c)
    decs = [GpuDecoder(0), GpuDecoder(0)]
    errs = []

    def work(k):
        try:
            for _ in range(3):
                sub = list(range(k, ncol, 2))
                got = decode_file(path, row_groups=[0], columns=sub, decoder=decs[k])
                assert got["_status"] == 0, got["_error"]
                for c in sub:
                    assert_chunk_equal(got[(0, c)], want[c], f"column {c}")
        except Exception as e:   # noqa: BLE001 (reported by the parent)
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for d in decs:
        d.close()
    print("ERRORS" if errs else "OK", errs[:2], flush=True)
    return 1 if errs else 0


if __name__ == "__main__":
    with (_native.diagnostics() if os.environ.get("PF_PAGE_NULL") == "1" else contextlib.nullcontext()):
        rc = main(sys.argv[1])
    sys.exit(rc)
