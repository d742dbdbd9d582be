"""Diagnostic: decompress the GPU Snappy test payloads repeatedly and report every mismatch
(first differing byte), to tell deterministic bugs from races."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]
from oracle_binding import Oracle  # noqa: E402
from pfloor.decoder import GpuDecoder  # noqa: E402
import test_gpu_snappy as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
o = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
dec = GpuDecoder(0)
bad = 0
for seed in (1, 2, 3):
    for name, data in T._payloads(np.random.default_rng(seed)).items():
        comp = o.snappy_compress(data, mode=0)
        for r in range(reps):
            got, fb = dec.snappy_decompress(comp)
            if got != data:
                bad += 1
                a, b = np.frombuffer(got, np.uint8), np.frombuffer(data, np.uint8)
                d = np.nonzero(a != b)[0] if len(a) == len(b) else [-1]
                print(f"seed {seed} {name} rep {r}: fb {fb} first diff {d[0]} ndiff {len(d)}", flush=True)
print("total bad", bad, "lib", os.environ.get("PFLOOR_LIB_PATH", "default"))
