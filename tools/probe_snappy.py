"""Diagnostic: time the Snappy kernels on single synthetic streams (run under rocprofv3).
With PFLOOR_LIB_PATH pointing at the stamp build (make -C parquet-floor_amd stamps) it also
prints per-phase s_memtime cycle sums of the index kernel."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-floor_amd"), os.path.join(ROOT, "tests")]
from oracle_binding import Oracle  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor.decoder import GpuDecoder  # noqa: E402

o = Oracle(os.path.join(ROOT, "oracle", "libpf_oracle.so"))
rng = np.random.default_rng(0)
words = [b"alpha ", b"beta ", b"gamma ", b"delta ", b"ironic ", b"deposits ", b"packages ", b"furiously "]
text = b"".join(words[i] for i in rng.integers(0, len(words), 200000))
rnd = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
cases = {"text64k": text[:65536], "text1m": text[:1 << 20], "rnd1m": rnd}
dec = GpuDecoder(0)
L = _native.lib()
stamps = getattr(L, "pf_debug_stamps", None) if os.environ.get("PFLOOR_LIB_PATH") else None
if stamps:
    stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
for name, data in cases.items():
    comp = o.snappy_compress(data, 0)
    ts = []
    buf = (C.c_ulonglong * 16)()
    if stamps:
        stamps(buf, 16, 1)
    for _ in range(5):
        t0 = time.perf_counter()
        got, fb = dec.snappy_decompress(comp)
        ts.append(time.perf_counter() - t0)
        assert got == data
    line = f"{name}: in {len(comp)} out {len(data)} windows {len(comp) // 2048} best {min(ts) * 1e3:.3f} ms fb={fb}"
    if stamps:
        stamps(buf, 16, 1)
        w = max(1, 5 * (len(comp) // 2048))
        line += " | cycles/window: " + " ".join(f"p{i}={buf[i] / w:.0f}" for i in range(8) if buf[i])
    print(line, flush=True)
