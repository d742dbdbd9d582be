"""Diagnostic: decode the SF1 bench file the way bench.py does (two contexts, row group r on
context r % 2) for many steps and report every Snappy job whose fallback flag is set after the
decode (1 = whole-page executor, 2 = redo, 3 = serial), per step, to tell a deterministic fallback
from a racy one. Usage: python tools/probe_fallback.py [steps]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-floor_amd")]
import bench  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor.decoder import GpuDecoder  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
d = "/tmp/pfloor_bench"
os.makedirs(d, exist_ok=True)
path = os.path.join(d, f"lineitem_{bench.SF1_ROWS}_seed{bench.SEED}_rg{bench.RG_ROWS}.parquet")
if not os.path.exists(path):
    bench.make_input(path, bench.SF1_ROWS)
pf, items, host, descs = bench.plan_file(path)
S = 2
decs = [GpuDecoder(0) for _ in range(S)]
parts = [[descs[i] for i, it in enumerate(items) if it[0] % S == k] for k in range(S)]
L = _native.lib()
L.pf_debug_snappy_fallback.restype = C.c_int
L.pf_debug_snappy_fallback.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
d_in = C.c_void_p()
_native.check(L.pf_device_alloc(decs[0].h, host.nbytes, C.byref(d_in)), decs[0].h, "alloc")
_native.check(L.pf_memcpy_h2d(decs[0].h, d_in, host.nbytes and host.ctypes.data, host.nbytes), decs[0].h, "h2d")
hist = {}
for s in range(steps):
    for dec, dd in zip(decs, parts):
        dec.decode(dd, d_in.value, host.nbytes, on_device=True)
    for k, dec in enumerate(decs):
        assert dec.wait() == 0, dec.error()
        nj = L.pf_debug_snappy_fallback(dec.h, None, 0)
        buf = (C.c_int * (5 * nj))()
        L.pf_debug_snappy_fallback(dec.h, buf, nj)
        t = dec.timing()
        for i in range(nj):
            fb, sl, dl, ch, pg = buf[5 * i: 5 * i + 5]
            if fb:
                key = (k, i, fb)
                hist[key] = hist.get(key, 0) + 1
                print(f"step {s} ctx {k} job {i} fb {fb} chunk {ch} page {pg} src {sl} dst {dl} "
                      f"exec_ms {t.get('snappy_exec', 0):.3f}", flush=True)
print("summary (ctx, job, fb): count over", steps, "steps:", hist, flush=True)
