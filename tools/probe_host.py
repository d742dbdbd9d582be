"""Diagnostic: host-side cost of pf_decode_row_group (planning + metadata upload + kernel enqueue)
per context on the SF1 bench file, and the step time with the contexts' decode calls issued
sequentially vs from one host thread per context."""
import ctypes as C
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parquet-floor_amd")]
import bench  # noqa: E402
from pfloor import _native  # noqa: E402
from pfloor.decoder import GpuDecoder  # noqa: E402

d = "/tmp/pfloor_bench"
os.makedirs(d, exist_ok=True)
path = os.path.join(d, f"lineitem_{bench.SF1_ROWS}_seed{bench.SEED}_rg{bench.RG_ROWS}.parquet")
if not os.path.exists(path):
    bench.make_input(path, bench.SF1_ROWS)
pf, items, host, descs = bench.plan_file(path)
S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
decs = [GpuDecoder(0) for _ in range(S)]
L = _native.lib()
d_in = C.c_void_p()
_native.check(L.pf_device_alloc(decs[0].h, host.nbytes, C.byref(d_in)), decs[0].h, "alloc")
_native.check(L.pf_memcpy_h2d(decs[0].h, d_in, host.ctypes.data, host.nbytes), decs[0].h, "h2d")
parts = [[descs[i] for i, it in enumerate(items) if it[0] % S == k] for k in range(S)]
for _ in range(3):
    for dd, dc in zip(parts, decs):
        dc.decode(dd, d_in.value, host.nbytes, on_device=True)
    for dc in decs:
        assert dc.wait() == 0
# host cost of one decode call (GPU idle before it)
for dc in decs:
    dc.wait()
t = []
for _ in range(10):
    t0 = time.perf_counter()
    decs[0].decode(parts[0], d_in.value, host.nbytes, on_device=True)
    t.append(time.perf_counter() - t0)
    decs[0].wait()
print(f"host decode() call, ctx0 ({len(parts[0])} chunks): median {sorted(t)[5] * 1e3:.3f} ms", flush=True)


def step_seq():
    for dd, dc in zip(parts, decs):
        dc.decode(dd, d_in.value, host.nbytes, on_device=True)
    for dc in decs:
        assert dc.wait() == 0


def step_thr():
    ts = [threading.Thread(target=dc.decode, args=(dd, d_in.value, host.nbytes, True)) for dd, dc in zip(parts, decs)]
    [x.start() for x in ts]
    [x.join() for x in ts]
    for dc in decs:
        assert dc.wait() == 0


for name, f in (("sequential", step_seq), ("threads", step_thr), ("sequential", step_seq), ("threads", step_thr)):
    for _ in range(3):
        f()
    t0 = time.perf_counter()
    for _ in range(10):
        f()
    print(f"{name:10s} {S} ctx: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms/step", flush=True)
