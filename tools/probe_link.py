"""Diagnostic: PCIe copy rates on this box -- pinned host -> HBM, HBM -> pinned host, and both at once on two
streams (is the link used full duplex by the copy engines?). Run with and without HSA_ENABLE_SDMA=0 (blit
kernels instead of SDMA engines).   python tools/probe_link.py [MiB]"""
import os
import sys
import time

import torch

n = int(sys.argv[1] if len(sys.argv) > 1 else 512) << 20
dev_a = torch.empty(n, dtype=torch.uint8, device="cuda")
dev_b = torch.empty(n, dtype=torch.uint8, device="cuda")
host_a = torch.empty(n, dtype=torch.uint8, pin_memory=True)
host_b = torch.empty(n, dtype=torch.uint8, pin_memory=True)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return best


def h2d():
    with torch.cuda.stream(s1):
        dev_a.copy_(host_a, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        host_b.copy_(dev_b, non_blocking=True)


def both():
    h2d()
    d2h()


def d2h_split(k):
    def f():
        ss = [torch.cuda.Stream() for _ in range(k)]
        m = n // k
        for i, s in enumerate(ss):
            with torch.cuda.stream(s):
                host_b[i * m:(i + 1) * m].copy_(dev_b[i * m:(i + 1) * m], non_blocking=True)
    return f


print(f"SDMA={os.environ.get('HSA_ENABLE_SDMA', 'default')} bytes={n}")
t = timed(h2d); print(f"h2d alone {n / t / 1e9:.2f} GB/s")
t = timed(d2h); print(f"d2h alone {n / t / 1e9:.2f} GB/s")
t = timed(both); print(f"both at once {2 * n / t / 1e9:.2f} GB/s total ({t * 1e3:.2f} ms for {n >> 20} MiB each way)")
for k in (2, 4):
    t = timed(d2h_split(k)); print(f"d2h over {k} streams {n / t / 1e9:.2f} GB/s")
