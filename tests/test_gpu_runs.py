"""Wave-parallel run discovery (wave_run_round / wave_walk_runs, pf_pages.hip) against the
one-lane header walk it replaced (walk_runs), on random RLE / bit-packed hybrid streams: long
stretches of equal bit-packed runs (what Arrow and parquet-mr write: 512 values per run), mixed
RLE runs, empty runs, a truncated final run, streams that end early, corrupt headers, value
windows (lo > 0), a start state past the first runs, and run tables that fill up (cap).
Both must agree on the return code, the runs, the covered count and the walker state.
Reference semantics: parquet-mr RunLengthBitPackingHybridDecoder (behind ParquetReader.java:146,200)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _stream(rng, bw, kind):
    out = bytearray()
    nb = (bw + 7) // 8
    nruns = int(rng.integers(1, 200))
    for i in range(nruns):
        if kind == "uniform" or (kind == "mixed" and rng.random() < 0.6):
            g = 64 if kind == "uniform" or rng.random() < 0.7 else int(rng.integers(1, 70))
            out += _uvarint((g << 1) | 1) + rng.integers(0, 256, g * bw, dtype=np.uint8).tobytes()
        else:
            cnt = int(rng.integers(0 if kind == "mixed" else 1, 3000))
            out += _uvarint(cnt << 1) + int(rng.integers(0, 1 << min(bw, 16))).to_bytes(nb, "little")
    if kind == "truncated" and len(out) > 10:
        out = out[: len(out) - int(rng.integers(1, 10))]
    if kind == "corrupt":
        out += bytes([0xFF] * 6)
    return bytes(out)


@pytest.mark.parametrize("kind", ["uniform", "mixed", "truncated", "corrupt"])
def test_wave_walk_matches_lane_walk(kind):
    from pfloor import _native
    with _native.diagnostics() as L:   # (pf_debug_walk_runs is built into the diagnostics library only)
        _walk_cases(L, kind)


def _walk_cases(L, kind):
    f = L.pf_debug_walk_runs
    f.argtypes = [C.c_char_p, C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                  C.POINTER(C.c_uint32)]
    rng = np.random.default_rng({"uniform": 1, "mixed": 2, "truncated": 3, "corrupt": 4}[kind])
    for it in range(60):
        bw = int(rng.choice([1, 2, 3, 7, 13, 14, 17, 20, 32]))
        s = _stream(rng, bw, kind)
        total = 10 ** 6
        limit = int(rng.integers(1, total))
        lo = int(rng.integers(0, limit)) if rng.random() < 0.3 else 0
        cap = int(rng.choice([4, 37, 256]))
        out = (C.c_uint32 * (2 * (5 + 4 * cap)))()
        assert f(s, len(s), bw, lo, limit, cap, 0, 0, out) == 0
        a = list(out[: 5 + 4 * cap])
        b = list(out[5 + 4 * cap:])
        n = a[1]
        assert a[:5] == b[:5], (kind, it, bw, lo, limit, cap, a[:5], b[:5])
        assert a[5: 5 + 4 * n] == b[5: 5 + 4 * n], (kind, it)
        if a[0] == 2:   # table full: continuing from the returned state agrees too
            out2 = (C.c_uint32 * (2 * (5 + 4 * cap)))()
            assert f(s, len(s), bw, lo, limit, cap, a[3], a[4], out2) == 0
            assert list(out2[:5 + 4 * cap])[:5] == list(out2[5 + 4 * cap:])[:5]
