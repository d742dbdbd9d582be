"""CPU check of the executor consumer's integer source arithmetic (pf_snappy_par.hip, k_snappy_exec5;
DESIGN 4.25): a copy byte at index j < 64 of a token with offset o < 4096 reads x - o * (1 + floor(j / o)),
and the consumer takes floor(j / o) as (j * m) >> 16 with m = floor(65536 * rcp(o)) + 1, where the
hardware reciprocal may round up by an ulp: m is floor(65536 / o) + 1 or one more. Both must be exact."""
import numpy as np


def test_reciprocal_floor_division_exact():
    o = np.arange(1, 4096, dtype=np.int64)[:, None]
    j = np.arange(0, 64, dtype=np.int64)[None, :]
    want = j // o
    for extra in (1, 2):
        m = 65536 // o + extra
        assert m.max() < (1 << 24)                     # a 24-bit multiply operand
        got = (j * m) >> 16
        assert np.array_equal(got, want), extra
    # float32 reciprocal as computed on the device, then truncated: within the two cases above
    r = (65536.0 * (1.0 / o.astype(np.float32))).astype(np.float32)
    m = r.astype(np.int64) + 1
    assert np.all((m == 65536 // o + 1) | (m == 65536 // o + 2))
