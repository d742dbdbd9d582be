"""Pin the CPU oracle (oracle/pf_oracle.c) against the committed golden vectors:
pyarrow-decoded expectations for every fixture (tests/golden/make_golden.py) and the
Snappy known-answer vectors. This is what makes the oracle trustworthy as the checker
for the HIP path."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from golden_util import assert_chunk_equal, load_expected


@pytest.mark.parametrize("name", golden_files())
def test_oracle_matches_golden(oracle, name):
    exp = load_expected(name)
    with oracle.open(os.path.join(GOLDEN, name + ".parquet")) as f:
        assert f.num_columns == len({c for _, c in exp})
        for (rg, col), e in sorted(exp.items()):
            got = oracle_decode = f.decode(rg, col)
            assert oracle_decode["status"] == 0, (name, rg, col, got["error"])
            assert_chunk_equal(got, e, f"{name} rg{rg} c{col} {e['path']}")


def test_snappy_known_answers(oracle):
    z = np.load(os.path.join(GOLDEN, "snappy_kat.npz"), allow_pickle=False)
    names = sorted({k.rsplit("_", 1)[0] for k in z.files})
    assert len(names) >= 8
    for n in names:
        raw, comp = z[n + "_raw"].tobytes(), z[n + "_comp"].tobytes()
        assert oracle.snappy_uncompress(comp) == raw, n


def test_snappy_rejects_corrupt(oracle):
    z = np.load(os.path.join(GOLDEN, "snappy_kat.npz"), allow_pickle=False)
    comp = bytearray(z["text_comp"].tobytes())
    # truncations must error (never read out of bounds)
    for cut in (1, 2, 5, len(comp) // 2, len(comp) - 1):
        r = oracle.snappy_uncompress(bytes(comp[:cut]))
        assert r is None or isinstance(r, int) and r < 0
    # a copy with offset 0 / beyond output is corrupt
    bad = bytes([8, 0x01 | (0 << 2), 0x00])  # len 8, copy-1 offset 0 at output position 0
    assert isinstance(oracle.snappy_uncompress(bad), int)


def test_reference_roundtrip_values(oracle):
    """ParquetReadWriteTest.java:66-73: rows {1,"hello1"} and {2,"hello2"}."""
    with oracle.open(os.path.join(GOLDEN, "ref_roundtrip.parquet")) as f:
        assert [f.top_name(c) for c in range(f.num_columns)] == ["id", "email"]
        ids = f.decode(0, 0)
        em = f.decode(0, 1)
        assert ids["values"].view(np.int64).tolist() == [1, 2]
        o, ch = em["offsets"], em["chars"].tobytes()
        assert [ch[o[i]:o[i + 1]].decode() for i in range(2)] == ["hello1", "hello2"]
