"""readValue's stringifier branch (ParquetReader.java:147-151: BINARY / FIXED_LEN_BYTE_ARRAY / INT96
-> primitiveType.stringifier().stringify(getBinary())), restated from upstream parquet-mr 1.12.2
PrimitiveStringifier in pfloor/reader.py. CPU tests check the restatement against independent
formatters (Python's decimal module implements the same to-scientific-string rule that
java.math.BigDecimal.toString documents); the GPU test reads a pyarrow-written file with DECIMAL
(FLBA), UUID, JSON, raw BINARY and INT96 columns through the reader mirror. Only the UTF8 branch is
pinned by the reference's own test (ParquetReadWriteTest.java:66-82); the rest is parity unpinned."""
import decimal
import os
import struct
import uuid

import numpy as np
import pytest


class _Col:
    def __init__(self, pt, lt=0, ct=-1, scale=0, tl=0):
        self.physical_type, self.logical_type, self.converted_type, self.scale, self.type_length = pt, lt, ct, scale, tl


def test_big_decimal_to_string_matches_decimal_module():
    from pfloor.reader import java_big_decimal_str
    rng = np.random.default_rng(1)
    cases = [(0, 0), (0, 2), (0, 8), (1, 7), (12, 8), (123, 2), (-5, 3), (1000, 1), (123456, 0), (-1, 6), (-1, 7),
             (10**30, 5), (-(10**20) + 7, 25)]
    for _ in range(2000):
        u = int(rng.integers(-10**12, 10**12)) * int(rng.choice([1, 10**6, 10**15]))
        cases.append((u, int(rng.integers(0, 30))))
    for u, s in cases:
        exp = str(decimal.Decimal(u).scaleb(-s))
        # Decimal keeps the exponent: (u, -s) exactly as BigDecimal(unscaled u, scale s)
        exp = str(decimal.Decimal((1 if u < 0 else 0, tuple(int(c) for c in str(abs(u))), -s)))
        assert java_big_decimal_str(u, s) == exp, (u, s)


def test_stringifier_selection_and_formats():
    from pfloor.reader import BINARY_INVALID, stringifier
    assert stringifier(_Col(6, lt=1))(b"h\xc3\xa9") == "hé"                       # STRING
    assert stringifier(_Col(6, ct=0))(b"abc") == "abc"                            # converted UTF8
    assert stringifier(_Col(6, lt=12))(b'{"a":1}') == '{"a":1}'                   # JSON
    assert stringifier(_Col(6, ct=4))(b"E") == "E"                                # ENUM
    assert stringifier(_Col(6))(b"\x00\xab\x10") == "0x00AB10"                   # unannotated BINARY
    assert stringifier(_Col(6, lt=13))(b"\x01") == "0x01"                         # BSON -> default
    assert stringifier(_Col(3))(bytes(range(12))) == "0x000102030405060708090A0B"  # INT96 -> default
    d = stringifier(_Col(7, lt=5, scale=2, tl=4))
    assert d((12345).to_bytes(4, "big", signed=True)) == "123.45"
    assert d((-5).to_bytes(4, "big", signed=True)) == "-0.05"
    assert d(b"") == BINARY_INVALID
    assert stringifier(_Col(6, ct=5, scale=9))((1).to_bytes(1, "big")) == "1E-9"
    u = uuid.UUID("12345678-9abc-def0-1234-56789abcdef0")
    assert stringifier(_Col(7, lt=14, tl=16))(u.bytes) == "12345678-9abc-def0-1234-56789abcdef0"
    iv = stringifier(_Col(7, ct=21, tl=12))
    assert iv(struct.pack("<III", 3, 0xFFFFFFFF, 7)) == "interval(3 months, 4294967295 days, 7 millis)"
    assert iv(b"\x00" * 11) == BINARY_INVALID


def _annotated_file(tmp_path, n=3000):
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(5)
    unscaled = rng.integers(-10**15, 10**15, n)
    decs = [decimal.Decimal((1 if u < 0 else 0, tuple(int(c) for c in str(abs(int(u)))), -4)) for u in unscaled]
    tiny = [decimal.Decimal((0, tuple(int(c) for c in str(int(u))), -9)) for u in rng.integers(0, 1000, n)]
    mask = rng.random(n) < 0.1
    uu = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    t = pa.table({
        "dec": pa.array(decs, pa.decimal128(20, 4), mask=mask),
        "tiny": pa.array(tiny, pa.decimal128(9, 9)),
        "uid": pa.array(uu, pa.uuid()),
        "js": pa.array([f'{{"k":{i}}}' for i in range(n)], pa.json_()),
        "raw": pa.array([bytes([i % 256, 7]) for i in range(n)], pa.binary()),
    })
    path = str(tmp_path / "annotated.parquet")
    pq.write_table(t, path, compression="snappy", store_decimal_as_integer=False)
    return path, t


@pytest.mark.gpu
def test_gpu_reader_rows_stringified(tmp_path):
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader
    path, t = _annotated_file(tmp_path)

    class H(Hydrator):
        def start(self):
            return {}

        def add(self, r, h, v):
            r[h] = v
            return r

        def finish(self, r):
            return r
    with ParquetReader.streamContent(path, HydratorSupplier.constantly(H())) as s:
        rows = s.collect()
    exp = t.to_pylist()
    assert len(rows) == len(exp)
    for r, e in zip(rows, exp):
        assert r["dec"] == (None if e["dec"] is None else str(e["dec"]))
        assert r["tiny"] == str(e["tiny"])
        assert r["uid"] == str(e["uid"])
        assert r["js"] == e["js"]
        assert r["raw"] == "0x" + e["raw"].hex().upper()
