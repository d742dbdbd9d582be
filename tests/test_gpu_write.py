"""Write path on the GPU (the reference's ParquetWriter.java:61-165): Snappy
compression, dictionary encoding, v2 data pages and the file writer, checked by reading the files
back with the CPU oracle, with pyarrow (an independent reader) and with the GPU read path.
Byte-for-byte parity with parquet-mr's writer is unpinned (no JDK / parquet-mr here): the
properties checked are round-trip equality, a valid Snappy stream, and the dictionary order
(first occurrence, parquet-mr's DictionaryValuesWriter order)."""
import os

import numpy as np
import pytest

from golden_util import assert_chunk_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


def gpu_compress(dec, data):
    import ctypes as C
    from pfloor._native import check, lib
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    cap = 32 + len(data) + len(data) // 6 + 64
    dst = np.zeros(cap, np.uint8)
    n = C.c_size_t()
    check(lib().pf_snappy_compress(dec.h, src.ctypes.data, len(data), dst.ctypes.data, cap, C.byref(n)), dec.h,
          "pf_snappy_compress")
    return dst[:n.value].tobytes()


def _buffers():
    rng = np.random.default_rng(11)
    text = b"".join(b"the quick brown fox %d jumps over the lazy dog %d\n" % (i, i * 7 % 13) for i in range(6000))
    ints = np.arange(50000, dtype=np.int64).tobytes()
    small = rng.integers(0, 4, 200000, dtype=np.uint8).tobytes()
    return {
        "empty": b"", "one": b"x", "short": b"abcabcabcabc", "zeros_64k": bytes(65536), "zeros_65537": bytes(65537),
        "random_300k": rng.integers(0, 256, 300000, dtype=np.uint8).tobytes(), "text": text, "ints": ints,
        "small_alphabet": small, "long_run": b"ab" * 100000 + b"tail",
    }


@pytest.mark.parametrize("name", sorted(_buffers()))
def test_snappy_compress_roundtrip(dec, oracle, name):
    data = _buffers()[name]
    comp = gpu_compress(dec, data)
    assert len(comp) <= 32 + len(data) + len(data) // 6
    assert oracle.snappy_uncompress(comp) == data                 # CPU restatement of the format
    got, _fb = dec.snappy_decompress(comp, cap=max(1, len(data)))  # the GPU read path
    assert got == data
    if len(data) >= 1000 and name not in ("random_300k",):
        assert len(comp) < 0.6 * len(data), (name, len(comp), len(data))


def test_snappy_compress_vs_pyarrow(dec):
    pa = pytest.importorskip("pyarrow")
    for name, data in _buffers().items():
        if not data:
            continue
        comp = gpu_compress(dec, data)
        assert pa.decompress(comp, decompressed_size=len(data), codec="snappy").to_pybytes() == data, name


def _config1(n, seed=1):
    """SURVEY §8(d) config 1 shape: id INT64 0..n-1, x DOUBLE U[0,1), n optional INT32 U[0,1000)
    with 10% nulls, s UTF8 from a 1,000-string vocabulary (len 8-24); plus a FLOAT and a BOOLEAN."""
    rng = np.random.default_rng(seed)
    vocab = [("w%05d" % i + "x" * int(rng.integers(2, 19))).encode() for i in range(1000)]
    pick = rng.integers(0, 1000, n)
    lens = np.array([len(vocab[i]) for i in pick], np.int64)
    offsets = np.zeros(n + 1, np.int32)
    np.cumsum(lens, out=offsets[1:])
    chars = np.frombuffer(b"".join(vocab[i] for i in pick), np.uint8)
    present = rng.random(n) >= 0.1
    return {
        "id": np.arange(n, dtype=np.int64),
        "x": rng.random(n),
        "n": (np.where(present, rng.integers(0, 1000, n), 0).astype(np.int32), np.packbits(present, bitorder="little")),
        "s": (offsets, chars),
        "f": rng.random(n).astype(np.float32),
        "b": (rng.random(n) < 0.3).astype(np.uint8),
    }, present, [vocab[i] for i in pick]


def _schema():
    from pfloor import writer as W
    return W.MessageType("config1", W.required(W.INT64).named("id"), W.required(W.DOUBLE).named("x"),
                         W.optional(W.INT32).named("n"), W.required(W.BINARY).as_string().named("s"),
                         W.required(W.FLOAT).named("f"), W.required(W.BOOLEAN).named("b"))


def test_write_roundtrip_config1(dec, oracle, tmp_path):
    """Two row groups of config-1-shaped columns: pyarrow, the oracle and the GPU reader all read
    back exactly what was written; dictionary columns are RLE_DICTIONARY, BOOLEAN falls back."""
    pq = pytest.importorskip("pyarrow.parquet")
    from pfloor.decoder import decode_file
    from pfloor.writer import ParquetWriter
    path = str(tmp_path / "w.parquet")
    n1, n2 = 50000, 30001
    c1, p1, s1 = _config1(n1, 1)
    c2, p2, s2 = _config1(n2, 2)
    w = ParquetWriter(_schema(), path, None, decoder=dec)
    w.write_columns(c1, n1)
    enc1 = list(w.last_chunks)
    w.write_columns(c2, n2)
    w.close()
    # id is all-distinct: 50000 x 8 B = 400 KB < 1 MiB, so dictionary; BOOLEAN never (fallback 3).
    # DELIBERATE DIVERGENCE (parity unpinned): parquet-mr's FallbackValuesWriter drops a
    # dictionary that does not compress its first page (isCompressionSatisfying) and, under
    # PARQUET_2_0, writes such an all-distinct INT64 column DELTA_BINARY_PACKED; this writer keeps the
    # dictionary while it fits the 1 MiB page limit. Asserted here as the chosen behaviour.
    assert [e[1] for e in enc1] == [8, 8, 8, 8, 8, 0], enc1
    assert enc1[5][2] == 3 and enc1[3][0] <= 1000
    t = pq.read_table(path)
    assert t.num_rows == n1 + n2
    for cols, pres, strs, lo, hi in ((c1, p1, s1, 0, n1), (c2, p2, s2, n1, n1 + n2)):
        sl = t.slice(lo, hi - lo)
        assert np.array_equal(sl.column("id").to_numpy(), cols["id"])
        assert np.array_equal(sl.column("x").to_numpy().view(np.uint64), cols["x"].view(np.uint64))
        assert np.array_equal(sl.column("f").to_numpy().view(np.uint32), cols["f"].view(np.uint32))
        assert np.array_equal(sl.column("b").to_numpy(zero_copy_only=False).astype(np.uint8), cols["b"])
        nn = sl.column("n").to_pylist()
        assert [v is not None for v in nn] == list(pres)
        assert all(v == int(e) for v, e, p in zip(nn, cols["n"][0], pres) if p)
        assert [v.encode() for v in sl.column("s").to_pylist()] == strs
    # the oracle and the GPU read path agree bit-exactly on every chunk
    got = decode_file(path, decoder=dec)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        for key, g in got.items():
            if isinstance(key, tuple):
                assert_chunk_equal(g, of.decode(*key), f"written rg{key[0]} c{key[1]}")


def test_dictionary_is_first_occurrence_order(dec, oracle, tmp_path):
    """parquet-mr's DictionaryValuesWriter numbers values in order of first appearance: the
    dictionary page holds the distinct values in that order."""
    pq = pytest.importorskip("pyarrow.parquet")
    from pfloor import writer as W
    rng = np.random.default_rng(5)
    vals = rng.integers(-500, 500, 40000).astype(np.int64)
    words = [("k%d" % v).encode() for v in rng.integers(0, 300, 40000)]
    offs = np.zeros(len(words) + 1, np.int32)
    np.cumsum([len(x) for x in words], out=offs[1:])
    path = str(tmp_path / "d.parquet")
    sch = W.MessageType("d", W.required(W.INT64).named("v"), W.required(W.BINARY).as_string().named("w"))
    w = W.ParquetWriter(sch, path, None, decoder=dec)
    w.write_columns({"v": vals, "w": (offs, np.frombuffer(b"".join(words), np.uint8))}, len(vals))
    w.close()
    from pfloor.decoder import ParquetFile

    def dict_page(col):
        """The chunk's dictionary page body, Snappy-decompressed by the oracle (PLAIN values)."""
        with ParquetFile(path) as pf:
            start, size = pf.chunk_range(0, col)
            d = pf.chunk_desc(0, col, 0)
            pages = [(d.pages[i].page_type, d.pages[i].offset, d.pages[i].compressed_size) for i in range(d.n_pages)]
        raw = open(path, "rb").read()[start:start + size]
        dp = [p for p in pages if p[0] == 2]
        assert len(dp) == 1 and pages[0][0] == 2
        return oracle.snappy_uncompress(raw[dp[0][1]:dp[0][1] + dp[0][2]])

    _u, first = np.unique(vals, return_index=True)
    assert np.array_equal(np.frombuffer(dict_page(0), np.int64), vals[np.sort(first)])
    seen, exp_w = set(), []
    for x in words:
        if x not in seen:
            seen.add(x)
            exp_w.append(x)
    body, got_w, k = dict_page(1), [], 0
    while k < len(body):
        ln = int.from_bytes(body[k:k + 4], "little")
        got_w.append(body[k + 4:k + 4 + ln])
        k += 4 + ln
    assert got_w == exp_w
    t = pq.read_table(path)
    assert np.array_equal(t.column("v").to_numpy(), vals)
    assert [x.encode() for x in t.column("w").to_pylist()] == words


def test_fallbacks_and_edges(dec, oracle, tmp_path):
    """Dictionary above the 1 MiB page limit -> PLAIN; all-null optional column; single-value
    dictionary; empty strings; pages that end mid-byte; an uncompressed chunk."""
    pq = pytest.importorskip("pyarrow.parquet")
    from pfloor import writer as W
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(9)
    n = 70003
    big = [("%020d" % i).encode() + bytes(rng.integers(97, 123, 40, dtype=np.uint8)) for i in range(n)]   # ~4 MB distinct
    offs = np.zeros(n + 1, np.int32)
    np.cumsum([len(x) for x in big], out=offs[1:])
    empty_offs = np.zeros(n + 1, np.int32)
    sch = W.MessageType("e", W.required(W.BINARY).as_string().named("big"), W.optional(W.DOUBLE).named("nul"),
                        W.required(W.INT32).named("one"), W.optional(W.BINARY).as_string().named("emp"))
    path = str(tmp_path / "e.parquet")
    w = W.ParquetWriter(sch, path, None, decoder=dec)
    w.write_columns({"big": (offs, np.frombuffer(b"".join(big), np.uint8)),
                     "nul": (np.zeros(n), np.zeros((n + 7) // 8, np.uint8)),
                     "one": np.full(n, 7, np.int32),
                     "emp": (empty_offs, np.zeros(0, np.uint8), np.packbits(rng.random(n) < 0.5, bitorder="little"))}, n)
    encs = list(w.last_chunks)
    w.close()
    assert encs[0][1] == 0 and encs[0][2] == 1          # PLAIN, dictionary too large
    assert encs[2][0] == 1 and encs[2][1] == 8          # one dictionary entry
    t = pq.read_table(path)
    assert [x.encode() for x in t.column("big").to_pylist()] == big
    assert t.column("nul").null_count == n
    assert set(t.column("one").to_numpy()) == {7}
    emp = t.column("emp").to_pylist()
    assert all(v in (None, "") for v in emp)
    got = decode_file(path, decoder=dec)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        for key, g in got.items():
            if isinstance(key, tuple):
                assert_chunk_equal(g, of.decode(*key), f"edges c{key[1]}")
    # uncompressed codec
    path2 = str(tmp_path / "u.parquet")
    w = W.ParquetWriter(W.MessageType("u", W.required(W.INT64).named("v")), path2, None, decoder=dec, codec=0)
    w.write_columns({"v": np.arange(1000, dtype=np.int64) % 17}, 1000)
    w.close()
    assert np.array_equal(pq.read_table(path2).column("v").to_numpy(), np.arange(1000) % 17)


def test_reference_write_read_test(dec, tmp_path):
    """ParquetReadWriteTest.java:28-83 end to end on this stack: the reference's schema
    (required INT64 id, required UTF8 email), its Dehydrator, two records written through the
    GPU write path, read back through the host mirror of ParquetReader, also with projection."""
    from pfloor import writer as W
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader

    sch = W.MessageType("foo", W.required(W.INT64).named("id"), W.required(W.BINARY).as_string().named("email"))

    class Deh(W.Dehydrator):
        def dehydrate(self, record, vw):
            vw.write("id", record[0])
            vw.write("email", record[1])

    class MapHydrator(Hydrator):
        def start(self):
            return {}

        def add(self, target, heading, value):
            r = dict(target)
            r[heading] = value
            return r

        def finish(self, target):
            return target

    path = str(tmp_path / "foo.parquet")
    w = W.ParquetWriter.writeFile(sch, path, Deh(), decoder=dec)
    w.write([1, "hello1@example.com"])
    w.write([2, "hello2@example.com"])
    w.close()
    rows = list(ParquetReader.streamContent(path, HydratorSupplier.constantly(MapHydrator())))
    assert {"id": 1, "email": "hello1@example.com"} in rows and {"id": 2, "email": "hello2@example.com"} in rows
    rows = list(ParquetReader.streamContent(path, HydratorSupplier.constantly(MapHydrator()), ["id"]))
    assert {"id": 1} in rows and {"id": 2} in rows
    with pytest.raises(NotImplementedError):
        bad = W.MessageType("bad", W.required(W.BINARY).named("raw"))

        class D2(W.Dehydrator):
            def dehydrate(self, record, vw):
                vw.write("raw", record)

        w2 = W.ParquetWriter.writeFile(bad, str(tmp_path / "bad.parquet"), D2(), decoder=dec)
        try:
            w2.write(b"x")
        finally:
            w2.buf.take()
            w2.close()


def test_parallel_column_encoding(dec, oracle, tmp_path):
    """ParquetWriter(decoders=[...]): columns encoded concurrently on several contexts, chunks
    appended in schema order; the file equals the single-context file byte for byte."""
    from pfloor.decoder import GpuDecoder
    from pfloor.writer import ParquetWriter
    n = 40000
    cols, _p, _s = _config1(n, 3)
    p1, p2 = str(tmp_path / "one.parquet"), str(tmp_path / "par.parquet")
    w = ParquetWriter(_schema(), p1, None, decoder=dec)
    w.write_columns(cols, n)
    w.close()
    extra = [GpuDecoder(0), GpuDecoder(0)]
    try:
        w = ParquetWriter(_schema(), p2, None, decoders=[dec] + extra)
        w.write_columns(cols, n)
        w.write_columns(cols, n)
        w.close()
        assert w.kernel_ms["snappy_in"] > 0 and w.kernel_ms["snappy"] > 0
    finally:
        for d in extra:
            d.close()
    b1, b2 = open(p1, "rb").read(), open(p2, "rb").read()
    # the parallel file holds the same row group twice: its first row group's bytes equal the serial file's
    assert b2[:len(b1) - 8 - int.from_bytes(b1[-8:-4], "little")] == b1[:len(b1) - 8 - int.from_bytes(b1[-8:-4], "little")]
    with oracle.open(p2) as of:
        assert of.num_row_groups == 2
        for rg in range(2):
            a = of.decode(rg, 0)
            assert np.array_equal(np.frombuffer(a["values"].tobytes(), np.int64), cols["id"])


def test_write_config4_shape(dec, oracle, tmp_path):
    """Config-4-shaped columns through the writer: nullable INT32 / FLOAT, 30 % nulls, values from
    100K-value pools (dictionary ~400 KB, ids of 17 bits), plus NaN payloads kept bit-exact
    (raw-bit dictionary keys); read back by the oracle, pyarrow and the GPU reader.
    DELIBERATE DIVERGENCE (parity unpinned): parquet-mr writes FLOAT / DOUBLE through
    floatToIntBits / doubleToLongBits, which canonicalise NaN payloads in PLAIN and dictionary pages
    alike; this writer keeps the payload bits. The assertion below pins this writer's behaviour,
    not the reference's."""
    pq = pytest.importorskip("pyarrow.parquet")
    from pfloor import writer as W
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(4)
    n, ncol = 200003, 6
    fields, cols, exp = [], {}, {}
    for k in range(ncol):
        t = W.INT32 if k % 2 == 0 else W.FLOAT
        pool = rng.integers(-2**31, 2**31 - 1, 100000, dtype=np.int64).astype(np.int32)
        if t == W.FLOAT:
            pool = pool.view(np.float32).copy()
            pool[:3] = np.array([0x7fc00001, 0x7fc00002, 0xffc00000], np.uint32).view(np.float32)   # NaN payloads
        vals = pool[rng.integers(0, 100000, n)]
        present = rng.random(n) >= 0.3
        vals = np.where(present, vals, np.zeros(1, vals.dtype))
        name = f"c{k}"
        fields.append(W.optional(t).named(name))
        cols[name] = (vals, np.packbits(present, bitorder="little"))
        exp[k] = (vals, present)
    path = str(tmp_path / "c4.parquet")
    w = W.ParquetWriter(W.MessageType("wide", *fields), path, None, decoder=dec)
    w.write_columns(cols, n)
    encs = list(w.last_chunks)
    w.close()
    assert all(e[1] == 8 for e in encs), encs
    got = decode_file(path, decoder=dec)
    assert got["_status"] == 0, got["_error"]
    with oracle.open(path) as of:
        for k in range(ncol):
            g = got[(0, k)]
            assert_chunk_equal(g, of.decode(0, k), f"c4 col {k}")
            vals, present = exp[k]
            gv = np.frombuffer(g["values"].tobytes(), np.uint32)
            assert np.array_equal(gv[present], vals.view(np.uint32)[present])
            assert np.array_equal(np.unpackbits(g["validity"], bitorder="little")[:n].astype(bool), present)
    t = pq.read_table(path)
    assert t.column("c0").null_count == int((~exp[0][1]).sum())
