"""GPU parity: the HIP path (through the C ABI) against the golden vectors AND the CPU oracle,
bit-exact, for every fixture (configs 1-5 shapes + edge cases), plus corrupt-input behaviour."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from golden_util import assert_chunk_equal, load_expected

pytestmark = pytest.mark.gpu

# Encodings the HIP path does not decode (none at present): chunks using them must fail loudly
# with PF_ERR_UNSUPPORTED_ENCODING (-3), never return wrong data.
UNSUPPORTED = set()


@pytest.fixture(scope="module")
def decoder():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


@pytest.mark.parametrize("name", golden_files())
def test_gpu_matches_golden_and_oracle(decoder, oracle, name):
    from pfloor.decoder import decode_file
    import json
    path = os.path.join(GOLDEN, name + ".parquet")
    exp = load_expected(name)
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    encs = {(c["rg"], c["col"]): set(c["encodings"]) for f in man["files"] if f["file"] == name + ".parquet"
            for c in f["chunks"]}
    got = decode_file(path, decoder=decoder)
    with oracle.open(path) as of:
        for key, e in sorted(exp.items()):
            g = got[key]
            label = f"{name} rg{key[0]} c{key[1]} {e['path']}"
            if encs[key] & UNSUPPORTED:
                assert g["status"] == -3, label
                continue
            assert g["status"] == 0, (label, got["_error"])
            assert_chunk_equal(g, e, label + " [golden]")
            o = of.decode(*key)
            assert_chunk_equal(g, o, label + " [oracle]")


def test_reference_roundtrip_rows():
    """ParquetReadWriteTest.java:66-82 through the host mirror of ParquetReader/Hydrator."""
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader

    class MapHydrator(Hydrator):
        def start(self):
            return {}

        def add(self, target, heading, value):
            r = dict(target)
            r[heading] = value
            return r

        def finish(self, target):
            return target

    path = os.path.join(GOLDEN, "ref_roundtrip.parquet")
    with ParquetReader.streamContent(path, HydratorSupplier.constantly(MapHydrator())) as s:
        result = s.collect()
    assert {"id": 1, "email": "hello1"} in result
    assert {"id": 2, "email": "hello2"} in result
    with ParquetReader.streamContent(path, HydratorSupplier.constantly(MapHydrator()), {"id"}) as s:
        result = s.collect()
    assert {"id": 1} in result and {"id": 2} in result


def test_reader_rows_match_oracle_flat(oracle):
    """Row-by-row Hydrator values for config-1 shape with nulls, against the oracle."""
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader

    class ListHydrator(Hydrator):
        def start(self):
            return []

        def add(self, t, h, v):
            t.append((h, v))
            return t

        def finish(self, t):
            return tuple(t)

    path = os.path.join(GOLDEN, "c1_flat_snappy_v2.parquet")
    with ParquetReader.streamContent(path, HydratorSupplier.constantly(ListHydrator())) as s:
        rows = s.collect()
    with oracle.open(path) as of:
        ids, xs, ns, ss = [], [], [], []
        for rg in range(of.num_row_groups):
            a = of.decode(rg, 0); b = of.decode(rg, 1); c = of.decode(rg, 2); d = of.decode(rg, 3)
            ids += a["values"].view(np.int64).tolist()
            xs += b["values"].view(np.float64).tolist()
            valid = np.unpackbits(c["validity"], bitorder="little")[:c["num_slots"]]
            ns += [int(v) if ok else None for v, ok in zip(c["values"].view(np.int32), valid)]
            o, ch = d["offsets"], d["chars"].tobytes()
            ss += [ch[o[i]:o[i + 1]].decode() for i in range(d["num_slots"])]
    assert len(rows) == len(ids)
    for r, i, x, n, s in zip(rows, ids, xs, ns, ss):
        assert r == (("id", i), ("x", x), ("n", n), ("s", s))


def test_unexpected_repetition():
    """Lists with >= 2 elements make the reference throw (ParquetReader.java:199-202)."""
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader

    class H(Hydrator):
        def start(self):
            return {}

        def add(self, t, h, v):
            return t

        def finish(self, t):
            return t

    path = os.path.join(GOLDEN, "list_prim.parquet")
    with pytest.raises(RuntimeError, match="Failed to read parquet") as ei:
        with ParquetReader.streamContent(path, HydratorSupplier.constantly(H())) as s:
            s.collect()
    assert "Unexpected repetition" in repr(ei.value.__cause__)


def _corrupt_variants(data, rng, n=12):
    out = []
    for _ in range(n):
        b = bytearray(data)
        k = int(rng.integers(8, len(b) - 8))
        for j in range(int(rng.integers(1, 16))):
            if k + j < len(b) - 8:
                b[k + j] = int(rng.integers(0, 256))
        out.append(bytes(b))
    return out


def test_corrupt_pages_error_not_fault(decoder, tmp_path):
    """Random byte damage inside page bodies: each chunk either decodes or reports an error;
    the GPU never faults and the context stays usable."""
    from pfloor.decoder import decode_file
    rng = np.random.default_rng(3)
    for name in ("c2_lineitem", "c5_nested", "c1_flat_none_v1", "edge_encodings"):
        data = open(os.path.join(GOLDEN, name + ".parquet"), "rb").read()
        for i, bad in enumerate(_corrupt_variants(data, rng, 6)):
            p = tmp_path / f"{name}_{i}.parquet"
            p.write_bytes(bad)
            try:
                got = decode_file(str(p), decoder=decoder)
            except Exception:
                continue   # metadata-level rejection on the host
            for k, v in got.items():
                if isinstance(k, tuple):
                    assert v["status"] in (0, -2, -3, -6), v["status"]
    # still healthy afterwards
    got = decode_file(os.path.join(GOLDEN, "ref_roundtrip.parquet"), decoder=decoder)
    assert got["_status"] == 0


def _big_file(tmp_path, rows, nulls):
    """pyarrow-written file with pages of 20K entries (> one k_flat block of 4096), a dictionary
    column in RLE runs of 9 (> RUN_CAP runs per block: windowed run tables), PLAIN and dictionary
    strings, doubles and an INT64 key; generated at test time (pyarrow is in the image)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(11)
    key = np.arange(rows, dtype=np.int64) // 3
    runs = (np.repeat(np.arange(rows // 9 + 1) % 50, 9)[:rows]).astype(np.int32)
    dbl = rng.random(rows)
    vocab = np.array([f"w{i:05d}" * (1 + i % 4) for i in range(700)])
    sdict = vocab[rng.integers(0, 700, rows)]
    text = np.array([f"comment {i} " + "x" * int(rng.integers(0, 30)) for i in range(rows)])
    cols = {"key": key, "runs": runs, "dbl": dbl, "sdict": sdict, "text": text}
    arrays = {}
    for k, v in cols.items():
        mask = (rng.random(rows) < 0.3) if nulls else None
        arrays[k] = pa.array(v, mask=mask)
    t = pa.table(arrays)
    path = str(tmp_path / f"big_{rows}_{int(nulls)}.parquet")
    pq.write_table(t, path, compression="snappy", row_group_size=rows // 2,
                   use_dictionary=["runs", "sdict", "key"], data_page_size=1 << 20)
    return path


@pytest.mark.parametrize("nulls", [False, True])
def test_gpu_multiblock_pages_match_oracle(decoder, oracle, tmp_path, nulls):
    from pfloor.decoder import decode_file
    path = _big_file(tmp_path, 120000, nulls)
    got = decode_file(path, decoder=decoder)
    with oracle.open(path) as of:
        for rg in range(of.num_row_groups):
            for c in range(of.num_columns):
                g = got[(rg, c)]
                assert g["status"] == 0, (rg, c, got["_error"])
                assert_chunk_equal(g, of.decode(rg, c), f"big rg{rg} c{c} nulls={nulls}")


def test_shared_stream_contexts_pipelined(oracle):
    """pf_ctx_create_shared: two contexts on one HIP stream, row group i+1 enqueued on one while
    row group i still decodes on the other (the bench's pipelined steps, a reader's prefetch).
    Every row group decoded this way is bit-exact vs the oracle; pf_wait on one context returns
    its own results; timing off gives PF_ERR_STATE from pf_last_timing; destroying the first
    context leaves the shared stream usable by the second."""
    from pfloor import _native
    from pfloor.decoder import GpuDecoder, ParquetFile, PinnedBuffer
    path = os.path.join(GOLDEN, "c2_lineitem.parquet")
    a = GpuDecoder(0)
    b = GpuDecoder(share=a)
    pair = (a, b)
    with ParquetFile(path) as pf, oracle.open(path) as of:
        cols = list(range(pf.num_columns))
        seq = [rg for _ in range(3) for rg in range(pf.num_row_groups)]
        bufs = []
        for rg in range(pf.num_row_groups):
            items, total = pf.plan([rg], cols)
            buf = PinnedBuffer(a.h, max(total, 1))
            descs = []
            for _rg, col, s, n, off in items:
                if n:
                    pf.read_into(s, n, buf.ptr.value + off)
                descs.append(pf.chunk_desc(_rg, col, off))
            bufs.append((items, descs, buf, max(total, 1)))
        for d in pair:
            d.set_timing(False)

        def check(d, rg):
            items = bufs[rg][0]
            for i, (_rg, col, *_r) in enumerate(items):
                c = pf.columns[col]
                g = d.fetch(i, c.physical_type, c.max_def, c.max_rep)
                assert g["status"] == 0
                assert_chunk_equal(g, of.decode(_rg, col), f"pipelined rg{_rg} c{col}")

        for k, rg in enumerate(seq):
            items, descs, buf, nb = bufs[rg]
            pair[k % 2].decode(descs, buf.ptr.value, nb)
            if k > 0:
                d = pair[(k - 1) % 2]
                assert d.wait() == 0, d.error()
                check(d, seq[k - 1])
        d = pair[(len(seq) - 1) % 2]
        assert d.wait() == 0, d.error()
        check(d, seq[-1])
        with pytest.raises(_native.PfError):
            a.timing()
        a.set_timing(True)
        a.close()   # b still owns the stream
        items, descs, buf, nb = bufs[0]
        b.decode(descs, buf.ptr.value, nb)
        assert b.wait() == 0, b.error()
        check(b, 0)
        for *_x, buf, _n in bufs:
            buf.free()
    b.close()


@pytest.mark.parametrize("pageable", [False, True])
@pytest.mark.parametrize("name", golden_files())
def test_batch_copy_matches_per_chunk_copy(decoder, oracle, name, pageable):
    """pf_copy_batch_async (one D2H per output arena) + pf_column_info_host give the same arrays
    as pf_copy_column per chunk, and both match the oracle (E2E path of bench.py). A mapped pinned
    buffer is written by the library's download kernel on its copy stream; an ordinary host array
    takes the SDMA copies (round 6)."""
    from pfloor.decoder import ParquetFile
    path = os.path.join(GOLDEN, name + ".parquet")
    with ParquetFile(path) as pf, oracle.open(path) as of:
        items, total = pf.plan(list(range(pf.num_row_groups)), list(range(pf.num_columns)))
        buf = decoder.staging(total)
        descs = []
        for rg, col, s, n, off in items:
            if n:
                pf.read_into(s, n, buf.ptr.value + off)
            descs.append(pf.chunk_desc(rg, col, off))
        decoder.decode(descs, buf.ptr.value, max(total, 1))
        rc = decoder.wait()
        types = [(pf.columns[col].physical_type, pf.columns[col].max_def, pf.columns[col].max_rep)
                 for _rg, col, *_r in items]
        got = decoder.fetch_batch(types, pageable=pageable)
        for i, (rg, col, *_r) in enumerate(items):
            one = decoder.fetch(i, *types[i])
            assert got[i]["status"] == one["status"]
            if one["status"] != 0:
                assert rc != 0
                continue
            assert_chunk_equal(got[i], one, f"{name} rg{rg} c{col} [batch vs chunk]")
            assert_chunk_equal(got[i], of.decode(rg, col), f"{name} rg{rg} c{col} [batch vs oracle]")


@pytest.mark.parametrize("name", ["c1_flat_snappy_v2", "c2_lineitem", "edge_types_v1"])
def test_reader_multi_device_rows_in_order(oracle, name):
    """Row groups dealt round-robin over several devices (two contexts on the visible GPU stand in
    for two GPUs, each with two pipelined contexts) come back as the single-device reader's rows,
    in file order (ParquetReader.java:176-212, :225-227), and match the oracle's values."""
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader

    class ListHydrator(Hydrator):
        def start(self):
            return []

        def add(self, t, h, v):
            t.append((h, v))
            return t

        def finish(self, t):
            return tuple(t)

    path = os.path.join(GOLDEN, name + ".parquet")
    with ParquetReader.streamContent(path, HydratorSupplier.constantly(ListHydrator())) as s:
        one = s.collect()
    with ParquetReader.streamContent(path, HydratorSupplier.constantly(ListHydrator()), devices=[0, 0]) as s:
        two = s.collect()
    assert len(one) == len(two) and len(one) > 0
    # NaN-safe comparison of the value sequences (doubles compared bit-exactly)
    import struct as _st

    def key(v):
        return ("f", _st.pack("<d", v)) if isinstance(v, float) else v
    assert [tuple((h, key(v)) for h, v in r) for r in one] == [tuple((h, key(v)) for h, v in r) for r in two]
    # the first column's values against the oracle, in file order
    with oracle.open(path) as of:
        vals = []
        for rg in range(of.num_row_groups):
            a = of.decode(rg, 0)
            valid = (np.unpackbits(a["validity"], bitorder="little")[:a["num_slots"]] if a.get("validity") is not None
                     else np.ones(a["num_slots"], np.uint8))
            if "offsets" in a:
                o, ch = a["offsets"], a["chars"].tobytes()
                vals += [ch[o[i]:o[i + 1]] if ok else None for i, ok in zip(range(a["num_slots"]), valid)]
            else:
                w = a["values"].nbytes // max(a["num_slots"], 1)
                raw = a["values"].tobytes()
                vals += [raw[i * w:(i + 1) * w] if ok else None for i, ok in enumerate(valid)]
    assert len(vals) == len(two)
    first = [r[0][1] for r in two]
    assert [v is None for v in first] == [v is None for v in vals]


def test_reader_multi_device_error_at_its_row_group(tmp_path):
    """A damaged chunk in row group 2 fails the read when row group 2 is reached, even though the
    pipeline decoded it ahead; the rows of row groups 0 and 1 come out first."""
    from pfloor.decoder import ParquetFile
    from pfloor.reader import Hydrator, HydratorSupplier, ParquetReader

    class H(Hydrator):
        def start(self):
            return []

        def add(self, t, h, v):
            return t

        def finish(self, t):
            return 1

    src = os.path.join(GOLDEN, "c1_flat_snappy_v2.parquet")
    data = bytearray(open(src, "rb").read())
    with ParquetFile(src) as pf:
        rows01 = pf.row_group_rows(0) + pf.row_group_rows(1)
        s, n = pf.chunk_range(2, 0)
        d = pf.chunk_desc(2, 0, 0)
        pg = d.pages[d.n_pages - 1]
        # overwrite a data page body with garbage: the Snappy stream / values become invalid
        for k in range(pg.offset + 1, min(pg.offset + pg.compressed_size, n)):
            data[s + k] = 0xff
    bad = tmp_path / "bad_rg2.parquet"
    bad.write_bytes(bytes(data))
    got = 0
    with pytest.raises(RuntimeError, match="Failed to read parquet"):
        with ParquetReader.streamContent(str(bad), HydratorSupplier.constantly(H()), devices=[0, 0]) as s:
            for _ in s:
                got += 1
    assert got == rows01


@pytest.mark.parametrize("kind", ["string", "int64"])
def test_dictionary_ids_out_of_range(decoder, oracle, tmp_path, kind):
    """Ids past the dictionary in a flat dictionary data page (0xff bytes written over an uncompressed v2
    page's bit-packed ids, 10-bit ids into 700 entries): the oracle reports the chunk; the GPU must too,
    from whichever kernel sees it first (strings: k_count_dict marks its block and k_count reports the
    page, round 5; fixed width: k_flat_fixed's id check), without a fault; a clean column of the same
    batch stays bit-exact."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from pfloor.decoder import ParquetFile, decode_file
    rng = np.random.default_rng(29)
    n = 60_000
    vocab = np.array([f"v{i:04d}" * (1 + i % 3) for i in range(700)]) if kind == "string" else \
        (np.arange(700, dtype=np.int64) * 7919)
    t = pa.table({"d": pa.array(vocab[rng.integers(0, 700, n)]), "k": pa.array(np.arange(n, dtype=np.int64))})
    path = str(tmp_path / f"badids_{kind}.parquet")
    pq.write_table(t, path, compression="NONE", data_page_version="2.0", use_dictionary=["d"], row_group_size=n)
    data = bytearray(open(path, "rb").read())
    with ParquetFile(path) as pf:   # (the page descriptors live in the handle: read them inside)
        start, _ = pf.chunk_range(0, 0)
        d = pf.chunk_desc(0, 0, 0)
        dp = [(d.pages[i].offset, d.pages[i].rep_bytes, d.pages[i].def_bytes) for i in range(d.n_pages)
              if d.pages[i].page_type in (0, 3)]
    assert dp
    off, rep_b, def_b = dp[0]
    vals = start + off + rep_b + def_b   # v2: [rep][def][values]; values: the bit width, then the runs
    assert data[vals] == 10, data[vals]
    for i in range(vals + 40, vals + 120):
        data[i] = 0xFF
    bad = tmp_path / f"badids_{kind}_bad.parquet"
    bad.write_bytes(bytes(data))
    with oracle.open(str(bad)) as of:
        assert of.decode(0, 0)["status"] != 0
        good = of.decode(0, 1)
    got = decode_file(str(bad), decoder=decoder)
    assert got[(0, 0)]["status"] != 0, "ids past the dictionary not reported"
    assert got[(0, 1)]["status"] == 0
    assert_chunk_equal(got[(0, 1)], good, "clean column next to the damaged one")
