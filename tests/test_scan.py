"""Page-header scan + page CRC32 (pf_scan_pages): the per-page Thrift walk of
parquet-mr's ParquetFileReader.readNextRowGroup (called at ParquetReader.java:183) and its
usePageChecksumVerification check, on the GPU.

CPU: the oracle's CRC32 against zlib (the algorithm java.util.zip.CRC32 implements) and the
known answer of "123456789"; the oracle's page walk against the host walk (pf_file_chunk_desc) and
against pyarrow's page_checksum_verification verdict on damaged files (pyarrow wrote the checksums:
tests/golden/crc/make_golden_crc.py). GPU: pf_scan_pages against both, on every golden file."""
import ctypes as C
import os
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, golden_files

PAGE_FIELDS = ("offset", "compressed_size", "uncompressed_size", "page_type", "encoding", "def_encoding",
               "rep_encoding", "num_values", "num_nulls", "num_rows", "def_bytes", "rep_bytes", "is_compressed")
CRC_FILES = ("crc_pages", "crc_pages_v2")


def _chunks(path):
    """Every chunk of the file: (bytes, [(offset, size, num_values)], host page descs, (rg, col))."""
    from pfloor.decoder import ParquetFile
    with ParquetFile(path) as pf:
        blob = bytearray()
        items, host, keys = [], [], []
        for rg in range(pf.num_row_groups):
            for col in range(pf.num_columns):
                s, n = pf.chunk_range(rg, col)
                b = np.zeros(max(n, 1), np.uint8)
                pf.read_into(s, n, b.ctypes.data)
                off = len(blob)
                blob += b[:n].tobytes() + bytes((-n) % 64 + 3)   # odd padding: unaligned chunk starts
                d = pf.chunk_desc(rg, col, 0)
                pages = [{f: getattr(d.pages[i], f) for f in PAGE_FIELDS} for i in range(d.n_pages)]
                nv = sum(p["num_values"] for p in pages if p["page_type"] != 2)
                items.append((off, n, nv))
                host.append(pages)
                keys.append((rg, col))
    return bytes(blob), items, host, keys


def test_crc32_matches_zlib(oracle):
    assert oracle.crc32(b"123456789") == 0xCBF43926
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 64, 1000, 65537):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.crc32(d) == zlib.crc32(d)


@pytest.mark.parametrize("name", CRC_FILES)
def test_oracle_page_walk_and_crc(oracle, name):
    path = os.path.join(GOLDEN, "crc", name + ".parquet")
    data, items, host, keys = _chunks(path)
    with oracle.open(path) as of:
        for (rg, col), hp in zip(keys, host):
            n, err, pages = of.chunk_pages(rg, col, verify_crc=True)
            assert n == len(hp) and err == -1, (rg, col)
            for p, h in zip(pages, hp):
                for f in ("offset", "compressed_size", "uncompressed_size", "page_type", "encoding", "num_values"):
                    assert p[f] == h[f], (rg, col, f)
                assert p["has_crc"] == 1 and p["crc_ok"] == 1


def _damage(path, which):
    """A copy of the file with one byte of one page body flipped, and the page's position."""
    from pfloor.decoder import ParquetFile
    raw = bytearray(open(path, "rb").read())
    with ParquetFile(path) as pf:
        rg, col, k = which
        s, _ = pf.chunk_range(rg, col)
        d = pf.chunk_desc(rg, col, 0)
        p = d.pages[k]
        raw[s + p.offset + p.compressed_size // 2] ^= 0x5A
    return bytes(raw)


def test_damaged_page_rejected_like_pyarrow(oracle, tmp_path):
    import pyarrow.parquet as pq
    path = os.path.join(GOLDEN, "crc", "crc_pages.parquet")
    bad = _damage(path, (1, 15, 3))
    f = tmp_path / "bad.parquet"
    f.write_bytes(bad)
    with pytest.raises(Exception):
        pq.read_table(f, page_checksum_verification=True)
    with oracle.open(data=bad) as of:
        n, err, _ = of.chunk_pages(1, 15, verify_crc=True)
        assert n == -2 and err == 3
        n, err, pages = of.chunk_pages(1, 15, verify_crc=False)
        assert n > 3 and pages[3]["crc_ok"] == 0


# ---------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def dec():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_files() + ["crc/" + f for f in CRC_FILES])
def test_gpu_scan_matches_host_walk(dec, oracle, name):
    path = os.path.join(GOLDEN, name + ".parquet")
    data, items, host, keys = _chunks(path)
    rc, res = dec.scan_pages(data, items, verify_crc=True)
    assert rc == 0
    with oracle.open(path) as of:
        for (rg, col), hp, (st, err, ncrc, pages) in zip(keys, host, res):
            assert st == 0 and err == -1
            assert pages == hp, (name, rg, col)
            n, _, op = of.chunk_pages(rg, col, verify_crc=True)
            assert n == len(pages)
            assert ncrc == sum(p["has_crc"] for p in op)


@pytest.mark.gpu
def test_gpu_crc_verified_and_damage_found(dec, oracle):
    path = os.path.join(GOLDEN, "crc", "crc_pages.parquet")
    data, items, host, keys = _chunks(path)
    rc, res = dec.scan_pages(data, items, verify_crc=True)
    assert rc == 0
    assert all(ncrc == len(pages) > 0 for _, _, ncrc, pages in res)
    # flip one byte in the body of page k of several chunks: exactly those chunks fail, at page k
    blob = bytearray(data)
    hits = {5: 2, 15: 6, 20: 0}
    for ci, k in hits.items():
        off, _, _ = items[ci]
        p = host[ci][k]
        blob[off + p["offset"] + p["compressed_size"] // 3] ^= 0x81
    rc, res = dec.scan_pages(bytes(blob), items, verify_crc=True)
    assert rc == -2
    for ci, (st, err, _, _) in enumerate(res):
        if ci in hits:
            assert (st, err) == (-2, hits[ci])
        else:
            assert st == 0
    rc, res = dec.scan_pages(bytes(blob), items, verify_crc=False)   # without verification: same pages
    assert rc == 0 and [r[3] for r in res] == host


@pytest.mark.gpu
def test_gpu_scan_corrupt_headers_error_not_fault(dec):
    path = os.path.join(GOLDEN, "c2_lineitem.parquet")
    data, items, host, keys = _chunks(path)
    rng = np.random.default_rng(11)
    for trial in range(40):
        blob = bytearray(data)
        ci = int(rng.integers(0, len(items)))
        off, n, _ = items[ci]
        # damage inside a page header (the bytes before a page body)
        k = int(rng.integers(0, len(host[ci])))
        body = host[ci][k]["offset"]
        pos = off + max(0, body - 1 - int(rng.integers(0, 12)))
        blob[pos] = int(rng.integers(0, 256))
        rc, res = dec.scan_pages(bytes(blob), items)
        st, err, _, pages = res[ci]
        if st == 0:
            assert sum(p["num_values"] for p in pages if p["page_type"] != 2) == items[ci][2]
        else:
            assert st == -2 and 0 <= err <= len(host[ci]) + 1
    # too few slots: capacity error
    rc, res = dec.scan_pages(data, items, page_cap=2)
    assert rc == -6 and any(r[0] == -6 for r in res)
