"""K1 (Snappy) on the GPU in isolation: known-answer vectors (pyarrow's Google Snappy), seeded
multi-block streams from the oracle's test compressor (Google-style 64 KiB blocks -> the
block-parallel path; cross-block streams -> the whole-page re-run), and corrupt streams.
pf_snappy_last_fallback: 0 block-parallel, 1 whole page in one executor wave, 2 pieces re-run as
one (block assumption broken), 3 serial kernel (stream not indexable / corrupt)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    from pfloor.decoder import GpuDecoder
    d = GpuDecoder(0)
    yield d
    d.close()


def _payloads(rng):
    words = [b"alpha ", b"beta ", b"gamma ", b"delta ", b"ironic ", b"deposits ", b"packages "]
    text = b"".join(words[i] for i in rng.integers(0, len(words), 60000))
    ints = np.cumsum(rng.integers(0, 9, 120000)).astype(np.int64).tobytes()
    rnd = rng.integers(0, 256, 200000, dtype=np.uint8).tobytes()
    runs = b"".join(bytes([int(b)]) * int(k) for b, k in zip(rng.integers(0, 4, 4000), rng.integers(1, 300, 4000)))
    mixed = b"".join((rng.integers(0, 256, int(rng.integers(1, 80)), dtype=np.uint8).tobytes() if rng.random() < 0.3
                      else words[int(rng.integers(0, 7))] * int(rng.integers(1, 20))) for _ in range(6000))
    # dense chains of dependent copies (offset 4/8 copies between 1-3 byte literals)
    stride = np.arange(0, 7 * 90000, 7, dtype=np.int64).tobytes()
    small = (np.arange(150000, dtype=np.int32) // 3).tobytes()
    return {"text": text, "ints": ints, "stride": stride, "small": small, "random": rnd, "runs": runs, "mixed": mixed, "tiny": b"ab", "empty": b""}


def test_known_answer_vectors(dec, oracle):
    z = np.load(os.path.join(GOLDEN, "snappy_kat.npz"), allow_pickle=False)
    for name in sorted({k.rsplit("_", 1)[0] for k in z.files}):
        raw, comp = z[name + "_raw"].tobytes(), z[name + "_comp"].tobytes()
        got, fb = dec.snappy_decompress(comp)
        assert got == raw, name
        assert fb == 0, f"{name}: Google Snappy stream should take the block-parallel path"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_block_parallel_path(dec, oracle, seed):
    rng = np.random.default_rng(seed)
    for name, data in _payloads(rng).items():
        comp = oracle.snappy_compress(data, mode=0)
        got, fb = dec.snappy_decompress(comp)
        assert got == data, (name, len(data))
        assert fb == 0, name


def test_unaligned_stream_single_piece(dec, oracle):
    """No token at the 64 KiB marks: the page decodes as one piece (copies may reach far back)."""
    rng = np.random.default_rng(7)
    data = _payloads(rng)["text"] * 3
    got, fb = dec.snappy_decompress(oracle.snappy_compress(data, mode=1))
    assert got == data and fb == 0


def test_cross_block_streams_fall_back(dec, oracle):
    """Tokens aligned to 64 KiB but copies reaching into earlier blocks: pieces are not
    independent, so the page is re-run as one piece — and still bit-exact."""
    rng = np.random.default_rng(7)
    data = _payloads(rng)["text"] * 3
    comp = oracle.snappy_compress(data, mode=2)
    got, fb = dec.snappy_decompress(comp)
    assert got == data
    assert fb == 2


def _boundary_streams(seed):
    """Streams whose sizes straddle the 8 KiB index windows and 64 KiB pieces at many offsets,
    mixing long literals (windows jumped over entirely) and dense short copies."""
    rng = np.random.default_rng(seed)
    pl = _payloads(rng)
    for size in (8191, 8192, 8193, 65535, 65536, 65537, 131072 + 5, 300001):
        parts, total = [], 0
        while total < size:
            kind = ("random", "text", "runs", "mixed", "ints")[int(rng.integers(0, 5))]
            src = pl[kind]
            a = int(rng.integers(0, len(src) - 1))
            piece = src[a:a + int(rng.integers(1, 40000))]
            parts.append(piece)
            total += len(piece)
        yield size, b"".join(parts)[:size]


@pytest.mark.parametrize("seed", [11, 12])
def test_window_boundaries(dec, oracle, seed):
    for size, data in _boundary_streams(seed):
        got, fb = dec.snappy_decompress(oracle.snappy_compress(data, mode=0))
        assert got == data, (size, seed)
        assert fb == 0, (size, seed)


def _far_after_literal(seed):
    """Long literals (incompressible runs) each followed by copies of their own bytes 3.3-4.1 KiB
    back: the first token after a long literal is a far copy whose source the executor is still
    writing (exec5 waits one batch for those stores to land), then dense near copies."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    while len(out) < 300_000:
        lit = rng.integers(0, 256, int(rng.integers(4200, 9000)), dtype=np.uint8).tobytes()
        out += lit
        for _ in range(int(rng.integers(1, 6))):
            back = int(rng.integers(3300, 4100))
            ln = int(rng.integers(4, 64))
            out += out[len(out) - back:len(out) - back + ln]
        out += (np.arange(int(rng.integers(100, 3000)), dtype=np.int32) // 3).tobytes()
    return bytes(out)


@pytest.mark.parametrize("executor", ["5", "2"])
def test_executors_agree(oracle, switches, executor):
    """Both block-parallel executors (default 5: producer / consumer waves; the diagnostics
    build's PF_EXEC=2: one wave per piece) on the seeded payloads and on far copies right after long
    literals."""
    from pfloor.decoder import GpuDecoder
    rng = np.random.default_rng(11)
    cases = dict(_payloads(rng), far1=_far_after_literal(1), far2=_far_after_literal(2))
    with switches(PF_EXEC=executor), GpuDecoder(0) as dec:
        for name, data in cases.items():
            got, fb = dec.snappy_decompress(oracle.snappy_compress(data, mode=0))
            assert got == data, (executor, name, len(data))
            assert fb == 0, (executor, name)


def _far_dense(seed):
    """Copies of 10-30 bytes from 4-12 KiB back, several dozen per executor batch: every batch's far-copy
    slots fill (the producer cuts at XFAR), at every source alignment."""
    rng = np.random.default_rng(seed)
    out = bytearray(rng.integers(0, 256, 12288, dtype=np.uint8).tobytes())
    while len(out) < 200_000:
        back = int(rng.integers(4096, 12288))
        ln = int(rng.integers(10, 31))
        out += out[len(out) - back:len(out) - back + ln]
        out += bytes([int(rng.integers(0, 256))])   # (a literal byte between the copies)
    return bytes(out)


def _periodic_all_offsets(seed):
    """Runs of period 1-200 (copies that overlap their own output, offsets 1..200, lengths to 64):
    the consumer's source arithmetic floor(j / offset) for every j < 64."""
    rng = np.random.default_rng(seed)
    parts = []
    for per in list(range(1, 201)) * 2:
        unit = rng.integers(0, 256, per, dtype=np.uint8).tobytes()
        parts.append(unit * (int(rng.integers(130, 400)) // per + 2))
    return b"".join(parts)


def test_executor_far_slots_and_periodic_copies(dec, oracle):
    for name, data in (("far_dense", _far_dense(3)), ("periodic", _periodic_all_offsets(4))):
        got, fb = dec.snappy_decompress(oracle.snappy_compress(data, mode=0))
        assert got == data, (name, len(data))
        assert fb == 0, name
