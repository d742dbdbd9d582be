"""Synthetic tables shaped like BASELINE.json's configs (pyarrow builders).

Used by bench.py (to write the lineitem-shaped SF1 input on the GPU box) and by
tests/golden/make_golden.py (fixtures). This module only *generates* files; the decode
path never imports pyarrow. All generators are seeded and vectorised.

Shapes:
  flat_table      config 1: id INT64 0..N-1, x DOUBLE U[0,1), n optional INT32 U[0,1000) 10% nulls,
                  s UTF8 from a 1,000-string vocabulary (len 8-24)
  lineitem_table  configs 2/3: TPC-H lineitem-shaped 16 columns
  wide_table      config 4: nullable INT32/FLOAT columns, 30% nulls, per-column value pools
  nested_table    config 5: l optional LIST<STRUCT<a INT64, b UTF8>>
"""
import numpy as np
import pyarrow as pa


def _strings_from_vocab(vocab, idx):
    """StringArray of vocab[idx] built from buffers (no Python loop over rows)."""
    vb = [v.encode() for v in vocab]
    lens = np.array([len(v) for v in vb], dtype=np.int64)
    starts = np.zeros(len(vb) + 1, dtype=np.int64)
    starts[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(vb), dtype=np.uint8)
    rl = lens[idx]
    offs = np.zeros(len(idx) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(rl)
    total = int(offs[-1])
    # byte gather: for every output byte, its source = starts[idx[row]] + (pos - offs[row])
    row_of_byte = np.repeat(np.arange(len(idx)), rl)
    src = starts[idx][row_of_byte] + (np.arange(total) - offs[:-1][row_of_byte])
    data = blob[src] if total else np.zeros(0, np.uint8)
    return pa.StringArray.from_buffers(len(idx), pa.py_buffer(offs.astype(np.int32).tobytes()),
                                       pa.py_buffer(data.tobytes()))


def _vocab(rng, n, lo, hi):
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
    out = set()
    while len(out) < n:
        ln = int(rng.integers(lo, hi + 1))
        out.add(letters[rng.integers(0, len(letters), ln)].tobytes().decode())
    return sorted(out)


def flat_table(n, seed=1):
    rng = np.random.default_rng(seed)
    vocab = _vocab(rng, 1000, 8, 24)
    nvals = rng.integers(0, 1000, n).astype(np.int32)
    nmask = rng.random(n) < 0.10
    schema = pa.schema([pa.field("id", pa.int64(), nullable=False),
                        pa.field("x", pa.float64(), nullable=False),
                        pa.field("n", pa.int32(), nullable=True),
                        pa.field("s", pa.string(), nullable=False)])
    return pa.table({"id": pa.array(np.arange(n, dtype=np.int64)),
                     "x": pa.array(rng.random(n)),
                     "n": pa.array(nvals, mask=nmask),
                     "s": _strings_from_vocab(vocab, rng.integers(0, len(vocab), n))}, schema=schema)


_WORDS = ("the quick brown fox jumps over lazy dog furiously regular accounts packages deposits ideas "
          "requests carefully slyly final blithely pending express instructions theodolites bold even "
          "special ironic silent foxes asymptotes pinto beans platelets dependencies courts").split()


def _comments(rng, n, lo=10, hi=43):
    """TPC-H-like comment text: 3-7 words from a small vocabulary, truncated to [lo, hi] chars."""
    words = [w.encode() for w in _WORDS]
    wl = np.array([len(w) + 1 for w in words], dtype=np.int64)      # word + trailing space
    wstart = np.zeros(len(words) + 1, dtype=np.int64)
    wstart[1:] = np.cumsum(wl)
    blob = np.frombuffer(b"".join(w + b" " for w in words), dtype=np.uint8)
    k = 7
    wi = rng.integers(0, len(words), (n, k))
    nw = rng.integers(3, k + 1, n)
    used = np.arange(k)[None, :] < nw[:, None]
    tl = np.where(used, wl[wi], 0)
    full = tl.sum(axis=1) - 1                                         # drop the final space
    rowlen = np.clip(full, 0, hi)
    # pad short rows by repeating: guarantee >= lo by adding words (rare); clip instead
    rowlen = np.maximum(rowlen, np.minimum(full, lo))
    # flat token stream
    flat_w = wi[used]
    flat_len = wl[flat_w]
    tok_off = np.zeros(len(flat_w) + 1, dtype=np.int64)
    tok_off[1:] = np.cumsum(flat_len)
    tok_of_byte = np.repeat(np.arange(len(flat_w)), flat_len)
    stream = blob[wstart[flat_w][tok_of_byte] + (np.arange(int(tok_off[-1])) - tok_off[:-1][tok_of_byte])]
    row_tok_start = np.zeros(n + 1, dtype=np.int64)
    row_tok_start[1:] = np.cumsum(nw)
    row_byte_start = tok_off[row_tok_start[:-1]]
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(rowlen)
    row_of_byte = np.repeat(np.arange(n), rowlen)
    data = stream[row_byte_start[row_of_byte] + (np.arange(int(offs[-1])) - offs[:-1][row_of_byte])]
    return pa.StringArray.from_buffers(n, pa.py_buffer(offs.astype(np.int32).tobytes()),
                                       pa.py_buffer(data.tobytes()))


def lineitem_table(n, seed=42, scale=None):
    """TPC-H lineitem-shaped table: 3 INT64 keys, 4 INT32
    (linenumber + 3 dates), 4 DOUBLE, 5 UTF8. Columns are pyarrow-default optional."""
    rng = np.random.default_rng(seed)
    sf = scale if scale is not None else max(1.0, n / 6001215.0)
    orders = max(1, n // 4)
    okey = np.sort(rng.integers(1, orders * 4 + 1, n)).astype(np.int64)
    pkey = rng.integers(1, int(200000 * sf) + 1, n).astype(np.int64)
    skey = rng.integers(1, int(10000 * sf) + 1, n).astype(np.int64)
    lnum = rng.integers(1, 8, n).astype(np.int32)
    qty = rng.integers(1, 51, n).astype(np.float64)
    price = np.round(qty * rng.uniform(900.0, 2000.0, n), 2)
    disc = rng.integers(0, 11, n) / 100.0
    tax = rng.integers(0, 9, n) / 100.0
    ship = rng.integers(8036, 8036 + 2526, n).astype(np.int32)
    commit = (ship + rng.integers(-60, 61, n)).astype(np.int32)
    receipt = (ship + rng.integers(1, 31, n)).astype(np.int32)
    return pa.table({
        "l_orderkey": okey, "l_partkey": pkey, "l_suppkey": skey, "l_linenumber": lnum,
        "l_quantity": qty, "l_extendedprice": price, "l_discount": disc, "l_tax": tax,
        "l_returnflag": _strings_from_vocab(["A", "N", "R"], rng.integers(0, 3, n)),
        "l_linestatus": _strings_from_vocab(["F", "O"], rng.integers(0, 2, n)),
        "l_shipdate": ship, "l_commitdate": commit, "l_receiptdate": receipt,
        "l_shipinstruct": _strings_from_vocab(["DELIVER IN PERSON", "COLLECT COD", "NONE", "TAKE BACK RETURN"],
                                              rng.integers(0, 4, n)),
        "l_shipmode": _strings_from_vocab(["REG AIR", "AIR", "RAIL", "SHIP", "TRUCK", "MAIL", "FOB"],
                                          rng.integers(0, 7, n)),
        "l_comment": _comments(rng, n),
    })


def wide_table(n, ncols=500, pool=100000, null_frac=0.3, seed=4):
    rng = np.random.default_rng(seed)
    cols = {}
    for c in range(ncols):
        mask = rng.random(n) < null_frac
        if c < ncols // 2:
            p = rng.integers(-2**31, 2**31 - 1, pool, dtype=np.int64).astype(np.int32)
            cols[f"i{c}"] = pa.array(p[rng.integers(0, pool, n)], mask=mask)
        else:
            p = rng.standard_normal(pool).astype(np.float32)
            cols[f"f{c}"] = pa.array(p[rng.integers(0, pool, n)], mask=mask)
    return pa.table(cols)


def nested_table(n, seed=5):
    """l optional LIST<STRUCT<a INT64, b UTF8>>: lengths U{0..4}, 10% null lists,
    5% null elements and 5% null leaves; a = running counter + small noise."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 5, n)
    null_list = rng.random(n) < 0.10
    lens = np.where(null_list, 0, lens)
    m = int(lens.sum())
    a = (np.arange(m, dtype=np.int64) * 7 + rng.integers(-3, 4, m)).astype(np.int64) + 10**12
    a_mask = rng.random(m) < 0.05
    vocab = ["red", "green", "blue", "cyan", "magenta", "yellow", "black", "white", "", "orange-ish"]
    b = _strings_from_vocab(vocab, rng.integers(0, len(vocab), m))
    b_mask = rng.random(m) < 0.05
    b = pa.array(b.to_pylist(), type=pa.string(), mask=b_mask)
    elem_mask = rng.random(m) < 0.05
    st = pa.StructArray.from_arrays([pa.array(a, mask=a_mask), b], names=["a", "b"],
                                    mask=pa.array(elem_mask))
    offs = np.zeros(n + 1, dtype=np.int32)
    offs[1:] = np.cumsum(lens)
    la = pa.ListArray.from_arrays(pa.array(offs), st, mask=pa.array(null_list))
    return pa.table({"l": la})


def list_prim_table(n, seed=9):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 6, n)
    null_list = rng.random(n) < 0.10
    lens = np.where(null_list, 0, lens)
    m = int(lens.sum())
    v = pa.array(rng.integers(-1000, 1000, m).astype(np.int32), mask=rng.random(m) < 0.1)
    offs = np.zeros(n + 1, dtype=np.int32)
    offs[1:] = np.cumsum(lens)
    return pa.table({"xs": pa.ListArray.from_arrays(pa.array(offs), v, mask=pa.array(null_list)),
                     "k": pa.array(np.arange(n, dtype=np.int64))})


def edge_types_table(n, seed=7):
    rng = np.random.default_rng(seed)
    fl = rng.standard_normal(n).astype(np.float32)
    fl[::97] = np.nan
    fl[1::89] = np.inf
    fl[2::83] = -0.0
    dl = rng.standard_normal(n)
    dl[::101] = np.frombuffer(np.array([0x7ff8dead00000001], dtype=np.uint64).tobytes(), dtype=np.float64)[0]
    ts = (rng.integers(-10**17, 10**17, n)).astype("datetime64[ns]")
    fixed = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(n)]
    binv = [rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes() for _ in range(n)]
    return pa.table({
        "flag": pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.2),
        "ts96": pa.array(ts, mask=rng.random(n) < 0.1),
        "fixed16": pa.array(fixed, type=pa.binary(16), mask=rng.random(n) < 0.1),
        "raw": pa.array(binv, type=pa.binary(), mask=rng.random(n) < 0.1),
        "all_null": pa.array([None] * n, type=pa.int32()),
        "const": pa.array(["k"] * n),
        "day": pa.array(rng.integers(-5000, 30000, n).astype(np.int32)).cast(pa.date32()),
        "f32": pa.array(fl),
        "f64": pa.array(dl),
        "req_bool": pa.array(rng.random(n) < 0.3),
    })


def edge_encodings_table(n, seed=8):
    rng = np.random.default_rng(seed)
    d32 = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    d32[: n // 3] = np.cumsum(rng.integers(-5, 50, n // 3)).astype(np.int32)
    d64 = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    d64[n // 2:] = np.cumsum(rng.integers(0, 1000, n - n // 2)).astype(np.int64)
    words = ["apple", "applesauce", "apply", "banana", "band", "bandana", "", "zz", "zebra" * 9]
    s1 = sorted(words[i] + str(j) for j, i in enumerate(rng.integers(0, len(words), n)))
    s2 = [words[i] * int(k) for i, k in zip(rng.integers(0, len(words), n), rng.integers(0, 3, n))]
    return pa.table({
        "d32": pa.array(d32, mask=rng.random(n) < 0.05),
        "d64": pa.array(d64),
        "dlba": pa.array(s2, mask=rng.random(n) < 0.05),
        "dba": pa.array(s1),
        "bss_f": pa.array(rng.standard_normal(n).astype(np.float32), mask=rng.random(n) < 0.1),
        "bss_d": pa.array(rng.standard_normal(n)),
        "bools": pa.array(rng.random(n) < 0.7),
    })
