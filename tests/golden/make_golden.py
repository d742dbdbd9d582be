#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Inputs  : small Parquet files shaped like BASELINE.json configs 1-5 plus edge cases, written
          by pyarrow 25.0.0 in the build container (the reference's own writer is Java/parquet-mr
          and cannot run here — see DESIGN.md "Oracle").
Expected: the decoded column chunks in the library's canonical layout (include/pfloor.h,
          pf_column_out), derived by pyarrow's reader — an implementation independent of
          both the oracle (oracle/pf_oracle.c) and the HIP path.  Stored as .npz
          (numpy, allow_pickle=False) next to each .parquet.
Also    : Snappy known-answer vectors produced by pyarrow's bundled Google Snappy.

The reference's only test (src/test/java/blue/strategic/parquet/ParquetReadWriteTest.java:28-83)
is mirrored by ref_roundtrip.parquet: required INT64 id + required UTF8 email, two rows,
SNAPPY + PARQUET_2_0 pages as the reference writer forces (ParquetWriter.java:65-66).

Run:  python tests/golden/make_golden.py      (pyarrow needed; never imported by product code)
"""
import json
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "parquet-floor_amd"))
from pfloor import datagen  # noqa: E402  (synthetic table builders shared with bench.py)


# ---------------------------------------------------------------- canonical expected layout
def _bits(mask):
    return np.packbits(np.asarray(mask, dtype=bool), bitorder="little")


def _fixed_bytes(arr, ptype, type_length):
    """Value bytes of a flat/child arrow array; null slots are zero."""
    n = len(arr)
    t = arr.type
    if ptype == 0:
        vals = np.array([1 if v else 0 for v in arr.to_pylist()], dtype=np.uint8) if n else np.zeros(0, np.uint8)
        return vals.tobytes()
    if ptype == 3:  # INT96 (from timestamp[ns]): nanos-of-day int64 LE + julian day int32 LE
        out = bytearray(12 * n)
        ns = arr.cast(pa.int64()).to_pylist()
        for i, v in enumerate(ns):
            if v is None:
                continue
            day, nod = divmod(v, 86400 * 10**9)
            out[12 * i:12 * i + 8] = int(nod).to_bytes(8, "little", signed=True)
            out[12 * i + 8:12 * i + 12] = int(day + 2440588).to_bytes(4, "little", signed=True)
        return bytes(out)
    if ptype == 7:
        out = bytearray(type_length * n)
        for i, v in enumerate(arr.to_pylist()):
            if v is not None:
                out[type_length * i:type_length * (i + 1)] = v
        return bytes(out)
    if pa.types.is_date32(t):
        arr = arr.cast(pa.int32())
    elif pa.types.is_timestamp(t) or pa.types.is_time64(t):
        arr = arr.cast(pa.int64())
    elif pa.types.is_time32(t):
        arr = arr.cast(pa.int32())
    np_t = {1: np.int32, 2: np.int64, 4: np.float32, 5: np.float64}[ptype]
    if n == 0:
        return b""
    if arr.null_count:
        # keep exact bits of valid values; zero the nulls
        buf = np.frombuffer(arr.buffers()[1], dtype=np_t, count=len(arr) + arr.offset)[arr.offset:].copy()
        buf[~np.asarray(arr.is_valid())] = 0
        return buf.tobytes()
    return np.frombuffer(arr.buffers()[1], dtype=np_t, count=len(arr) + arr.offset)[arr.offset:].tobytes()


def _binary(arr):
    offs = [0]
    chars = bytearray()
    for v in arr.to_pylist():
        if v is not None:
            chars += v.encode("utf-8") if isinstance(v, str) else bytes(v)
        offs.append(len(chars))
    return np.array(offs, dtype=np.int32), np.frombuffer(bytes(chars), dtype=np.uint8)


def _leaf_arrays(table_col, leaf_path):
    """Walk the arrow nesting of one top-level column down to the leaf named by leaf_path.
    Returns (kind, info): kind 'flat' -> leaf array; kind 'list' -> dict with list array and
    the leaf child array aligned with list elements."""
    arr = table_col.combine_chunks() if isinstance(table_col, pa.ChunkedArray) else table_col
    parts = leaf_path.split(".")[1:]
    if not parts:
        return "flat", arr
    if pa.types.is_struct(arr.type):
        return "struct", arr
    assert pa.types.is_list(arr.type), arr.type
    return "list", arr


def expected_for_column(tbl, meta, col_idx):
    """Canonical expected arrays for leaf column col_idx of one row group's table."""
    schema = meta.schema
    c = schema.column(col_idx)
    ptype = {"BOOLEAN": 0, "INT32": 1, "INT64": 2, "INT96": 3, "FLOAT": 4, "DOUBLE": 5,
             "BYTE_ARRAY": 6, "FIXED_LEN_BYTE_ARRAY": 7}[c.physical_type]
    tl = c.length if ptype == 7 else 0
    path = c.path
    top = path.split(".")[0]
    kind, arr = _leaf_arrays(tbl.column(top), path)
    out = {}
    if kind == "flat":
        n = len(arr)
        valid = np.asarray(arr.is_valid()) if n else np.zeros(0, bool)
        out["num_entries"] = n
        out["num_slots"] = n
        out["num_rows"] = n
        out["num_values"] = int(valid.sum())
        if c.max_definition_level > 0:
            out["validity"] = _bits(valid)
        if ptype == 6:
            o, ch = _binary(arr)
            out["offsets"], out["chars"] = o, ch
        else:
            out["values"] = np.frombuffer(_fixed_bytes(arr, ptype, tl), dtype=np.uint8)
        return out
    # list<...>: levels per Dremel shredding of one level of repetition
    assert c.max_repetition_level == 1, path
    sub = path.split(".")[1:]  # e.g. ['list', 'element', 'a'] or ['list', 'element']
    lst = arr
    elems = lst.flatten() if False else lst.values  # all elements incl. under null lists' ranges
    offsets = np.asarray(lst.offsets)
    list_valid = np.asarray(lst.is_valid())
    # element-level arrays
    if len(sub) == 3:  # list<struct<...>>
        struct_arr = elems
        field = struct_arr.type.get_field_index(sub[2])
        leaf = struct_arr.field(field)
        elem_valid = np.asarray(struct_arr.is_valid())
        # struct field validity does not include the parent's nulls
        leaf_valid = np.asarray(leaf.is_valid()) & elem_valid
    else:  # list<prim>
        leaf = elems
        elem_valid = np.ones(len(elems), bool)
        leaf_valid = np.asarray(leaf.is_valid())
    max_def = c.max_definition_level
    # def levels: 0 null list (if list optional) ... as computed from the schema
    defs, reps = [], []
    slot_idx = []  # element index per slot
    row_first = []
    list_null_def = max_def - (3 if len(sub) == 3 else 2) + 0
    for r in range(len(lst)):
        lo, hi = offsets[r], offsets[r + 1]
        if not list_valid[r]:
            defs.append(max_def - (4 if len(sub) == 3 else 3)); reps.append(0); continue
        if hi == lo:
            defs.append(max_def - (3 if len(sub) == 3 else 2)); reps.append(0); continue
        for j in range(lo, hi):
            reps.append(0 if j == lo else 1)
            if len(sub) == 3 and not elem_valid[j]:
                d = max_def - 2
            elif not leaf_valid[j]:
                d = max_def - 1
            else:
                d = max_def
            defs.append(d)
            slot_idx.append(j)
    del list_null_def, row_first
    slot_idx = np.array(slot_idx, dtype=np.int64)
    # list offsets in slots (elements under null/empty lists do not exist in parquet)
    lens = np.where(list_valid, offsets[1:] - offsets[:-1], 0)
    lo_out = np.zeros(len(lst) + 1, np.int32)
    lo_out[1:] = np.cumsum(lens)
    slot_leaf = leaf.take(pa.array(slot_idx)) if len(slot_idx) else leaf.slice(0, 0)
    slot_valid = leaf_valid[slot_idx] if len(slot_idx) else np.zeros(0, bool)
    if len(slot_idx) and not slot_valid.all():
        slot_leaf = pa.array(slot_leaf.to_pylist(), type=slot_leaf.type, mask=~slot_valid)
    out["num_entries"] = len(defs)
    out["num_slots"] = len(slot_idx)
    out["num_rows"] = len(lst)
    out["num_values"] = int(slot_valid.sum())
    out["validity"] = _bits(slot_valid)
    out["list_offsets"] = lo_out
    out["list_validity"] = _bits(list_valid)
    out["def_levels"] = np.array(defs, dtype=np.uint8)
    out["rep_levels"] = np.array(reps, dtype=np.uint8)
    if ptype == 6:
        o, ch = _binary(slot_leaf)
        out["offsets"], out["chars"] = o, ch
    else:
        out["values"] = np.frombuffer(_fixed_bytes(slot_leaf, ptype, tl), dtype=np.uint8)
    return out


def dump_expected(path):
    pf = pq.ParquetFile(path)
    meta = pf.metadata
    arrays = {}
    manifest = {"file": os.path.basename(path), "row_groups": meta.num_row_groups,
                "columns": meta.num_columns, "num_rows": meta.num_rows, "chunks": []}
    for g in range(meta.num_row_groups):
        tbl = pf.read_row_group(g)
        for ci in range(meta.num_columns):
            exp = expected_for_column(tbl, meta, ci)
            cm = meta.row_group(g).column(ci)
            manifest["chunks"].append({"rg": g, "col": ci, "path": cm.path_in_schema,
                                       "encodings": list(cm.encodings), "codec": cm.compression,
                                       **{k: int(v) for k, v in exp.items() if k.startswith("num_")}})
            for k, v in exp.items():
                if not k.startswith("num_"):
                    arrays[f"rg{g}_c{ci}_{k}"] = np.asarray(v)
    np.savez_compressed(path[:-len(".parquet")] + ".npz", **arrays)
    return manifest


# ---------------------------------------------------------------- fixture files
def write_all(out_dir):
    manifests = []

    def emit(name, table, **kw):
        p = os.path.join(out_dir, name + ".parquet")
        pq.write_table(table, p, **kw)
        manifests.append(dump_expected(p))

    # The reference test's file (ParquetReadWriteTest.java:32-35,61-64): SNAPPY + PARQUET_2_0.
    ref = pa.table({"id": pa.array([1, 2], pa.int64()), "email": pa.array(["hello1", "hello2"])},
                   schema=pa.schema([pa.field("id", pa.int64(), nullable=False),
                                     pa.field("email", pa.string(), nullable=False)]))
    emit("ref_roundtrip", ref, compression="snappy", data_page_version="2.0", version="2.6")

    # config 1 shape (BASELINE.json configs[0]), scaled to 20k rows
    t1 = datagen.flat_table(20000, seed=1)
    emit("c1_flat_none_v1", t1, compression="none", row_group_size=8192, data_page_size=16384)
    emit("c1_flat_snappy_v2", t1, compression="snappy", row_group_size=8192, data_page_version="2.0",
         data_page_size=16384)

    # config 2 shape: lineitem, Snappy + dictionary, multi-page chunks, dict->PLAIN fallback
    t2 = datagen.lineitem_table(30000, seed=42)
    emit("c2_lineitem", t2, compression="snappy", row_group_size=12000, data_page_size=8192,
         dictionary_pagesize_limit=8192)

    # config 4 shape: wide nullable INT32/FLOAT, 30% nulls, large dictionaries
    t4 = datagen.wide_table(6000, ncols=16, pool=3000, null_frac=0.3, seed=4)
    emit("c4_wide", t4, compression="snappy", row_group_size=3000)

    # config 5 shape: LIST<STRUCT<a INT64 (DELTA_BINARY_PACKED), b UTF8 (dict)>>, v2 pages
    t5 = datagen.nested_table(4000, seed=5)
    emit("c5_nested", t5, compression="snappy", data_page_version="2.0", row_group_size=2500,
         data_page_size=4096, use_dictionary=["l.list.element.b"],
         column_encoding={"l.list.element.a": "DELTA_BINARY_PACKED"})

    # edge cases: types
    te = datagen.edge_types_table(3000, seed=7)
    emit("edge_types_v1", te, compression="snappy", row_group_size=1000, data_page_size=2048,
         use_deprecated_int96_timestamps=True)
    emit("edge_types_v2", te, compression="none", data_page_version="2.0", row_group_size=1500,
         use_deprecated_int96_timestamps=True)

    # edge cases: encodings (no dictionary)
    tn = datagen.edge_encodings_table(5000, seed=8)
    emit("edge_encodings", tn, compression="snappy", data_page_version="2.0", use_dictionary=False,
         row_group_size=2048, data_page_size=4096,
         column_encoding={"d32": "DELTA_BINARY_PACKED", "d64": "DELTA_BINARY_PACKED",
                          "dlba": "DELTA_LENGTH_BYTE_ARRAY", "dba": "DELTA_BYTE_ARRAY",
                          "bss_f": "BYTE_STREAM_SPLIT", "bss_d": "BYTE_STREAM_SPLIT"})

    # edge: zero rows
    emit("edge_empty", pa.table({"a": pa.array([], pa.int64()), "s": pa.array([], pa.string())}),
         compression="snappy")

    # edge: list<int32> with null elements, uncompressed v1
    tl = datagen.list_prim_table(3000, seed=9)
    emit("list_prim", tl, compression="none", row_group_size=1000, data_page_size=1024)

    return manifests


def snappy_vectors(out_dir):
    rng = np.random.default_rng(11)
    cases = {
        "empty": b"",
        "one": b"x",
        "rle_a": b"a" * 5000,                        # overlapping copies (offset 1)
        "rle_ab": b"ab" * 7777,
        "random": rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),  # long literals, >64K
        "text": (b"the quick brown fox jumps over the lazy dog " * 3000),
        "mixed": b"".join(rng.choice([b"alpha", b"beta", b"gamma", b"delta", rng.integers(0, 256, 7, dtype=np.uint8).tobytes()])
                          for _ in range(20000)),
        "big_ints": np.arange(0, 200000, 3, dtype=np.int64).tobytes(),
    }
    arrays = {}
    for k, raw in cases.items():
        comp = pa.compress(raw, codec="snappy", asbytes=True) if raw else pa.compress(b"", codec="snappy", asbytes=True)
        arrays[f"{k}_raw"] = np.frombuffer(raw, dtype=np.uint8)
        arrays[f"{k}_comp"] = np.frombuffer(comp, dtype=np.uint8)
    np.savez_compressed(os.path.join(out_dir, "snappy_kat.npz"), **arrays)
    return list(cases)


if __name__ == "__main__":
    out = HERE
    mans = write_all(out)
    kat = snappy_vectors(out)
    with open(os.path.join(out, "manifest.json"), "w") as f:
        json.dump({"generator": "pyarrow " + pa.__version__, "files": mans, "snappy_kat": kat}, f, indent=1)
    print("wrote", len(mans), "fixtures")
