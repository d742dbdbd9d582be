"""Load golden fixtures and compare a decoded chunk against them bit-exactly."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ARRAYS = ("values", "validity", "offsets", "chars", "list_offsets", "list_validity", "def_levels", "rep_levels")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_expected(name):
    """{(rg, col): {field: array, num_*: int}} for fixture `name`."""
    man = next(m for m in manifest()["files"] if m["file"] == name + ".parquet")
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {}
    for ch in man["chunks"]:
        key = (ch["rg"], ch["col"])
        d = {k: v for k, v in ch.items() if k.startswith("num_")}
        d["path"] = ch["path"]
        for a in ARRAYS:
            k = f"rg{ch['rg']}_c{ch['col']}_{a}"
            if k in z.files:
                d[a] = z[k]
        out[key] = d
    return out


def valid_mask(validity_bytes, n):
    return np.unpackbits(np.asarray(validity_bytes, dtype=np.uint8), bitorder="little")[:n].astype(bool)


def assert_chunk_equal(got, exp, label=""):
    """Bit-exact comparison of one decoded chunk against golden expectations.
    Values are compared as raw bytes (floats as bits); null slots must be zero."""
    for k in ("num_entries", "num_slots", "num_values", "num_rows"):
        assert int(got[k]) == int(exp[k]), f"{label}: {k} {got[k]} != {exp[k]}"
    for a in ARRAYS:
        if a not in exp:
            continue
        assert a in got, f"{label}: missing {a}"
        g = np.asarray(got[a]).view(np.uint8).ravel()
        e = np.asarray(exp[a]).view(np.uint8).ravel()
        if a in ("validity", "list_validity"):
            n = exp["num_slots"] if a == "validity" else exp["num_rows"]
            gm, em = valid_mask(g, n), valid_mask(e, n)
            assert np.array_equal(gm, em), f"{label}: {a} differs at {np.flatnonzero(gm != em)[:10]}"
            continue
        assert g.shape == e.shape, f"{label}: {a} size {g.shape} != {e.shape}"
        if not np.array_equal(g, e):
            bad = np.flatnonzero(g != e)
            raise AssertionError(f"{label}: {a} differs at bytes {bad[:10]} (n={len(bad)})")
