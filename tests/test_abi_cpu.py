"""CPU-side checks of the product library: it loads, exports every symbol include/pfloor.h
declares, and its host metadata parser (the stand-in for the Java-side footer/PageHeader
parse) agrees with the oracle and with pyarrow's metadata. No GPU calls here."""
import ctypes as C
import json
import os
import re

import pytest

from conftest import GOLDEN, ROOT, golden_files


@pytest.fixture(scope="session")
def native():
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "parquet-floor_amd")], check=True)
    from pfloor import _native
    return _native


def header_functions():
    src = open(os.path.join(ROOT, "include", "pfloor.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|int64_t)\s+\**(pf_\w+)\s*\(", src, flags=re.M)))


def test_exports_every_header_symbol(native):
    L = native.lib()
    fns = header_functions()
    assert len(fns) >= 25, fns
    missing = [f for f in fns if not hasattr(L, f)]
    assert not missing, missing


def test_abi_version(native):
    assert native.lib().pf_abi_version() == 1


def test_no_device_is_an_error_not_a_fallback(native):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    n = C.c_int(-1)
    rc = native.lib().pf_device_count(C.byref(n))
    assert n.value == 0
    ctx = C.c_void_p()
    assert native.lib().pf_ctx_create(0, C.byref(ctx)) != 0


@pytest.mark.parametrize("name", golden_files())
def test_metadata_matches_oracle(native, oracle, name):
    from pfloor.decoder import ParquetFile
    path = os.path.join(GOLDEN, name + ".parquet")
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    fm = next(m for m in man["files"] if m["file"] == name + ".parquet")
    with ParquetFile(path) as pf, oracle.open(path) as of:
        assert pf.num_row_groups == of.num_row_groups == fm["row_groups"]
        assert pf.num_columns == of.num_columns == fm["columns"]
        assert pf.num_rows == fm["num_rows"]
        for c, col in enumerate(pf.columns):
            sch = of.schema(c)
            assert ".".join(col.path) == of.column_path(c)
            assert col.path[0] == of.top_name(c)
            assert (col.physical_type, col.max_def, col.max_rep, col.repeated_def, col.list_null_def) == \
                (sch["type"], sch["max_def"], sch["max_rep"], sch["repeated_def"], sch["list_null_def"])
        for rg in range(pf.num_row_groups):
            for c in range(pf.num_columns):
                d = pf.chunk_desc(rg, c, 0)
                total = sum(d.pages[i].num_values for i in range(d.n_pages) if d.pages[i].page_type != 2)
                exp = next(ch for ch in fm["chunks"] if ch["rg"] == rg and ch["col"] == c)
                assert total == exp["num_entries"]


def test_struct_layouts_match_header(native, tmp_path):
    """The ctypes mirror (what an FFM/ctypes binding declares) matches the C header's layout:
    sizeof and every field offset, from a probe compiled against include/pfloor.h."""
    import subprocess
    structs = {"pf_page_desc": native.PageDesc, "pf_chunk_desc": native.ChunkDesc,
               "pf_column_out": native.ColumnOut, "pf_column_info": native.ColumnInfo,
               "pf_column_meta": native.ColumnMeta, "pf_scan_chunk": native.ScanChunk,
               "pf_scan_result": native.ScanResult}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pfloor.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = ln.split()
        got[(s, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)
