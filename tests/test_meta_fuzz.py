"""AddressSanitizer + UndefinedBehaviorSanitizer run of the host metadata parser (csrc/pf_meta.cpp,
csrc/pf_file.cpp — the untrusted-input side of the boundary, standing in for parquet-mr's footer /
PageHeader parse, ParquetReader.java:120, :183) over mutated golden files: truncations, bit flips,
0x00/0xff bytes in the footer and the page headers. Host code only (no GPU), built here with g++."""
import glob
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

CSRC = os.path.join(ROOT, "parquet-floor_amd", "csrc")


@pytest.fixture(scope="module")
def fuzzer(tmp_path_factory):
    out = tmp_path_factory.mktemp("fuzz") / "pf_meta_fuzz"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
           os.path.join(ROOT, "tests", "native", "pf_meta_fuzz.cpp"), os.path.join(CSRC, "pf_meta.cpp"),
           os.path.join(CSRC, "pf_file.cpp"), "-o", str(out)]
    subprocess.run(cmd, check=True)
    return str(out)


@pytest.mark.parametrize("seed", [1, 2])
def test_host_parser_survives_mutations_under_asan(fuzzer, tmp_path, seed):
    files = sorted(glob.glob(os.path.join(GOLDEN, "*.parquet")) + glob.glob(os.path.join(GOLDEN, "crc", "*.parquet")))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=97",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
    env.pop("LD_PRELOAD", None) if "libasan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([fuzzer, str(seed), "1500", str(tmp_path)] + files, capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "iterations 1500" in r.stdout
