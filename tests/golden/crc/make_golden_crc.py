#!/usr/bin/env python3
"""Fixture of the page-header scan / CRC tests (tests/test_scan.py): crc_pages.parquet, written by
pyarrow 25.0.0 with write_page_checksum=True (PageHeader.crc, field 4, on every dictionary and data
page), small pages so each chunk has many headers, v1 pages with statistics (exercises the Thrift
skip of binary min/max) in row group 0's columns, and a second file layout with v2 pages
(crc_pages_v2.parquet). pyarrow's own reader with page_checksum_verification=True is the reference
for which damaged files must be rejected (tests/test_scan.py).

Run:  python tests/golden/crc/make_golden_crc.py"""
import os
import sys

import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "parquet-floor_amd"))
from pfloor import datagen  # noqa: E402


def main():
    t = datagen.lineitem_table(8000, seed=7)
    pq.write_table(t, os.path.join(HERE, "crc_pages.parquet"), compression="snappy", row_group_size=5000,
                   data_page_size=2048, write_batch_size=128, write_page_checksum=True,
                   write_statistics=True)
    n = datagen.nested_table(3000, seed=8)
    pq.write_table(n, os.path.join(HERE, "crc_pages_v2.parquet"), compression="snappy", data_page_version="2.0",
                   data_page_size=1024, write_batch_size=64, write_page_checksum=True,
                   use_dictionary=["l.list.element.b"],
                   column_encoding={"l.list.element.a": "DELTA_BINARY_PACKED"})


if __name__ == "__main__":
    main()
