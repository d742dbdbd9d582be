/*
 * pf_oracle.h — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * Plain-C restatement of the decode that parquet-floor's read path delegates to
 * parquet-mr 1.12.2 + snappy-java (un-vendored upstream deps, pom.xml:61-77).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / CPU baseline.  It is pinned against golden vectors that
 * pyarrow 25.0.0 (an independent Parquet implementation) produced in the build
 * container (tests/golden/make_golden.py), and against the reference's only test
 * (src/test/java/blue/strategic/parquet/ParquetReadWriteTest.java:28-83).
 */
#ifndef PF_ORACLE_H
#define PF_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pfo_file pfo_file;

typedef struct pfo_column {
    int32_t status;               /* 0 ok, <0 error (same codes as pfloor.h) */
    char    error[256];
    int32_t physical_type, type_length, max_def, max_rep, repeated_def, list_null_def, width;
    int64_t num_entries, num_slots, num_values, num_rows, num_chars;
    uint8_t* values;              /* num_slots * width */
    uint8_t* validity;            /* ceil(num_slots/8) */
    int32_t* offsets;             /* num_slots + 1 (BYTE_ARRAY) */
    uint8_t* chars;               /* num_chars */
    int32_t* list_offsets;        /* num_rows + 1 (max_rep == 1) */
    uint8_t* list_validity;       /* ceil(num_rows/8) */
    uint8_t* def_levels;          /* num_entries (max_rep > 0) */
    uint8_t* rep_levels;
} pfo_column;

int  pfo_open(const char* path, pfo_file** out, char* err, int errlen);
int  pfo_open_mem(const uint8_t* data, size_t n, pfo_file** out, char* err, int errlen);
void pfo_close(pfo_file* f);
int  pfo_num_row_groups(const pfo_file* f);
int  pfo_num_columns(const pfo_file* f);
int64_t pfo_num_rows(const pfo_file* f);
int64_t pfo_row_group_rows(const pfo_file* f, int rg);
/* leaf column info: dotted path into buf */
int  pfo_column_path(const pfo_file* f, int col, char* buf, int buflen);
int  pfo_column_top_name(const pfo_file* f, int col, char* buf, int buflen);
int  pfo_column_schema(const pfo_file* f, int col, int32_t* out7); /* type,len,maxdef,maxrep,repdef,listnulldef,converted */
int  pfo_column_logical(const pfo_file* f, int col);

/* Decode one column chunk. Returns status; fills *out (free with pfo_free_column). */
int  pfo_decode(pfo_file* f, int rg, int col, pfo_column* out);
void pfo_free_column(pfo_column* c);

/* Raw Snappy (snappy-java Snappy.uncompress / Google Snappy format). Returns bytes written or <0. */
int64_t pfo_snappy_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap);
int64_t pfo_snappy_uncompressed_length(const uint8_t* in, size_t n);
/* Test-vector generator: greedy Snappy compressor (mode 0 Google-style 64 KiB blocks, mode 1 cross-block). */
/* Page-header walk + CRC32 of one chunk (oracle of pf_scan_pages). */
typedef struct pfo_page {
    uint64_t offset;              /* page body, relative to the chunk's first byte */
    int32_t compressed_size, uncompressed_size, page_type, encoding, num_values;
    int32_t has_crc;              /* PageHeader.crc present */
    uint32_t crc;
    int32_t crc_ok;               /* CRC32 of the page bytes == crc (1 without a crc) */
} pfo_page;
int pfo_chunk_pages(pfo_file* f, int rg, int col, pfo_page* out, int cap, int verify_crc, int* err_page);
uint32_t pfo_crc32(const uint8_t* p, size_t n);

int64_t pfo_snappy_compress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, int mode);

#ifdef __cplusplus
}
#endif
#endif
