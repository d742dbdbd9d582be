/*
 * pfloor.h — C ABI of the MI355X-native Parquet column-chunk decoder.
 *
 * This is the drop-in boundary beneath parquet-floor's
 *   ParquetReader.streamContent(File|InputFile, HydratorSupplier[, columns])
 *   (reference: src/main/java/blue/strategic/parquet/ParquetReader.java:47-61)
 * Today that call pulls every value through parquet-mr 1.12.2's ColumnReader
 * (ParquetReader.java:141-168, :176-212) and decompresses pages through the
 * Hadoop codec shim into snappy-java (src/main/java/org/apache/hadoop/io/compress/
 * DecompressorStream.java:61-70,101-173; ReflectionUtils.java:10-21; CodecPool.java:6-8).
 *
 * The Java side keeps footer / schema / page-header (Thrift) parsing and fills the
 * POD descriptors below; chunk bytes are handed over in one buffer (pinned host memory
 * from pf_host_alloc, or device memory already resident in HBM).  The library decodes
 * every page on the GPU and returns columnar buffers (values, validity, BYTE_ARRAY
 * offsets + chars, list offsets, raw levels) that the Java adapter walks in
 * ParquetReader.tryAdvance order to call Hydrator.add(record, path[0], value).
 *
 * Rules of the ABI: plain C, no C++/torch types, every function returns a pf_status
 * (0 = OK, negative = error) except pf_abi_version / pf_last_error. No callbacks into
 * the caller. One context per GPU; one host thread drives a context at a time.
 * Error text for the last failing call on a context (or, for ctx-less calls, the
 * calling thread) is returned by pf_last_error.
 */
#ifndef PFLOOR_H
#define PFLOOR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PF_ABI_VERSION 1

/* ---- status codes (mapped by the Java bridge onto the reference's exceptions:
 *      IOException for open/footer errors, RuntimeException("Failed to read parquet", cause)
 *      for iteration errors — ParquetReader.java:120, :209-211) ---------------------- */
typedef enum pf_status {
    PF_OK = 0,
    PF_ERR_INVALID_ARG = -1,
    PF_ERR_CORRUPT_PAGE = -2,         /* bounds / varint / RLE overrun; never an OOB read */
    PF_ERR_UNSUPPORTED_ENCODING = -3,
    PF_ERR_UNSUPPORTED_CODEC = -4,
    PF_ERR_HIP = -5,
    PF_ERR_CAPACITY = -6,             /* caller buffer too small; required sizes are reported */
    PF_ERR_UNSUPPORTED_TYPE = -7,     /* ParquetReader.java:162-163 "Unsupported type" */
    PF_ERR_IO = -8,
    PF_ERR_STATE = -9
} pf_status;

/* ---- Parquet enums (Thrift ids of parquet-format; values are the wire values) ---- */
typedef enum pf_physical_type {
    PF_BOOLEAN = 0, PF_INT32 = 1, PF_INT64 = 2, PF_INT96 = 3,
    PF_FLOAT = 4, PF_DOUBLE = 5, PF_BYTE_ARRAY = 6, PF_FIXED_LEN_BYTE_ARRAY = 7
} pf_physical_type;

typedef enum pf_codec {
    PF_CODEC_UNCOMPRESSED = 0, PF_CODEC_SNAPPY = 1, PF_CODEC_GZIP = 2, PF_CODEC_LZO = 3,
    PF_CODEC_BROTLI = 4, PF_CODEC_LZ4 = 5, PF_CODEC_ZSTD = 6, PF_CODEC_LZ4_RAW = 7
} pf_codec;

typedef enum pf_page_type {
    PF_PAGE_DATA = 0, PF_PAGE_INDEX = 1, PF_PAGE_DICTIONARY = 2, PF_PAGE_DATA_V2 = 3
} pf_page_type;

typedef enum pf_encoding {
    PF_ENC_PLAIN = 0, PF_ENC_PLAIN_DICTIONARY = 2, PF_ENC_RLE = 3, PF_ENC_BIT_PACKED = 4,
    PF_ENC_DELTA_BINARY_PACKED = 5, PF_ENC_DELTA_LENGTH_BYTE_ARRAY = 6,
    PF_ENC_DELTA_BYTE_ARRAY = 7, PF_ENC_RLE_DICTIONARY = 8, PF_ENC_BYTE_STREAM_SPLIT = 9
} pf_encoding;

/* ---- descriptors filled from the Java Thrift parse (PageHeader / ColumnMetaData) ---- */

/* One page of a column chunk. `offset` locates the page BODY (the bytes after the
 * Thrift PageHeader) relative to the chunk's first byte. */
typedef struct pf_page_desc {
    uint64_t offset;
    uint32_t compressed_size;     /* PageHeader.compressed_page_size   (field 3) */
    uint32_t uncompressed_size;   /* PageHeader.uncompressed_page_size (field 2) */
    int32_t  page_type;           /* pf_page_type                       (field 1) */
    int32_t  encoding;            /* values encoding (DataPageHeader[V2] / DictionaryPageHeader) */
    int32_t  def_encoding;        /* v1 only: RLE or BIT_PACKED */
    int32_t  rep_encoding;        /* v1 only */
    int32_t  num_values;          /* level entries (data) / dictionary entries (dict) */
    int32_t  num_nulls;           /* v2: header; v1: page statistics null_count, -1 if absent.
                                     A routing hint (0 skips the null-page tables); results never
                                     depend on it */
    int32_t  num_rows;            /* v2 only */
    int32_t  def_bytes;           /* v2 only: definition_levels_byte_length */
    int32_t  rep_bytes;           /* v2 only: repetition_levels_byte_length */
    int32_t  is_compressed;       /* v2 only (Thrift default true); v1 pages: 1 */
} pf_page_desc;

/* One column chunk (one leaf column of one row group). */
typedef struct pf_chunk_desc {
    int32_t  physical_type;       /* pf_physical_type */
    int32_t  type_length;         /* FIXED_LEN_BYTE_ARRAY width; ignored otherwise */
    int32_t  max_def;             /* ColumnDescriptor.getMaxDefinitionLevel() */
    int32_t  max_rep;             /* ColumnDescriptor.getMaxRepetitionLevel() (<= 1 supported for list offsets) */
    int32_t  repeated_def;        /* def level of the innermost REPEATED ancestor (0 if max_rep == 0):
                                     an entry is a list element ("slot") iff def >= repeated_def */
    int32_t  list_null_def;       /* the innermost list is non-null iff def >= list_null_def */
    int32_t  codec;               /* pf_codec */
    int32_t  n_pages;             /* pages, including the dictionary page if present */
    const pf_page_desc* pages;
    uint64_t chunk_offset;        /* offset of the chunk's first byte in the bytes buffer */
    uint64_t chunk_size;          /* ColumnMetaData.total_compressed_size */
    int64_t  num_rows;            /* RowGroup.num_rows (flat columns: = level entries) */
} pf_chunk_desc;

/* Decoded layout of one column chunk ("slots" = rows for flat columns, list elements for
 * max_rep == 1; null slots hold zero bytes / zero-length strings):
 *   values        slots * width bytes (BOOLEAN: 1 byte 0/1; INT96: 12; FLBA: type_length)
 *   validity      ceil(slots/8) bytes, LSB-first, bit = (def == max_def)     [max_def > 0]
 *   offsets       (slots+1) int32, BYTE_ARRAY only; chars = concatenated bytes
 *   list_offsets  (rows+1) int32, max_rep == 1: slots before each row
 *   list_validity ceil(rows/8) bytes, bit = (def of the row's first entry >= list_null_def)
 *   def_levels / rep_levels  one byte per level entry                          [max_rep > 0]
 * Capacities are in BYTES. Any pointer may be NULL to skip that array. */
typedef struct pf_column_out {
    void*    values;        size_t values_cap;
    uint8_t* validity;      size_t validity_cap;
    int32_t* offsets;       size_t offsets_cap;
    uint8_t* chars;         size_t chars_cap;
    int32_t* list_offsets;  size_t list_offsets_cap;
    uint8_t* list_validity; size_t list_validity_cap;
    uint8_t* def_levels;    size_t def_levels_cap;
    uint8_t* rep_levels;    size_t rep_levels_cap;
} pf_column_out;

/* Sizes (and device pointers) of one decoded chunk, valid after pf_wait. */
typedef struct pf_column_info {
    int64_t num_entries;          /* level entries (= Σ page num_values) */
    int64_t num_slots;
    int64_t num_values;           /* non-null leaf values (def == max_def) */
    int64_t num_rows;             /* entries with rep == 0 */
    int64_t num_chars;            /* BYTE_ARRAY bytes */
    int32_t width;                /* bytes per slot in `values` (0 for BYTE_ARRAY) */
    int32_t status;               /* per-chunk pf_status */
    const void*    d_values;      /* device pointers (owned by the context, valid until the next decode) */
    const uint8_t* d_validity;
    const int32_t* d_offsets;
    const uint8_t* d_chars;
    const int32_t* d_list_offsets;
    const uint8_t* d_list_validity;
    const uint8_t* d_def_levels;
    const uint8_t* d_rep_levels;
} pf_column_info;

typedef struct pf_ctx pf_ctx;

int         pf_abi_version(void);
const char* pf_last_error(pf_ctx* ctx);           /* ctx may be NULL: thread-local message */

int pf_device_count(int* count);
int pf_ctx_create(int device, pf_ctx** out);
int pf_ctx_destroy(pf_ctx* ctx);
/* A second context on peer's GPU that enqueues onto peer's HIP stream (own device buffers,
 * results and completion event). Two such contexts let a reader plan and enqueue row group
 * i+1 while row group i is still decoding (the same stream keeps them in order), and pf_wait
 * on one waits only for its own decode. The shared stream lives until both are destroyed. */
int pf_ctx_create_shared(pf_ctx* peer, pf_ctx** out);
/* Per-stage timing events (pf_last_timing); on by default. Each event is a marker on the
 * stream between kernels, so a throughput-critical caller turns them off. */
int pf_ctx_set_timing(pf_ctx* ctx, int on);

/* Pinned host memory (hipHostMalloc) for chunk bytes and outputs; Java wraps it with
 * MemorySegment.reinterpret. */
int pf_host_alloc(pf_ctx* ctx, size_t bytes, void** out);
int pf_host_free(pf_ctx* ctx, void* ptr);

/* Device memory owned by the context (for callers that keep inputs resident in HBM). */
int pf_device_alloc(pf_ctx* ctx, size_t bytes, void** out);
int pf_device_free(pf_ctx* ctx, void* ptr);
int pf_memcpy_h2d(pf_ctx* ctx, void* dst, const void* src, size_t bytes);   /* async on ctx stream */

/* Enqueue the decode of n_chunks column chunks whose bytes live in `bytes`
 * (n_bytes long; host memory, ideally pinned, unless bytes_on_device != 0).
 * Asynchronous: returns after enqueueing H2D + kernels on the context's stream.
 * Descriptor arrays are copied before return. Results live in context-owned device
 * buffers until the next pf_decode_row_group on this context. */
int pf_decode_row_group(pf_ctx* ctx, const pf_chunk_desc* chunks, int n_chunks,
                        const uint8_t* bytes, size_t n_bytes, int bytes_on_device);

/* Block until the enqueued decode has finished; returns the first per-chunk error. */
int pf_wait(pf_ctx* ctx);

/* Sizes + device pointers of chunk i of the last decode (after pf_wait). */
int pf_column_info_get(pf_ctx* ctx, int chunk, pf_column_info* out);

/* Copy chunk i's decoded arrays into caller buffers (host, synchronous: returns when these
 * copies are done, without waiting for a peer context's work queued behind them).
 * Fails with PF_ERR_CAPACITY (nothing copied) if any non-NULL buffer is too small. */
int pf_copy_column(pf_ctx* ctx, int chunk, const pf_column_out* out);

/* Batched, asynchronous form of pf_copy_column for the end-to-end pipeline (the Java side reads
 * a row group's selected chunks into pinned output segments, ParquetReader.java:183-192): all
 * capacities are checked first (PF_ERR_CAPACITY, nothing enqueued), then the D2H copies of the
 * n chunks are enqueued on the context stream. Destination buffers should be pinned
 * (pf_host_alloc) and stay valid until pf_sync. A later pf_decode_row_group on the same
 * context is ordered after these copies (same stream), so decode i+1 can be enqueued at once. */
int pf_copy_columns_async(pf_ctx* ctx, int n, const int* chunks, const pf_column_out* outs);

/* Whole-batch form for the end-to-end pipeline: ONE D2H copy per output arena (values / offsets /
 * levels, validity bits, chars) into a caller buffer of pf_batch_bytes bytes (pinned), instead of
 * up to 8 copies per chunk. After pf_sync, pf_column_info_host returns chunk i's pf_column_info
 * with its d_* pointers rebased into that host buffer (same layout rules as the device arrays).
 * Valid after pf_wait until the next decode on this context. A mapped pinned buffer (pf_host_alloc,
 * hipHostMalloc) is written by a download kernel on a copy stream the context shares with its twin
 * (pf_ctx_create_shared), ordered after the decode, so the link carries uploads and downloads at
 * once (round 6); any other buffer takes SDMA copies on the context stream. */
int pf_batch_bytes(pf_ctx* ctx, size_t* bytes);
int pf_copy_batch_async(pf_ctx* ctx, void* host, size_t cap);
int pf_column_info_host(pf_ctx* ctx, int chunk, const void* host, pf_column_info* out);

/* Block until the copies this context enqueued (pf_copy_columns_async / pf_copy_batch_async) have
 * finished. A peer context's decode queued behind them on a shared stream is not waited for. */
int pf_sync(pf_ctx* ctx);

/* Kernel timing of the last decode (sum of per-stage HIP-event times, ms). */
int pf_last_timing(pf_ctx* ctx, float* stage_ms, int n_stages, int* n_written);

/* Decompress one raw Snappy buffer (snappy-java Snappy.uncompress semantics) with the
 * page kernels (K1). Host buffers; synchronous. *out_len = uncompressed length.
 * Invalidates the results of the last pf_decode_row_group on this context. */
int pf_snappy_decompress(pf_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
/* 1 if the last pf_snappy_decompress needed the serial fallback kernel (stream not split into
 * independent 64 KiB blocks, or corrupt), 0 if the block-parallel kernels decoded it. */
int pf_snappy_last_fallback(pf_ctx* ctx);

/* ---- GPU page-header scan (the per-page Thrift walk of ParquetFileReader.readNextRowGroup,
 *      ParquetReader.java:183, moved to the device) with optional page CRC32 verification
 *      (parquet-mr ParquetReadOptions.usePageChecksumVerification: a page whose PageHeader.crc,
 *      field 4, differs from the CRC32 of its on-disk page bytes is rejected). Pages are read
 *      until the chunk's num_values level entries have been seen; INDEX / unknown pages are
 *      skipped; the descriptors are exactly what pf_file_chunk_desc (the host walk) produces. */
typedef struct pf_scan_chunk {
    uint64_t chunk_offset;        /* first byte of the chunk in `bytes` */
    uint64_t chunk_size;          /* ColumnMetaData.total_compressed_size */
    int64_t  num_values;          /* ColumnMetaData.num_values */
    int32_t  page_base;           /* first slot of this chunk's descriptors in pages_out */
    int32_t  page_cap;            /* slots available to it */
} pf_scan_chunk;
typedef struct pf_scan_result {
    int32_t n_pages;              /* dictionary + data pages found */
    int32_t status;               /* PF_OK, PF_ERR_CORRUPT_PAGE (header, bounds or CRC), PF_ERR_CAPACITY */
    int32_t err_page;             /* chunk-relative page of the first error, -1 */
    int32_t crc_pages;            /* pages whose CRC was verified (verify_crc, header has a crc) */
} pf_scan_result;
/* Synchronous. `bytes` is host memory (copied to the device) unless bytes_on_device != 0.
 * pages_out has room for every chunk's [page_base, page_base + page_cap) slots; results has
 * n_chunks entries. Returns the first chunk error (PF_OK if none). */
int pf_scan_pages(pf_ctx* ctx, const pf_scan_chunk* chunks, int n_chunks, const uint8_t* bytes, size_t n_bytes,
                  int bytes_on_device, int verify_crc, pf_page_desc* pages_out, pf_scan_result* results);
/* ---- host-side metadata parse: the stand-in for the Java side's parquet-mr footer /
 *      PageHeader parse (ParquetFileReader.open + readNextRowGroup,
 *      ParquetReader.java:120, :183). Builds the descriptors above from a file. ---- */
typedef struct pf_file pf_file;

typedef struct pf_column_meta {
    const char* path;             /* dotted path_in_schema */
    const char* top_name;         /* ColumnDescriptor.getPath()[0] (the Hydrator heading) */
    int32_t physical_type, type_length, max_def, max_rep, repeated_def, list_null_def;
    int32_t converted_type;       /* SchemaElement.converted_type or -1 */
    int32_t logical_type;         /* LogicalType union field id or 0 */
    int32_t scale, precision;     /* DECIMAL (SchemaElement 7/8 or LogicalType DecimalType) */
} pf_column_meta;

int pf_file_open(const char* path, pf_file** out);
int pf_file_close(pf_file* f);
int pf_file_num_row_groups(pf_file* f, int* out);
int pf_file_num_columns(pf_file* f, int* out);
int pf_file_num_rows(pf_file* f, int64_t* out);
int pf_file_column_meta(pf_file* f, int column, pf_column_meta* out);
int pf_file_row_group_rows(pf_file* f, int row_group, int64_t* out);
/* Byte range [start, start+size) of a chunk in the file. */
int pf_file_chunk_range(pf_file* f, int row_group, int column, uint64_t* start, uint64_t* size);
/* Parse the chunk's page headers; fills *desc (pages owned by the pf_file) with
 * chunk_offset = `chunk_offset_in_buffer`. */
int pf_file_chunk_desc(pf_file* f, int row_group, int column, uint64_t chunk_offset_in_buffer,
                       pf_chunk_desc* desc);
/* Read raw bytes of the file (host). */
int pf_file_read(pf_file* f, uint64_t offset, uint64_t size, void* dst);
const char* pf_file_created_by(pf_file* f);

/* ---- write path: the reference's ParquetWriter (ParquetWriter.java:61-165: SNAPPY,
 *      WriterVersion.PARQUET_2_0, parquet-mr 1.12.2 defaults) with the column encoding on the
 *      GPU: dictionary encode (entries in first-occurrence order, like parquet-mr's
 *      DictionaryValuesWriter), RLE/bit-packed hybrid ids, PLAIN values, Snappy compression of
 *      every page. Flat schemas of the types the reference writes (ParquetWriter.java:143-157):
 *      BOOLEAN, INT32, INT64, FLOAT, DOUBLE, BYTE_ARRAY (UTF8). ---- */
typedef struct pf_encode_column {
    int32_t  physical_type;       /* PF_BOOLEAN, PF_INT32, PF_INT64, PF_FLOAT, PF_DOUBLE, PF_BYTE_ARRAY */
    int32_t  max_def;             /* 0 = REQUIRED, 1 = OPTIONAL */
    int64_t  num_rows;
    const void*    values;        /* fixed width, row-indexed (null rows ignored); BOOLEAN: one byte per row */
    const uint8_t* validity;      /* LSB-first, bit = present; NULL = all present (max_def 1) */
    const int32_t* offsets;       /* BYTE_ARRAY: num_rows + 1 (null rows: empty) */
    const uint8_t* chars;         /* BYTE_ARRAY */
    int64_t  chars_len;
    int32_t  dictionary;          /* 1: dictionary-encode (PLAIN above dict_page_limit or on a hash collision) */
    int32_t  page_rows;           /* rows per data page; 0 = 20000 (parquet-mr page.row.count.limit) */
    int32_t  dict_page_limit;     /* dictionary page bytes; 0 = 1 MiB (parquet.dictionary.page.size) */
    int32_t  codec;               /* PF_CODEC_SNAPPY (the reference's) or PF_CODEC_UNCOMPRESSED */
} pf_encode_column;

typedef struct pf_encoded_chunk {
    const uint8_t* bytes;         /* page headers + bodies as they appear in the file (owned by the ctx,
                                     valid until its next pf_encode_chunk) */
    int64_t  size;                /* = ColumnMetaData.total_compressed_size */
    int64_t  total_uncompressed_size;
    int64_t  num_values;
    int64_t  dictionary_page_offset;   /* relative to bytes, -1 if none */
    int64_t  data_page_offset;         /* relative to bytes */
    int32_t  n_data_pages;
    int32_t  dict_entries;        /* 0 when not dictionary-encoded */
    int32_t  data_encoding;       /* PF_ENC_RLE_DICTIONARY or PF_ENC_PLAIN */
    int32_t  fallback;            /* 0; 1 dictionary above the limit; 2 hash collision; 3 type (BOOLEAN) */
    int32_t  codec;               /* ColumnMetaData.codec */
    float    snappy_ms;           /* k_snappy_compress time (HIP events; 0 when stage timing is off) */
    float    encode_ms;           /* dictionary + page kernels time (HIP events; 0 when timing is off) */
    int64_t  snappy_in, snappy_out;    /* bytes into / out of the compressor */
} pf_encoded_chunk;

/* Encode one column chunk on the context's GPU. Inputs are host memory (copied) unless
 * on_device != 0. Synchronous. */
int pf_encode_chunk(pf_ctx* ctx, const pf_encode_column* col, int on_device, pf_encoded_chunk* out);
/* Snappy-compress one buffer on the GPU: independent 8 KiB jobs (one wave each; a job's matches stay
 * inside it, so tokens never cross a 64 KiB output boundary). Host buffers, synchronous;
 * *out_len = compressed length (cap >= 32 + n + n / 6 always suffices). */
int pf_snappy_compress(pf_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

/* File writer (host): "PAR1", row groups of encoded chunks, Thrift compact FileMetaData footer. */
typedef struct pf_writer pf_writer;
typedef struct pf_write_field {
    const char* name;
    int32_t physical_type;
    int32_t optional;             /* 1 = OPTIONAL, 0 = REQUIRED */
    int32_t utf8;                 /* BYTE_ARRAY: STRING logical type (the only BINARY the reference writes) */
} pf_write_field;
int pf_writer_open(const char* path, const pf_write_field* fields, int n_fields, pf_writer** out);
/* Append the chunk of field `field` (fields in schema order) to the current row group. */
int pf_writer_add_chunk(pf_writer* w, int field, const pf_encoded_chunk* chunk);
int pf_writer_end_row_group(pf_writer* w, int64_t num_rows);
int pf_writer_close(pf_writer* w);   /* footer; frees w (also on error) */
const char* pf_writer_last_error(void);
const char* pf_file_last_error(void);            /* thread-local message of the last pf_file_* error */

#ifdef __cplusplus
}
#endif
#endif /* PFLOOR_H */
