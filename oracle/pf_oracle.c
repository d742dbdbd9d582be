/*
 * pf_oracle.c — CPU ORACLE for the Parquet column-chunk decode (TEST INFRASTRUCTURE ONLY).
 *
 * Restates, in plain C, the algorithm the reference's read path runs:
 *   parquet-floor ParquetReader (src/main/java/blue/strategic/parquet/ParquetReader.java)
 *     :120  ParquetFileReader.open            -> footer Thrift parse        (pfo_open)
 *     :183  readNextRowGroup                  -> chunk bytes + PageHeaders  (walk_pages)
 *     :192  ColumnReadStoreImpl.getColumnReader -> dictionary + page init   (decode_dictionary)
 *     :146  getCurrentDefinitionLevel()==maxDef -> value or null            (assemble)
 *     :148-161 getBinary/getBoolean/getDouble/getFloat/getInteger/getLong   (decode_values)
 *     :199-200 consume()/getCurrentRepetitionLevel()                        (levels)
 * with the arithmetic of the un-vendored upstream jars (parquet-mr 1.12.2, pom.xml:61-77;
 * snappy-java, transitive) restated from their published algorithms:
 *   org.apache.parquet.format (Thrift compact protocol, parquet.thrift field ids)
 *   RunLengthBitPackingHybridDecoder, ByteBitPackingValuesReader (levels, dict ids, RLE bool)
 *   PlainValuesReader.*, BinaryPlainValuesReader, BooleanPlainValuesReader, FixedLenByteArrayPlainValuesReader
 *   DictionaryValuesReader + PlainValuesDictionary.*
 *   DeltaBinaryPackingValuesReader(ForLong), DeltaLengthByteArrayValuesReader, DeltaByteArrayReader
 *   ByteStreamSplitValuesReader(ForFloat|ForDouble)
 *   Google Snappy raw format (SnappyDecompressor -> Snappy.uncompress), reached through the
 *   Hadoop shim oah/io/compress/DecompressorStream.java:61-70,101-173.
 * Parity is pinned by tests/golden (pyarrow-produced vectors, tests/golden/make_golden.py)
 * and the reference's own round trip (src/test/java/blue/strategic/parquet/ParquetReadWriteTest.java:28-83).
 */
#define _POSIX_C_SOURCE 200809L
#include "pf_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { E_OK = 0, E_ARG = -1, E_CORRUPT = -2, E_ENC = -3, E_CODEC = -4, E_CAP = -6, E_TYPE = -7, E_IO = -8 };

/* ------------------------------------------------------------------ growable buffer */
typedef struct { uint8_t* p; size_t n, cap; } buf_t;
static int buf_reserve(buf_t* b, size_t extra) {
    if (b->n + extra <= b->cap) return 0;
    size_t nc = b->cap ? b->cap : 256;
    while (nc < b->n + extra) nc *= 2;
    uint8_t* q = (uint8_t*)realloc(b->p, nc);
    if (!q) return -1;
    b->p = q; b->cap = nc; return 0;
}
static int buf_put(buf_t* b, const void* src, size_t n) {
    if (buf_reserve(b, n)) return -1;
    if (n) memcpy(b->p + b->n, src, n);
    b->n += n; return 0;
}

/* ------------------------------------------------------------------ Thrift compact protocol */
typedef struct { const uint8_t* p; const uint8_t* end; int err; } tr_t;

static uint8_t tr_byte(tr_t* r) { if (r->p >= r->end) { r->err = 1; return 0; } return *r->p++; }
static uint64_t tr_varint(tr_t* r) {
    uint64_t v = 0; int sh = 0;
    for (;;) {
        uint8_t c = tr_byte(r);
        if (r->err) return 0;
        if (sh < 64) v |= (uint64_t)(c & 0x7f) << sh;
        if (!(c & 0x80)) return v;
        sh += 7;
        if (sh > 70) { r->err = 1; return 0; }
    }
}
static int64_t tr_zz(tr_t* r) { uint64_t v = tr_varint(r); return (int64_t)(v >> 1) ^ -(int64_t)(v & 1); }

static void tr_skip(tr_t* r, int type, int depth);
static void tr_skip_struct(tr_t* r, int depth) {
    if (depth > 64) { r->err = 1; return; }
    for (;;) {
        uint8_t h = tr_byte(r);
        if (r->err || h == 0) return;
        if ((h >> 4) == 0) tr_zz(r);
        tr_skip(r, h & 0xf, depth + 1);
        if (r->err) return;
    }
}
static void tr_skip(tr_t* r, int type, int depth) {
    switch (type) {
    case 1: case 2: return;                       /* bool in field header */
    case 3: tr_byte(r); return;
    case 4: case 5: case 6: tr_varint(r); return;
    case 7: if (r->end - r->p < 8) r->err = 1; else r->p += 8; return;
    case 8: { uint64_t n = tr_varint(r); if ((uint64_t)(r->end - r->p) < n) r->err = 1; else r->p += n; return; }
    case 9: case 10: {
        uint8_t h = tr_byte(r); uint64_t n = h >> 4; int et = h & 0xf;
        if (n == 15) n = tr_varint(r);
        for (uint64_t i = 0; i < n && !r->err; i++) {
            if (et == 1 || et == 2) tr_byte(r); else tr_skip(r, et, depth + 1);
        }
        return;
    }
    case 11: {
        uint64_t n = tr_varint(r);
        if (n == 0) return;
        uint8_t kv = tr_byte(r);
        for (uint64_t i = 0; i < n && !r->err; i++) { tr_skip(r, kv >> 4, depth + 1); tr_skip(r, kv & 0xf, depth + 1); }
        return;
    }
    case 12: tr_skip_struct(r, depth + 1); return;
    default: r->err = 1; return;
    }
}
/* iterate fields: returns field id, sets *type; 0 on STOP */
static int tr_field(tr_t* r, int* last, int* type) {
    uint8_t h = tr_byte(r);
    if (r->err || h == 0) return 0;
    int d = h >> 4;
    *type = h & 0xf;
    int id = d ? *last + d : (int)tr_zz(r);
    *last = id;
    return id;
}
static int64_t tr_int(tr_t* r, int type) {
    if (type == 3) return (int8_t)tr_byte(r);
    if (type == 4 || type == 5 || type == 6) return tr_zz(r);
    tr_skip(r, type, 0); r->err = 1; return 0;
}
static int tr_bool(tr_t* r, int type) { if (type == 1) return 1; if (type == 2) return 0; tr_skip(r, type, 0); return 0; }
static char* tr_string(tr_t* r, int type) {
    if (type != 8) { tr_skip(r, type, 0); return NULL; }
    uint64_t n = tr_varint(r);
    if (r->err || (uint64_t)(r->end - r->p) < n) { r->err = 1; return NULL; }
    char* s = (char*)malloc(n + 1);
    memcpy(s, r->p, n); s[n] = 0; r->p += n; return s;
}
static uint64_t tr_list_begin(tr_t* r, int* et) {
    uint8_t h = tr_byte(r); uint64_t n = h >> 4; *et = h & 0xf;
    if (n == 15) n = tr_varint(r);
    return n;
}

/* ------------------------------------------------------------------ file model */
typedef struct {
    char* name; int type, type_length, repetition, num_children, converted_type, logical_type;
} schema_el;

typedef struct {
    int codec, type;
    int64_t num_values, total_compressed_size, data_page_offset, dictionary_page_offset;
    int has_dict_offset;
} chunk_meta;

typedef struct { chunk_meta* cols; int ncols; int64_t num_rows; } row_group;

typedef struct {
    char* path; char* top; int schema_index;
    int type, type_length, max_def, max_rep, repeated_def, list_null_def, converted_type, logical_type;
} leaf_t;

struct pfo_file {
    uint8_t* data; size_t size;
    schema_el* schema; int nschema;
    row_group* rgs; int nrg;
    leaf_t* leaves; int nleaves;
    int64_t num_rows;
    char* created_by;
};

static void set_err(char* err, int errlen, const char* msg) { if (err && errlen > 0) { strncpy(err, msg, errlen - 1); err[errlen - 1] = 0; } }

static int parse_logical(tr_t* r) {   /* LogicalType union: return the set field id */
    int last = 0, t, id, got = 0;
    while ((id = tr_field(r, &last, &t))) { got = id; tr_skip(r, t, 0); if (r->err) return 0; }
    return got;
}

static int parse_schema_el(tr_t* r, schema_el* e) {
    int last = 0, t, id;
    e->type = -1; e->type_length = 0; e->repetition = 0; e->num_children = 0; e->converted_type = -1; e->logical_type = 0; e->name = NULL;
    while ((id = tr_field(r, &last, &t))) {
        switch (id) {
        case 1: e->type = (int)tr_int(r, t); break;
        case 2: e->type_length = (int)tr_int(r, t); break;
        case 3: e->repetition = (int)tr_int(r, t); break;
        case 4: e->name = tr_string(r, t); break;
        case 5: e->num_children = (int)tr_int(r, t); break;
        case 6: e->converted_type = (int)tr_int(r, t); break;
        case 10: if (t == 12) e->logical_type = parse_logical(r); else tr_skip(r, t, 0); break;
        default: tr_skip(r, t, 0);
        }
        if (r->err) return -1;
    }
    return r->err ? -1 : 0;
}

static int parse_col_meta(tr_t* r, chunk_meta* m) {
    int last = 0, t, id;
    while ((id = tr_field(r, &last, &t))) {
        switch (id) {
        case 1: m->type = (int)tr_int(r, t); break;
        case 4: m->codec = (int)tr_int(r, t); break;
        case 5: m->num_values = tr_int(r, t); break;
        case 7: m->total_compressed_size = tr_int(r, t); break;
        case 9: m->data_page_offset = tr_int(r, t); break;
        case 11: m->dictionary_page_offset = tr_int(r, t); m->has_dict_offset = 1; break;
        default: tr_skip(r, t, 0);
        }
        if (r->err) return -1;
    }
    return 0;
}

static int parse_column_chunk(tr_t* r, chunk_meta* m) {
    int last = 0, t, id;
    memset(m, 0, sizeof(*m));
    while ((id = tr_field(r, &last, &t))) {
        if (id == 3 && t == 12) { if (parse_col_meta(r, m)) return -1; }
        else tr_skip(r, t, 0);
        if (r->err) return -1;
    }
    return 0;
}

static int parse_row_group(tr_t* r, row_group* g) {
    int last = 0, t, id;
    g->cols = NULL; g->ncols = 0; g->num_rows = 0;
    while ((id = tr_field(r, &last, &t))) {
        if (id == 1 && t == 9) {
            int et; uint64_t n = tr_list_begin(r, &et);
            if (r->err || et != 12 || n > 1000000) return -1;
            g->cols = (chunk_meta*)calloc(n ? n : 1, sizeof(chunk_meta));
            g->ncols = (int)n;
            for (uint64_t i = 0; i < n; i++) if (parse_column_chunk(r, &g->cols[i])) return -1;
        } else if (id == 3) g->num_rows = tr_int(r, t);
        else tr_skip(r, t, 0);
        if (r->err) return -1;
    }
    return 0;
}

static int parse_footer(pfo_file* f, const uint8_t* p, size_t n) {
    tr_t r = { p, p + n, 0 };
    int last = 0, t, id;
    while ((id = tr_field(&r, &last, &t))) {
        if (id == 2 && t == 9) {
            int et; uint64_t cnt = tr_list_begin(&r, &et);
            if (r.err || et != 12 || cnt > 10000000) return -1;
            f->schema = (schema_el*)calloc(cnt ? cnt : 1, sizeof(schema_el));
            f->nschema = (int)cnt;
            for (uint64_t i = 0; i < cnt; i++) if (parse_schema_el(&r, &f->schema[i])) return -1;
        } else if (id == 3) f->num_rows = tr_int(&r, t);
        else if (id == 4 && t == 9) {
            int et; uint64_t cnt = tr_list_begin(&r, &et);
            if (r.err || et != 12 || cnt > 10000000) return -1;
            f->rgs = (row_group*)calloc(cnt ? cnt : 1, sizeof(row_group));
            f->nrg = (int)cnt;
            for (uint64_t i = 0; i < cnt; i++) if (parse_row_group(&r, &f->rgs[i])) return -1;
        } else if (id == 6) f->created_by = tr_string(&r, t);
        else tr_skip(&r, t, 0);
        if (r.err) return -1;
    }
    return r.err ? -1 : 0;
}

/* Leaf columns in schema order with their levels (parquet-mr ColumnDescriptor via
 * MessageType.getColumns(); ParquetReader.java:126-128 filters these by path[0]). */
typedef struct { int def, rep, repeated_def, list_null_def; } lvl_state;

static int build_leaves(pfo_file* f, int* idx, int depth, lvl_state st, char* path, const char* top) {
    if (*idx >= f->nschema || depth > 100) return -1;
    int me = *idx;
    schema_el* e = &f->schema[me];
    (*idx)++;
    lvl_state s = st;
    int parent_def = st.def;
    if (depth > 0) {
        if (e->repetition == 1) s.def++;
        else if (e->repetition == 2) { s.def++; s.rep++; s.repeated_def = s.def; s.list_null_def = parent_def; }
    }
    char p2[4096];
    const char* nm = e->name ? e->name : "";
    if (depth == 0) p2[0] = 0;
    else if (path[0]) snprintf(p2, sizeof p2, "%s.%s", path, nm);
    else snprintf(p2, sizeof p2, "%s", nm);
    const char* top2 = depth == 1 ? nm : top;
    if (e->num_children > 0 || depth == 0) {
        for (int c = 0; c < e->num_children; c++)
            if (build_leaves(f, idx, depth + 1, s, p2, top2)) return -1;
        return 0;
    }
    f->leaves = (leaf_t*)realloc(f->leaves, sizeof(leaf_t) * (f->nleaves + 1));
    leaf_t* L = &f->leaves[f->nleaves++];
    L->path = strdup(p2); L->top = strdup(top2 ? top2 : nm); L->schema_index = me;
    L->type = e->type; L->type_length = e->type_length;
    L->max_def = s.def; L->max_rep = s.rep;
    L->repeated_def = s.rep ? s.repeated_def : 0;
    L->list_null_def = s.rep ? s.list_null_def : 0;
    L->converted_type = e->converted_type; L->logical_type = e->logical_type;
    return 0;
}

int pfo_open_mem(const uint8_t* data, size_t n, pfo_file** out, char* err, int errlen) {
    *out = NULL;
    if (n < 12 || memcmp(data, "PAR1", 4) || memcmp(data + n - 4, "PAR1", 4)) { set_err(err, errlen, "not a parquet file (magic)"); return E_IO; }
    uint32_t flen = (uint32_t)data[n - 8] | (uint32_t)data[n - 7] << 8 | (uint32_t)data[n - 6] << 16 | (uint32_t)data[n - 5] << 24;
    if ((uint64_t)flen + 12 > n) { set_err(err, errlen, "corrupt footer length"); return E_IO; }
    pfo_file* f = (pfo_file*)calloc(1, sizeof(pfo_file));
    f->data = (uint8_t*)malloc(n); memcpy(f->data, data, n); f->size = n;
    if (parse_footer(f, f->data + n - 8 - flen, flen)) { set_err(err, errlen, "corrupt footer"); pfo_close(f); return E_IO; }
    int idx = 0; lvl_state s = { 0, 0, 0, 0 }; char root[1] = { 0 };
    if (f->nschema == 0 || build_leaves(f, &idx, 0, s, root, NULL)) { set_err(err, errlen, "corrupt schema"); pfo_close(f); return E_IO; }
    for (int g = 0; g < f->nrg; g++)
        if (f->rgs[g].ncols != f->nleaves) { set_err(err, errlen, "row group column count mismatch"); pfo_close(f); return E_IO; }
    *out = f;
    return E_OK;
}

int pfo_open(const char* path, pfo_file** out, char* err, int errlen) {
    FILE* fp = fopen(path, "rb");
    if (!fp) { set_err(err, errlen, "cannot open file"); return E_IO; }
    fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
    uint8_t* d = (uint8_t*)malloc(n > 0 ? n : 1);
    if (n > 0 && fread(d, 1, n, fp) != (size_t)n) { fclose(fp); free(d); set_err(err, errlen, "read error"); return E_IO; }
    fclose(fp);
    int rc = pfo_open_mem(d, (size_t)n, out, err, errlen);
    free(d);
    return rc;
}

void pfo_close(pfo_file* f) {
    if (!f) return;
    for (int i = 0; i < f->nschema; i++) free(f->schema[i].name);
    free(f->schema);
    for (int g = 0; g < f->nrg; g++) free(f->rgs[g].cols);
    free(f->rgs);
    for (int i = 0; i < f->nleaves; i++) { free(f->leaves[i].path); free(f->leaves[i].top); }
    free(f->leaves); free(f->created_by); free(f->data); free(f);
}

int pfo_num_row_groups(const pfo_file* f) { return f->nrg; }
int pfo_num_columns(const pfo_file* f) { return f->nleaves; }
int64_t pfo_num_rows(const pfo_file* f) { return f->num_rows; }
int64_t pfo_row_group_rows(const pfo_file* f, int rg) { return (rg >= 0 && rg < f->nrg) ? f->rgs[rg].num_rows : -1; }
int pfo_column_path(const pfo_file* f, int c, char* b, int n) { if (c < 0 || c >= f->nleaves) return -1; snprintf(b, n, "%s", f->leaves[c].path); return 0; }
int pfo_column_top_name(const pfo_file* f, int c, char* b, int n) { if (c < 0 || c >= f->nleaves) return -1; snprintf(b, n, "%s", f->leaves[c].top); return 0; }
int pfo_column_schema(const pfo_file* f, int c, int32_t* o) {
    if (c < 0 || c >= f->nleaves) return -1;
    const leaf_t* L = &f->leaves[c];
    o[0] = L->type; o[1] = L->type_length; o[2] = L->max_def; o[3] = L->max_rep; o[4] = L->repeated_def; o[5] = L->list_null_def; o[6] = L->converted_type;
    return 0;
}
int pfo_column_logical(const pfo_file* f, int c) { return (c < 0 || c >= f->nleaves) ? -1 : f->leaves[c].logical_type; }

/* ------------------------------------------------------------------ Snappy (raw format)
 * Restatement of the Google Snappy decompressor that snappy-java's Snappy.uncompress wraps:
 * preamble = varint uncompressed length; tags: 00 literal (len-1 in tag>>2, 60..63 -> 1..4
 * little-endian length bytes), 01 copy (len 4..11, 11-bit offset), 10 copy (len 1..64,
 * 16-bit offset), 11 copy (len 1..64, 32-bit offset). Copies may overlap their output. */
int64_t pfo_snappy_uncompressed_length(const uint8_t* in, size_t n) {
    uint64_t v = 0; int sh = 0; size_t i = 0;
    for (;;) {
        if (i >= n || sh > 28) return -1;
        uint8_t c = in[i++];
        v |= (uint64_t)(c & 0x7f) << sh;
        if (!(c & 0x80)) break;
        sh += 7;
    }
    if (v > 0xffffffffull) return -1;
    return (int64_t)v;
}

int64_t pfo_snappy_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
    uint64_t ulen = 0; int sh = 0; size_t i = 0;
    for (;;) {
        if (i >= n || sh > 28) return E_CORRUPT;
        uint8_t c = in[i++];
        ulen |= (uint64_t)(c & 0x7f) << sh;
        if (!(c & 0x80)) break;
        sh += 7;
    }
    if (ulen > cap) return E_CAP;
    size_t op = 0;
    while (i < n) {
        uint8_t tag = in[i++];
        size_t len, off;
        switch (tag & 3) {
        case 0: {
            len = tag >> 2;
            if (len >= 60) {
                size_t nb = len - 59;
                if (i + nb > n) return E_CORRUPT;
                len = 0;
                for (size_t k = 0; k < nb; k++) len |= (size_t)in[i + k] << (8 * k);
                i += nb;
            }
            len += 1;
            if (i + len > n || op + len > ulen) return E_CORRUPT;
            memcpy(out + op, in + i, len);
            i += len; op += len;
            continue;
        }
        case 1:
            if (i + 1 > n) return E_CORRUPT;
            len = 4 + ((tag >> 2) & 7);
            off = ((size_t)(tag >> 5) << 8) | in[i];
            i += 1;
            break;
        case 2:
            if (i + 2 > n) return E_CORRUPT;
            len = (tag >> 2) + 1;
            off = (size_t)in[i] | (size_t)in[i + 1] << 8;
            i += 2;
            break;
        default:
            if (i + 4 > n) return E_CORRUPT;
            len = (tag >> 2) + 1;
            off = (size_t)in[i] | (size_t)in[i + 1] << 8 | (size_t)in[i + 2] << 16 | (size_t)in[i + 3] << 24;
            i += 4;
            break;
        }
        if (off == 0 || off > op || op + len > ulen) return E_CORRUPT;
        for (size_t k = 0; k < len; k++) out[op + k] = out[op + k - off];   /* byte-wise: overlap allowed */
        op += len;
    }
    if (op != ulen) return E_CORRUPT;
    return (int64_t)op;
}

/* Test-vector generator (NOT part of the decode restatement): a greedy Snappy compressor.
 * mode 0 = Google-style: independent 64 KiB blocks (what snappy-java produces);
 * mode 1 = one window over the whole input: copies reach back across 64 KiB blocks
 *          (valid Snappy that exercises the decoder's non-block path). Returns bytes or <0. */
static size_t put_varint(uint8_t* o, uint64_t v) { size_t i = 0; while (v >= 128) { o[i++] = (uint8_t)(v | 128); v >>= 7; } o[i++] = (uint8_t)v; return i; }
static size_t emit_literal(uint8_t* o, const uint8_t* s, size_t len) {
    size_t i = 0, n = len - 1;
    if (n < 60) o[i++] = (uint8_t)(n << 2);
    else { int nb = n < 256 ? 1 : n < 65536 ? 2 : n < (1u << 24) ? 3 : 4; o[i++] = (uint8_t)((59 + nb) << 2); for (int k = 0; k < nb; k++) o[i++] = (uint8_t)(n >> (8 * k)); }
    memcpy(o + i, s, len);
    return i + len;
}
static size_t emit_copy(uint8_t* o, size_t off, size_t len) {
    size_t i = 0;
    while (len > 0) {
        size_t l = len > 64 ? (len - 64 >= 4 ? 64 : len - 4) : len;
        if (l >= 4 && l <= 11 && off < 2048) { o[i++] = (uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5)); o[i++] = (uint8_t)off; }
        else if (off < 65536) { o[i++] = (uint8_t)(2 | ((l - 1) << 2)); o[i++] = (uint8_t)off; o[i++] = (uint8_t)(off >> 8); }
        else { o[i++] = (uint8_t)(3 | ((l - 1) << 2)); for (int k = 0; k < 4; k++) o[i++] = (uint8_t)(off >> (8 * k)); }
        len -= l;
    }
    return i;
}
int64_t pfo_snappy_compress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, int mode) {
    if (cap < 32 + n + n / 6) return E_CAP;
    size_t o = put_varint(out, n);
    enum { HB = 14 };
    int64_t* table = (int64_t*)malloc(sizeof(int64_t) << HB);
    size_t bstart = 0;
    for (int i = 0; i < (1 << HB); i++) table[i] = -1;
    while (bstart < n) {
        /* mode 0/2: tokens never cross a 64 KiB output boundary; mode 0 also restarts the match
         * window per block, mode 2 keeps matching into earlier blocks (cross-block copies). */
        size_t bend = mode == 1 ? n : (n - bstart > 65536 ? bstart + 65536 : n);
        if (mode == 0) for (int i = 0; i < (1 << HB); i++) table[i] = -1;
        size_t lo = mode == 0 ? bstart : 0;
        size_t i = bstart, lit = bstart;
        while (i + 4 <= bend) {
            uint32_t v = (uint32_t)in[i] | (uint32_t)in[i + 1] << 8 | (uint32_t)in[i + 2] << 16 | (uint32_t)in[i + 3] << 24;
            uint32_t h = (v * 0x1e35a7bdu) >> (32 - HB);
            int64_t cand = table[h];
            table[h] = (int64_t)i;
            if (cand >= (int64_t)lo && memcmp(in + cand, in + i, 4) == 0) {
                size_t len = 4;
                while (i + len < bend && in[cand + len] == in[i + len]) len++;
                if (lit < i) o += emit_literal(out + o, in + lit, i - lit);
                o += emit_copy(out + o, i - (size_t)cand, len);
                i += len;
                lit = i;
            } else i++;
        }
        if (lit < bend) o += emit_literal(out + o, in + lit, bend - lit);
        bstart = bend;
    }
    free(table);
    return (int64_t)o;
}

/* ------------------------------------------------------------------ bit helpers */
static int bit_width_of(uint32_t max_level) {  /* BytesUtils.getWidthFromMaxInt */
    int w = 0; while (max_level) { w++; max_level >>= 1; } return w;
}
static uint64_t get_bits_le(const uint8_t* buf, size_t nbytes, uint64_t bitpos, int w) {
    /* little-endian bit packing (LSB first), bytes past nbytes read as 0 */
    uint64_t v = 0;
    for (int k = 0; k < w; k++) {
        uint64_t b = bitpos + k;
        size_t by = (size_t)(b >> 3);
        if (by < nbytes && ((buf[by] >> (b & 7)) & 1)) v |= 1ull << k;
    }
    return v;
}

/* RunLengthBitPackingHybridDecoder(bitWidth, in): decode exactly `count` values.
 * RLE run: header>>1 repeats of a ceil(bw/8)-byte LE value; bit-packed run: (header>>1)*8
 * values from (header>>1)*bw bytes, truncated to what is left of the stream (parquet-mr
 * reads min(bytes, available) and zero-pads). A run header that cannot be read while
 * values are still owed is a decoding error. */
static int rle_hybrid_decode(const uint8_t* p, size_t n, int bw, uint32_t* out, int64_t count) {
    size_t i = 0; int64_t k = 0;
    if (bw < 0 || bw > 32) return E_CORRUPT;
    while (k < count) {
        uint64_t h = 0; int sh = 0;
        for (;;) {
            if (i >= n || sh > 35) return E_CORRUPT;
            uint8_t c = p[i++];
            h |= (uint64_t)(c & 0x7f) << sh;
            if (!(c & 0x80)) break;
            sh += 7;
        }
        if (h & 1) {
            uint64_t groups = h >> 1;
            uint64_t nb = groups * (uint64_t)bw;
            size_t avail = n - i;
            size_t take = nb < avail ? (size_t)nb : avail;
            uint64_t nv = groups * 8;
            for (uint64_t j = 0; j < nv && k < count; j++)
                out[k++] = (uint32_t)get_bits_le(p + i, take, j * (uint64_t)bw, bw);
            i += take;
        } else {
            uint64_t run = h >> 1;
            int nbv = (bw + 7) / 8;
            if (i + nbv > n) return E_CORRUPT;
            uint32_t v = 0;
            for (int b = 0; b < nbv; b++) v |= (uint32_t)p[i + b] << (8 * b);
            i += nbv;
            for (uint64_t j = 0; j < run && k < count; j++) out[k++] = v;
        }
    }
    return E_OK;
}

/* Deprecated BIT_PACKED levels (ByteBitPackingValuesReader, big-endian bit order). */
static int bitpacked_be_decode(const uint8_t* p, size_t n, int bw, uint32_t* out, int64_t count) {
    for (int64_t k = 0; k < count; k++) {
        uint32_t v = 0;
        for (int b = 0; b < bw; b++) {
            uint64_t bit = (uint64_t)k * bw + b;
            size_t by = (size_t)(bit >> 3);
            if (by >= n) return E_CORRUPT;
            v = (v << 1) | ((p[by] >> (7 - (bit & 7))) & 1);
        }
        out[k] = v;
    }
    return E_OK;
}

static int rd_uvarint(const uint8_t* p, size_t n, size_t* i, uint64_t* v) {
    uint64_t r = 0; int sh = 0;
    for (;;) {
        if (*i >= n || sh > 63) return E_CORRUPT;
        uint8_t c = p[(*i)++];
        r |= (uint64_t)(c & 0x7f) << sh;
        if (!(c & 0x80)) break;
        sh += 7;
    }
    *v = r; return 0;
}

/* DeltaBinaryPackingValuesReader / ...ForLong: header <block size><miniblocks><total><zigzag first>,
 * blocks of <zigzag min delta><bit widths><miniblocks>; v[i] = v[i-1] + min_delta + d[i] in
 * two's-complement wrap-around (32-bit for INT32, 64-bit for INT64). A miniblock is read
 * whole while values remain (parquet-mr unpacks all 8-value groups of it). Writes
 * *consumed = bytes used. */
static int delta_binary_decode(const uint8_t* p, size_t n, int is64, uint64_t* out, int64_t need,
                               size_t* consumed, int64_t* total_out) {
    size_t i = 0; uint64_t block, nmini, total, zz;
    if (rd_uvarint(p, n, &i, &block) || rd_uvarint(p, n, &i, &nmini) || rd_uvarint(p, n, &i, &total) || rd_uvarint(p, n, &i, &zz))
        return E_CORRUPT;
    /* parquet-mr 1.12.2 DeltaBinaryPackingConfig: only "miniBlockSize must be multiple of 8" (the format
     * spec's block % 128 / miniblock % 32 are writer rules it does not enforce on read) */
    if (nmini == 0 || block == 0 || block % nmini || (block / nmini) % 8 || nmini > block) return E_CORRUPT;
    uint64_t vpm = block / nmini;
    int64_t first = (int64_t)(zz >> 1) ^ -(int64_t)(zz & 1);
    if (total_out) *total_out = (int64_t)total;
    if ((uint64_t)need > total) return E_CORRUPT;
    uint64_t have = 0, prev = (uint64_t)first;
    if (total > 0) { if (need > 0) out[0] = is64 ? prev : (uint64_t)(uint32_t)prev; have = 1; }
    uint8_t widths[256];
    while (have < total) {
        uint64_t mz;
        if (rd_uvarint(p, n, &i, &mz)) return E_CORRUPT;
        int64_t min_delta = (int64_t)(mz >> 1) ^ -(int64_t)(mz & 1);
        if (!is64) min_delta = (int32_t)min_delta;
        if (nmini > 256 || i + nmini > n) return E_CORRUPT;
        memcpy(widths, p + i, nmini); i += nmini;
        for (uint64_t m = 0; m < nmini && have < total; m++) {
            int w = widths[m];
            if (w > (is64 ? 64 : 32)) return E_CORRUPT;
            size_t nb = (size_t)(vpm * (uint64_t)w / 8);
            if (i + nb > n) return E_CORRUPT;
            for (uint64_t j = 0; j < vpm; j++) {
                uint64_t d = 0;
                for (int b = 0; b < w; b++) {
                    uint64_t bit = j * (uint64_t)w + b;
                    if ((p[i + (bit >> 3)] >> (bit & 7)) & 1) d |= 1ull << b;
                }
                if (have < total) {
                    uint64_t v = prev + (uint64_t)min_delta + d;
                    if (!is64) v = (uint32_t)v;
                    if ((int64_t)have < need) out[have] = v;
                    prev = v; have++;
                }
            }
            i += nb;
        }
    }
    *consumed = i;
    return E_OK;
}

/* ------------------------------------------------------------------ page walk */
typedef struct {
    int type; int32_t usize, csize;
    int32_t num_values, encoding, def_enc, rep_enc, num_nulls, num_rows, def_bytes, rep_bytes, is_compressed;
    int has_crc; uint32_t crc;                 /* PageHeader.crc (field 4) */
    const uint8_t* body;
} page_t;

static int parse_page_header(tr_t* r, page_t* pg) {
    int last = 0, t, id;
    memset(pg, 0, sizeof(*pg)); pg->type = -1; pg->is_compressed = 1;
    while ((id = tr_field(r, &last, &t))) {
        if (id == 1) pg->type = (int)tr_int(r, t);
        else if (id == 2) pg->usize = (int32_t)tr_int(r, t);
        else if (id == 3) pg->csize = (int32_t)tr_int(r, t);
        else if (id == 4 && t == 5) { pg->crc = (uint32_t)tr_int(r, t); pg->has_crc = 1; }
        else if ((id == 5 || id == 7 || id == 8) && t == 12) {
            int l2 = 0, t2, f2;
            while ((f2 = tr_field(r, &l2, &t2))) {
                if (id == 5) {
                    if (f2 == 1) pg->num_values = (int32_t)tr_int(r, t2);
                    else if (f2 == 2) pg->encoding = (int32_t)tr_int(r, t2);
                    else if (f2 == 3) pg->def_enc = (int32_t)tr_int(r, t2);
                    else if (f2 == 4) pg->rep_enc = (int32_t)tr_int(r, t2);
                    else tr_skip(r, t2, 0);
                } else if (id == 7) {
                    if (f2 == 1) pg->num_values = (int32_t)tr_int(r, t2);
                    else if (f2 == 2) pg->encoding = (int32_t)tr_int(r, t2);
                    else tr_skip(r, t2, 0);
                } else {
                    if (f2 == 1) pg->num_values = (int32_t)tr_int(r, t2);
                    else if (f2 == 2) pg->num_nulls = (int32_t)tr_int(r, t2);
                    else if (f2 == 3) pg->num_rows = (int32_t)tr_int(r, t2);
                    else if (f2 == 4) pg->encoding = (int32_t)tr_int(r, t2);
                    else if (f2 == 5) pg->def_bytes = (int32_t)tr_int(r, t2);
                    else if (f2 == 6) pg->rep_bytes = (int32_t)tr_int(r, t2);
                    else if (f2 == 7) pg->is_compressed = tr_bool(r, t2);
                    else tr_skip(r, t2, 0);
                }
                if (r->err) return -1;
            }
        } else tr_skip(r, t, 0);
        if (r->err) return -1;
    }
    return r->err ? -1 : 0;
}

/* ------------------------------------------------------------------ column decode state */
typedef struct {
    const leaf_t* L; int width;
    /* dictionary */
    int has_dict; int64_t dict_n; uint8_t* dict_fixed; int32_t* dict_off; uint8_t* dict_chars; buf_t dict_store;
    /* outputs */
    buf_t values, validity_bits, offsets, chars, list_off, list_valid, defs, reps;
    int64_t entries, slots, nvalues, rows, nchars;
    char* err; int errlen;
} col_t;

static int type_width(const leaf_t* L) {
    switch (L->type) {
    case 0: return 1; case 1: return 4; case 2: return 8; case 3: return 12; case 4: return 4; case 5: return 8;
    case 6: return 0; case 7: return L->type_length;
    default: return -1;
    }
}

static void push_bit(buf_t* b, int64_t idx, int bit) {
    size_t by = (size_t)(idx >> 3);
    while (b->n <= by) { uint8_t z = 0; buf_put(b, &z, 1); }
    if (bit) b->p[by] |= (uint8_t)(1u << (idx & 7));
}

/* decode the page's non-null values into a temporary: fixed-width -> vals (nv*width);
 * BYTE_ARRAY -> (voff, vchars) */
typedef struct { buf_t fixed; buf_t off; buf_t chr; } vals_t;

static int decode_plain_bytearray(const uint8_t* p, size_t n, int64_t nv, vals_t* V, size_t* used) {
    size_t i = 0; int32_t o = 0;
    buf_put(&V->off, &o, 4);
    for (int64_t k = 0; k < nv; k++) {
        if (i + 4 > n) return E_CORRUPT;
        uint32_t len = (uint32_t)p[i] | (uint32_t)p[i + 1] << 8 | (uint32_t)p[i + 2] << 16 | (uint32_t)p[i + 3] << 24;
        i += 4;
        if (len > n - i) return E_CORRUPT;
        buf_put(&V->chr, p + i, len); i += len;
        o = (int32_t)V->chr.n; buf_put(&V->off, &o, 4);
    }
    if (used) *used = i;
    return E_OK;
}

static int decode_values(col_t* C, int enc, const uint8_t* p, size_t n, int64_t nv, vals_t* V) {
    const leaf_t* L = C->L; int w = C->width;
    if (nv == 0) return E_OK;
    if (enc == 2 || enc == 8) {                     /* PLAIN_DICTIONARY / RLE_DICTIONARY */
        if (!C->has_dict) return E_CORRUPT;
        if (n < 1) return E_CORRUPT;
        int bw = p[0];
        if (bw > 32) return E_CORRUPT;
        uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * nv);
        int rc = rle_hybrid_decode(p + 1, n - 1, bw, ids, nv);
        if (rc) { free(ids); return rc; }
        if (L->type == 6) {
            int32_t o = 0; buf_put(&V->off, &o, 4);
            for (int64_t k = 0; k < nv; k++) {
                if ((int64_t)ids[k] >= C->dict_n) { free(ids); return E_CORRUPT; }
                int32_t a = C->dict_off[ids[k]], b = C->dict_off[ids[k] + 1];
                buf_put(&V->chr, C->dict_chars + a, b - a);
                o = (int32_t)V->chr.n; buf_put(&V->off, &o, 4);
            }
        } else {
            for (int64_t k = 0; k < nv; k++) {
                if ((int64_t)ids[k] >= C->dict_n) { free(ids); return E_CORRUPT; }
                buf_put(&V->fixed, C->dict_fixed + (size_t)ids[k] * w, w);
            }
        }
        free(ids);
        return E_OK;
    }
    if (enc == 0) {                                  /* PLAIN */
        if (L->type == 6) return decode_plain_bytearray(p, n, nv, V, NULL);
        if (L->type == 0) {                          /* BooleanPlainValuesReader: LSB-first bits */
            if ((size_t)((nv + 7) / 8) > n) return E_CORRUPT;
            for (int64_t k = 0; k < nv; k++) { uint8_t b = (p[k >> 3] >> (k & 7)) & 1; buf_put(&V->fixed, &b, 1); }
            return E_OK;
        }
        if ((uint64_t)nv * (uint64_t)w > n) return E_CORRUPT;
        return buf_put(&V->fixed, p, (size_t)nv * w) ? E_CAP : E_OK;
    }
    if (enc == 3 && L->type == 0) {                  /* RLE boolean: 4-byte length + hybrid bw=1 */
        if (n < 4) return E_CORRUPT;
        uint32_t len = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
        if (len > n - 4) return E_CORRUPT;
        uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * nv);
        int rc = rle_hybrid_decode(p + 4, len, 1, tmp, nv);
        for (int64_t k = 0; k < nv && !rc; k++) { uint8_t b = (uint8_t)tmp[k]; buf_put(&V->fixed, &b, 1); }
        free(tmp);
        return rc;
    }
    if (enc == 5 && (L->type == 1 || L->type == 2)) { /* DELTA_BINARY_PACKED */
        uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * nv);
        size_t used; int64_t tot;
        int rc = delta_binary_decode(p, n, L->type == 2, tmp, nv, &used, &tot);
        for (int64_t k = 0; k < nv && !rc; k++) {
            if (L->type == 2) buf_put(&V->fixed, &tmp[k], 8);
            else { uint32_t v = (uint32_t)tmp[k]; buf_put(&V->fixed, &v, 4); }
        }
        free(tmp);
        return rc;
    }
    if (enc == 6 && L->type == 6) {                  /* DELTA_LENGTH_BYTE_ARRAY */
        uint64_t* lens = (uint64_t*)malloc(sizeof(uint64_t) * nv);
        size_t used; int64_t tot;
        int rc = delta_binary_decode(p, n, 0, lens, nv, &used, &tot);
        if (!rc) {
            size_t i = used; int32_t o = 0; buf_put(&V->off, &o, 4);
            for (int64_t k = 0; k < nv; k++) {
                int32_t len = (int32_t)(uint32_t)lens[k];
                if (len < 0 || (size_t)len > n - i) { rc = E_CORRUPT; break; }
                buf_put(&V->chr, p + i, len); i += len;
                o = (int32_t)V->chr.n; buf_put(&V->off, &o, 4);
            }
        }
        free(lens);
        return rc;
    }
    if (enc == 7 && (L->type == 6 || L->type == 7)) { /* DELTA_BYTE_ARRAY: prefix lengths + DLBA suffixes */
        uint64_t* pre = (uint64_t*)malloc(sizeof(uint64_t) * nv);
        uint64_t* suf = (uint64_t*)malloc(sizeof(uint64_t) * nv);
        size_t u1, u2; int64_t t1, t2;
        int rc = delta_binary_decode(p, n, 0, pre, nv, &u1, &t1);
        if (!rc) rc = delta_binary_decode(p + u1, n - u1, 0, suf, nv, &u2, &t2);
        if (!rc) {
            size_t i = u1 + u2; int32_t o = 0;
            int64_t prev_start = 0, prev_len = 0;
            if (L->type == 6) buf_put(&V->off, &o, 4);
            for (int64_t k = 0; k < nv; k++) {
                int32_t pl = (int32_t)(uint32_t)pre[k], sl = (int32_t)(uint32_t)suf[k];
                if (pl < 0 || sl < 0 || pl > prev_len || (size_t)sl > n - i) { rc = E_CORRUPT; break; }
                buf_t* dst = L->type == 6 ? &V->chr : &V->fixed;
                int64_t start = (int64_t)dst->n;
                if (buf_reserve(dst, (size_t)pl + sl)) { rc = E_CAP; break; }
                memmove(dst->p + dst->n, dst->p + prev_start, pl); dst->n += pl;
                buf_put(dst, p + i, sl); i += sl;
                prev_start = start; prev_len = pl + sl;
                if (L->type == 7 && prev_len != w) { rc = E_CORRUPT; break; }
                if (L->type == 6) { o = (int32_t)V->chr.n; buf_put(&V->off, &o, 4); }
            }
        }
        free(pre); free(suf);
        return rc;
    }
    if (enc == 9 && (L->type == 4 || L->type == 5)) { /* BYTE_STREAM_SPLIT */
        if ((uint64_t)nv * w > n) return E_CORRUPT;
        size_t total = n / w;                          /* streams are total-values long */
        if (buf_reserve(&V->fixed, (size_t)nv * w)) return E_CAP;
        for (int64_t k = 0; k < nv; k++)
            for (int b = 0; b < w; b++) V->fixed.p[V->fixed.n + k * w + b] = p[(size_t)b * total + k];
        V->fixed.n += (size_t)nv * w;
        return E_OK;
    }
    return E_ENC;
}

static int decode_dictionary(col_t* C, const page_t* pg, const uint8_t* body, size_t n) {
    if (pg->encoding != 0 && pg->encoding != 2) return E_ENC;   /* Encoding.PLAIN[_DICTIONARY].initDictionary */
    int64_t nv = pg->num_values;
    if (nv < 0) return E_CORRUPT;
    vals_t V; memset(&V, 0, sizeof V);
    if (C->L->type == 6) {
        size_t used;
        int rc = decode_plain_bytearray(body, n, nv, &V, &used);
        if (rc) { free(V.off.p); free(V.chr.p); return rc; }
        C->dict_off = (int32_t*)V.off.p; C->dict_chars = V.chr.p;
    } else {
        if (C->L->type == 0) return E_ENC;             /* boolean dictionaries are not defined */
        if ((uint64_t)nv * C->width > n) return E_CORRUPT;
        C->dict_fixed = (uint8_t*)malloc((size_t)nv * C->width + 1);
        memcpy(C->dict_fixed, body, (size_t)nv * C->width);
    }
    C->dict_n = nv; C->has_dict = 1;
    return E_OK;
}

static int decode_data_page(col_t* C, const page_t* pg, const uint8_t* lv, size_t lvn, const uint8_t* vals, size_t valn, int v2) {
    const leaf_t* L = C->L;
    int64_t ne = pg->num_values;
    if (ne < 0) return E_CORRUPT;
    uint32_t* rep = (uint32_t*)calloc(ne ? ne : 1, 4);
    uint32_t* def = (uint32_t*)calloc(ne ? ne : 1, 4);
    int rc = E_OK;
    size_t pos = 0;
    /* levels: v1 = [rep][def] each 4-byte-length-prefixed RLE (or BIT_PACKED); v2 = raw hybrid */
    for (int which = 0; which < 2 && !rc; which++) {
        int maxl = which == 0 ? L->max_rep : L->max_def;
        uint32_t* dst = which == 0 ? rep : def;
        if (maxl == 0) continue;
        int bw = bit_width_of((uint32_t)maxl);
        if (v2) {
            size_t len = which == 0 ? (size_t)pg->rep_bytes : (size_t)pg->def_bytes;
            size_t start = which == 0 ? 0 : (size_t)pg->rep_bytes;
            if (start + len > lvn) { rc = E_CORRUPT; break; }
            rc = rle_hybrid_decode(lv + start, len, bw, dst, ne);
        } else {
            int enc = which == 0 ? pg->rep_enc : pg->def_enc;
            if (enc == 3) {
                if (pos + 4 > lvn) { rc = E_CORRUPT; break; }
                uint32_t len = (uint32_t)lv[pos] | (uint32_t)lv[pos + 1] << 8 | (uint32_t)lv[pos + 2] << 16 | (uint32_t)lv[pos + 3] << 24;
                pos += 4;
                if (len > lvn - pos) { rc = E_CORRUPT; break; }
                rc = rle_hybrid_decode(lv + pos, len, bw, dst, ne);
                pos += len;
            } else if (enc == 4) {
                size_t len = (size_t)(((uint64_t)ne * bw + 7) / 8);
                if (pos + len > lvn) { rc = E_CORRUPT; break; }
                rc = bitpacked_be_decode(lv + pos, len, bw, dst, ne);
                pos += len;
            } else rc = E_ENC;
        }
        for (int64_t k = 0; k < ne && !rc; k++) if ((int)dst[k] > maxl) rc = E_CORRUPT;
    }
    if (!v2) { vals = lv + pos; valn = lvn - pos; }
    int64_t nv = 0;
    for (int64_t k = 0; k < ne && !rc; k++) if ((int)def[k] == L->max_def) nv++;
    vals_t V; memset(&V, 0, sizeof V);
    if (!rc) rc = decode_values(C, pg->encoding, vals, valn, nv, &V);
    if (!rc) {
        int64_t vi = 0; int w = C->width;
        for (int64_t k = 0; k < ne; k++) {
            int d = (int)def[k], r = (int)rep[k];
            if (L->max_rep > 0) {
                uint8_t db = (uint8_t)d, rb = (uint8_t)r;
                buf_put(&C->defs, &db, 1); buf_put(&C->reps, &rb, 1);
                if (r == 0) {
                    if (L->max_rep == 1) {
                        int32_t so = (int32_t)C->slots; buf_put(&C->list_off, &so, 4);
                        push_bit(&C->list_valid, C->rows, d >= L->list_null_def);
                    }
                    C->rows++;
                }
            } else C->rows++;
            int is_slot = L->max_rep == 0 || d >= L->repeated_def;
            if (!is_slot) continue;
            int present = d == L->max_def;
            if (L->max_def > 0) push_bit(&C->validity_bits, C->slots, present);
            if (L->type == 6) {
                if (present) {
                    int32_t a = ((int32_t*)V.off.p)[vi], b = ((int32_t*)V.off.p)[vi + 1];
                    buf_put(&C->chars, V.chr.p + a, b - a);
                }
                int32_t o = (int32_t)C->chars.n; buf_put(&C->offsets, &o, 4);
            } else {
                if (present) buf_put(&C->values, V.fixed.p + vi * w, w);
                else { uint8_t z[64] = { 0 }; int left = w; while (left > 0) { int t = left > 64 ? 64 : left; buf_put(&C->values, z, t); left -= t; } }
            }
            if (present) vi++;
            C->slots++;
        }
        C->nvalues += nv;
        C->entries += ne;
    }
    free(V.fixed.p); free(V.off.p); free(V.chr.p);
    free(rep); free(def);
    return rc;
}

int pfo_decode(pfo_file* f, int rg, int col, pfo_column* out) {
    memset(out, 0, sizeof(*out));
    if (rg < 0 || rg >= f->nrg || col < 0 || col >= f->nleaves) { out->status = E_ARG; snprintf(out->error, sizeof out->error, "bad index"); return E_ARG; }
    const leaf_t* L = &f->leaves[col];
    const chunk_meta* m = &f->rgs[rg].cols[col];
    col_t C; memset(&C, 0, sizeof C);
    C.L = L; C.width = type_width(L);
    out->physical_type = L->type; out->type_length = L->type_length; out->max_def = L->max_def; out->max_rep = L->max_rep;
    out->repeated_def = L->repeated_def; out->list_null_def = L->list_null_def; out->width = C.width;
    int rc = E_OK;
    if (C.width < 0 || (L->type == 7 && L->type_length <= 0)) { rc = E_TYPE; snprintf(out->error, sizeof out->error, "Unsupported type"); goto done; }
    if (m->codec != 0 && m->codec != 1) { rc = E_CODEC; snprintf(out->error, sizeof out->error, "unsupported codec %d", m->codec); goto done; }
    {
        /* ColumnChunkMetaData.getStartingPos(): dictionary offset when it precedes the data pages */
        int64_t start = m->data_page_offset;
        if (m->has_dict_offset && m->dictionary_page_offset > 0 && m->dictionary_page_offset < start) start = m->dictionary_page_offset;
        int64_t end = start + m->total_compressed_size;
        if (m->num_values == 0) goto done;   /* empty chunk: nothing to read */
        if (start < 4 || end > (int64_t)f->size || m->total_compressed_size < 0) { rc = E_CORRUPT; snprintf(out->error, sizeof out->error, "chunk out of file"); goto done; }
        int64_t seen = 0;
        const uint8_t* p = f->data + start;
        const uint8_t* e = f->data + end;
        buf_t scratch; memset(&scratch, 0, sizeof scratch);
        /* parquet-mr Chunk.readAllPages: read pages until num_values level entries are seen */
        while (seen < m->num_values && !rc) {
            tr_t r = { p, e, 0 };
            page_t pg;
            if (parse_page_header(&r, &pg) || pg.csize < 0 || pg.usize < 0 || (int64_t)(e - r.p) < pg.csize) { rc = E_CORRUPT; snprintf(out->error, sizeof out->error, "corrupt page header"); break; }
            const uint8_t* body = r.p;
            p = body + pg.csize;
            if (pg.type != 0 && pg.type != 2 && pg.type != 3) continue;   /* index / unknown pages skipped */
            int v2 = pg.type == 3;
            size_t lvl_len = v2 ? (size_t)pg.rep_bytes + (size_t)pg.def_bytes : 0;
            if (v2 && (pg.rep_bytes < 0 || pg.def_bytes < 0 || lvl_len > (size_t)pg.csize)) { rc = E_CORRUPT; break; }
            const uint8_t* payload = body + lvl_len;
            size_t plen = (size_t)pg.csize - lvl_len;
            size_t ulen = (size_t)pg.usize - (v2 ? lvl_len : 0);
            if (v2 && lvl_len > (size_t)pg.usize) { rc = E_CORRUPT; break; }
            int compressed = m->codec == 1 && (!v2 || pg.is_compressed);
            if (compressed) {
                scratch.n = 0;
                if (buf_reserve(&scratch, ulen + 1)) { rc = E_CAP; break; }
                int64_t got = pfo_snappy_uncompress(payload, plen, scratch.p, ulen);
                if (got < 0 || (size_t)got != ulen) { rc = E_CORRUPT; snprintf(out->error, sizeof out->error, "snappy: corrupt page"); break; }
                payload = scratch.p; plen = ulen;
            }
            if (pg.type == 2) {
                if (C.has_dict) { rc = E_CORRUPT; break; }
                rc = decode_dictionary(&C, &pg, payload, plen);
                continue;
            }
            if (v2) rc = decode_data_page(&C, &pg, body, lvl_len, payload, plen, 1);
            else rc = decode_data_page(&C, &pg, payload, plen, NULL, 0, 0);
            seen += pg.num_values;
        }
        free(scratch.p);
        if (!rc && seen != m->num_values) rc = E_CORRUPT;
    }
done:
    out->status = rc;
    if (rc) { if (!out->error[0]) snprintf(out->error, sizeof out->error, "decode failed (%d)", rc); }
    {
        int32_t last = (int32_t)C.slots;
        if (!rc && L->max_rep == 1) buf_put(&C.list_off, &last, 4);
        if (!rc && L->type == 6 && C.offsets.n == 0) { int32_t z = 0; buf_put(&C.offsets, &z, 4); }
    }
    out->num_entries = C.entries; out->num_slots = C.slots; out->num_values = C.nvalues; out->num_rows = C.rows;
    out->num_chars = (int64_t)C.chars.n;
    out->values = C.values.p;
    /* validity padded to ceil(slots/8) */
    if (L->max_def > 0) { while ((int64_t)C.validity_bits.n < (C.slots + 7) / 8) { uint8_t z = 0; buf_put(&C.validity_bits, &z, 1); } out->validity = C.validity_bits.p; }
    else free(C.validity_bits.p);
    if (L->type == 6) {
        /* prepend the leading 0 offset */
        int32_t* o = (int32_t*)malloc(sizeof(int32_t) * (C.slots + 1));
        o[0] = 0;
        if (C.slots) memcpy(o + 1, C.offsets.p, sizeof(int32_t) * C.slots);
        free(C.offsets.p);
        out->offsets = o; out->chars = C.chars.p;
    } else { free(C.offsets.p); free(C.chars.p); }
    if (L->max_rep == 1) {
        while ((int64_t)C.list_valid.n < (C.rows + 7) / 8) { uint8_t z = 0; buf_put(&C.list_valid, &z, 1); }
        out->list_offsets = (int32_t*)C.list_off.p; out->list_validity = C.list_valid.p;
    } else { free(C.list_off.p); free(C.list_valid.p); }
    if (L->max_rep > 0) { out->def_levels = C.defs.p; out->rep_levels = C.reps.p; }
    else { free(C.defs.p); free(C.reps.p); }
    free(C.dict_fixed); free(C.dict_off); free(C.dict_chars);
    return rc;
}

void pfo_free_column(pfo_column* c) {
    free(c->values); free(c->validity); free(c->offsets); free(c->chars);
    free(c->list_offsets); free(c->list_validity); free(c->def_levels); free(c->rep_levels);
    memset(c, 0, sizeof(*c));
}

/* ------------------------------------------------------------------ page walk + CRC32 (scan oracle) */
/* CRC-32 of java.util.zip.CRC32 / zlib (reflected polynomial 0xEDB88320, init and final xor ~0),
 * bit at a time. parquet-mr 1.12.2 ParquetFileReader.Chunk.verifyCrc compares it with PageHeader.crc
 * over the page's on-disk (compressed) bytes. */
uint32_t pfo_crc32(const uint8_t* p, size_t n) {
    uint32_t c = 0xffffffffu;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xedb88320u : c >> 1;
    }
    return c ^ 0xffffffffu;
}

/* parquet-mr Chunk.readAllPages: PageHeaders until num_values level entries are seen (the loop of
 * pfo_decode above); dictionary and data pages are listed, INDEX / unknown pages skipped. With
 * verify_crc, a listed page whose header carries a crc must match pfo_crc32 of its bytes
 * (usePageChecksumVerification). Returns the page count, or a negative status with *err_page. */
int pfo_chunk_pages(pfo_file* f, int rg, int col, pfo_page* out, int cap, int verify_crc, int* err_page) {
    *err_page = -1;
    if (rg < 0 || rg >= f->nrg || col < 0 || col >= f->nleaves) return E_ARG;
    const chunk_meta* m = &f->rgs[rg].cols[col];
    int64_t start = m->data_page_offset;
    if (m->has_dict_offset && m->dictionary_page_offset > 0 && m->dictionary_page_offset < start) start = m->dictionary_page_offset;
    const int64_t end = start + m->total_compressed_size;
    if (m->num_values == 0) return 0;
    if (start < 4 || end > (int64_t)f->size || m->total_compressed_size < 0) return E_CORRUPT;
    const uint8_t* base = f->data + start;
    const uint8_t* p = base;
    const uint8_t* e = f->data + end;
    int64_t seen = 0;
    int n = 0;
    while (seen < m->num_values) {
        if (p >= e) { *err_page = n; return E_CORRUPT; }
        tr_t r = { p, e, 0 };
        page_t pg;
        if (parse_page_header(&r, &pg) || pg.csize < 0 || (int64_t)(e - r.p) < pg.csize) { *err_page = n; return E_CORRUPT; }
        p = r.p + pg.csize;
        if (pg.type != 0 && pg.type != 2 && pg.type != 3) continue;
        if (pg.type == 2 && n > 0) { *err_page = n; return E_CORRUPT; }
        if (pg.type != 2) {
            if (pg.num_values < 0) { *err_page = n; return E_CORRUPT; }
            seen += pg.num_values;
        }
        if (n >= cap) { *err_page = n; return E_CAP; }
        pfo_page* o = &out[n];
        o->offset = (uint64_t)(r.p - base);
        o->compressed_size = pg.csize; o->uncompressed_size = pg.usize; o->page_type = pg.type;
        o->encoding = pg.encoding; o->num_values = pg.num_values; o->has_crc = pg.has_crc; o->crc = pg.crc;
        o->crc_ok = pg.has_crc ? pfo_crc32(r.p, (size_t)pg.csize) == pg.crc : 1;
        if (verify_crc && !o->crc_ok) { *err_page = n; return E_CORRUPT; }
        n++;
    }
    return n;
}
