// pf_write.cpp — host side of the write path: Thrift compact serialisation of PageHeaders (used by
// pf_encode_chunk) and the file writer (pf_writer_*: "PAR1", row groups, FileMetaData footer).
//
// The reference's writer is parquet-mr's ParquetWriter configured by
// src/main/java/blue/strategic/parquet/ParquetWriter.java:61-68 (SNAPPY, PARQUET_2_0), with a
// flat schema of the primitive types SimpleWriteSupport.writeField accepts (:143-160). Field ids
// follow parquet.thrift (parquet-format 2.9, what parquet-mr 1.12.2 writes). No GPU calls.
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pf_host.h"
#include "pfloor.h"

namespace pf {

namespace {
enum : uint8_t { T_TRUE = 1, T_FALSE = 2, T_I32 = 5, T_I64 = 6, T_BINARY = 8, T_LIST = 9, T_STRUCT = 12 };
}

// Thrift compact protocol writer (the inverse of pf_meta.cpp's ThriftReader).
struct ThriftWriter {
    std::vector<uint8_t>& out;
    std::vector<int> last{0};
    explicit ThriftWriter(std::vector<uint8_t>& o) : out(o) {}
    void uvarint(uint64_t v) {
        while (v >= 0x80) { out.push_back(uint8_t(v | 0x80)); v >>= 7; }
        out.push_back(uint8_t(v));
    }
    void zigzag(int64_t v) { uvarint((uint64_t(v) << 1) ^ uint64_t(v >> 63)); }
    void field(int id, uint8_t type) {
        const int d = id - last.back();
        if (d > 0 && d <= 15) out.push_back(uint8_t(d << 4 | type));
        else { out.push_back(type); zigzag(id); }
        last.back() = id;
    }
    void i32(int id, int64_t v) { field(id, T_I32); zigzag(v); }
    void i64(int id, int64_t v) { field(id, T_I64); zigzag(v); }
    void boolean(int id, bool v) { field(id, v ? T_TRUE : T_FALSE); }
    void binary(int id, const std::string& s) { field(id, T_BINARY); uvarint(s.size()); out.insert(out.end(), s.begin(), s.end()); }
    void begin_struct(int id) { field(id, T_STRUCT); last.push_back(0); }
    void end_struct() { out.push_back(0); last.pop_back(); }
    void list_header(int id, uint8_t elem, size_t n) {
        field(id, T_LIST);
        if (n < 15) out.push_back(uint8_t(n << 4 | elem));
        else { out.push_back(uint8_t(0xf0 | elem)); uvarint(n); }
    }
    void list_struct_begin() { last.push_back(0); }   // a struct element of a list
    void stop() { out.push_back(0); }
};

// PageHeader (parquet.thrift): 1 type, 2 uncompressed_page_size, 3 compressed_page_size,
// 7 dictionary_page_header {1 num_values, 2 encoding}, 8 data_page_header_v2 {1 num_values,
// 2 num_nulls, 3 num_rows, 4 encoding, 5 definition_levels_byte_length,
// 6 repetition_levels_byte_length, 7 is_compressed}.
void write_page_header(std::vector<uint8_t>& out, const PageHeaderOut& h) {
    ThriftWriter w(out);
    w.i32(1, h.page_type);
    w.i32(2, h.uncompressed_size);
    w.i32(3, h.compressed_size);
    if (h.page_type == PF_PAGE_DICTIONARY) {
        w.begin_struct(7);
        w.i32(1, h.num_values);
        w.i32(2, h.encoding);
        w.end_struct();
    } else {
        w.begin_struct(8);
        w.i32(1, h.num_values);
        w.i32(2, h.num_nulls);
        w.i32(3, h.num_rows);
        w.i32(4, h.encoding);
        w.i32(5, h.def_bytes);
        w.i32(6, 0);
        w.boolean(7, h.is_compressed);
        w.end_struct();
    }
    w.stop();
}

}  // namespace pf

using namespace pf;

namespace {
thread_local std::string w_err;
int werr(int code, const std::string& m) { w_err = m; return code; }

struct ChunkRec {
    int64_t file_offset = 0, size = 0, uncompressed = 0, num_values = 0, dict_offset = -1, data_offset = 0;
    int32_t data_encoding = 0, codec = 0;
};
struct RowGroupRec {
    int64_t num_rows = 0;
    std::vector<ChunkRec> chunks;
};
}  // namespace

struct pf_writer {
    FILE* fp = nullptr;
    int64_t pos = 0;
    std::vector<pf_write_field> fields;
    std::vector<std::string> names;
    std::vector<RowGroupRec> groups;
    RowGroupRec cur;
    bool failed = false;
};

namespace {
int put(pf_writer* w, const void* p, size_t n) {
    if (n && std::fwrite(p, 1, n, w->fp) != n) { w->failed = true; return werr(PF_ERR_IO, std::string("write: ") + std::strerror(errno)); }
    w->pos += int64_t(n);
    return PF_OK;
}
}  // namespace

extern "C" {

const char* pf_writer_last_error(void) { return w_err.c_str(); }

int pf_writer_open(const char* path, const pf_write_field* fields, int n_fields, pf_writer** out) {
    if (!path || !out || n_fields <= 0 || !fields) return werr(PF_ERR_INVALID_ARG, "bad arguments");
    *out = nullptr;
    for (int i = 0; i < n_fields; i++) {
        const int t = fields[i].physical_type;
        if (!fields[i].name) return werr(PF_ERR_INVALID_ARG, "null field name");
        if (t != PF_BOOLEAN && t != PF_INT32 && t != PF_INT64 && t != PF_FLOAT && t != PF_DOUBLE && t != PF_BYTE_ARRAY)
            return werr(PF_ERR_UNSUPPORTED_TYPE, std::string("We don't support writing type of ") + fields[i].name);
    }
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return werr(PF_ERR_IO, std::string("cannot create ") + path + ": " + std::strerror(errno));
    auto* w = new pf_writer;
    w->fp = fp;
    for (int i = 0; i < n_fields; i++) {
        w->names.emplace_back(fields[i].name);
        w->fields.push_back(fields[i]);
    }
    if (put(w, "PAR1", 4)) { std::fclose(fp); delete w; return PF_ERR_IO; }
    *out = w;
    return PF_OK;
}

int pf_writer_add_chunk(pf_writer* w, int field, const pf_encoded_chunk* c) {
    if (!w || !c || (c->size > 0 && !c->bytes)) return werr(PF_ERR_INVALID_ARG, "bad arguments");
    if (field != int(w->cur.chunks.size()) || field >= int(w->fields.size()))
        return werr(PF_ERR_STATE, "chunks must be added in field order, one per field");
    ChunkRec r;
    r.file_offset = w->pos;
    r.size = c->size;
    r.uncompressed = c->total_uncompressed_size;
    r.num_values = c->num_values;
    r.dict_offset = c->dictionary_page_offset >= 0 ? w->pos + c->dictionary_page_offset : -1;
    r.data_offset = w->pos + c->data_page_offset;
    r.data_encoding = c->data_encoding;
    r.codec = c->codec;
    int rc = put(w, c->bytes, size_t(c->size));
    if (rc) return rc;
    w->cur.chunks.push_back(r);
    return PF_OK;
}

int pf_writer_end_row_group(pf_writer* w, int64_t num_rows) {
    if (!w || num_rows < 0) return werr(PF_ERR_INVALID_ARG, "bad arguments");
    if (w->cur.chunks.size() != w->fields.size()) return werr(PF_ERR_STATE, "row group is missing chunks");
    for (const ChunkRec& c : w->cur.chunks)
        if (c.num_values != num_rows) return werr(PF_ERR_STATE, "chunk value count differs from the row count");
    w->cur.num_rows = num_rows;
    w->groups.push_back(w->cur);
    w->cur = RowGroupRec{};
    return PF_OK;
}

// FileMetaData: 1 version, 2 schema, 3 num_rows, 4 row_groups, 6 created_by.
int pf_writer_close(pf_writer* w) {
    if (!w) return werr(PF_ERR_INVALID_ARG, "null writer");
    int rc = PF_OK;
    if (!w->cur.chunks.empty()) rc = werr(PF_ERR_STATE, "unfinished row group");
    if (rc == PF_OK && !w->failed) {
        std::vector<uint8_t> f;
        ThriftWriter t(f);
        int64_t rows = 0;
        for (const RowGroupRec& g : w->groups) rows += g.num_rows;
        t.i32(1, 1);
        t.list_header(2, T_STRUCT, w->fields.size() + 1);
        {   // root: name, num_children
            t.list_struct_begin();
            t.binary(4, "schema");
            t.i32(5, int64_t(w->fields.size()));
            t.end_struct();
        }
        for (size_t i = 0; i < w->fields.size(); i++) {
            const pf_write_field& fd = w->fields[i];
            t.list_struct_begin();
            t.i32(1, fd.physical_type);
            t.i32(3, fd.optional ? 1 : 0);
            t.binary(4, w->names[i]);
            if (fd.physical_type == PF_BYTE_ARRAY && fd.utf8) {
                t.i32(6, 0);              // ConvertedType UTF8
                t.begin_struct(10);       // LogicalType { 1: STRING {} }
                t.begin_struct(1);
                t.end_struct();
                t.end_struct();
            }
            t.end_struct();
        }
        t.i64(3, rows);
        t.list_header(4, T_STRUCT, w->groups.size());
        for (const RowGroupRec& g : w->groups) {
            t.list_struct_begin();
            int64_t total_unc = 0, total_comp = 0;
            t.list_header(1, T_STRUCT, g.chunks.size());
            for (size_t i = 0; i < g.chunks.size(); i++) {
                const ChunkRec& c = g.chunks[i];
                total_unc += c.uncompressed;
                total_comp += c.size;
                t.list_struct_begin();
                t.i64(2, c.file_offset);
                t.begin_struct(3);   // ColumnMetaData
                t.i32(1, w->fields[i].physical_type);
                const bool dict = c.data_encoding == PF_ENC_RLE_DICTIONARY;
                t.list_header(2, T_I32, dict ? 3 : 2);
                t.zigzag(PF_ENC_PLAIN);
                t.zigzag(PF_ENC_RLE);
                if (dict) t.zigzag(PF_ENC_RLE_DICTIONARY);
                t.list_header(3, T_BINARY, 1);
                t.uvarint(w->names[i].size());
                f.insert(f.end(), w->names[i].begin(), w->names[i].end());
                t.i32(4, c.codec);
                t.i64(5, c.num_values);
                t.i64(6, c.uncompressed);
                t.i64(7, c.size);
                t.i64(9, c.data_offset);
                if (c.dict_offset >= 0) t.i64(11, c.dict_offset);
                t.end_struct();
                t.end_struct();
            }
            t.i64(2, total_unc);
            t.i64(3, g.num_rows);
            t.i64(5, g.chunks.empty() ? w->pos : g.chunks[0].file_offset);
            t.i64(6, total_comp);
            t.end_struct();
        }
        t.binary(6, "parquet-floor_amd (GPU encoder; parquet-mr 1.12.2 ParquetWriter settings)");
        t.stop();
        const uint32_t n = uint32_t(f.size());
        uint8_t tail[8];
        std::memcpy(tail, &n, 4);
        std::memcpy(tail + 4, "PAR1", 4);
        rc = put(w, f.data(), f.size());
        if (!rc) rc = put(w, tail, 8);
    } else if (rc == PF_OK) {
        rc = werr(PF_ERR_IO, "an earlier write failed");
    }
    if (std::fclose(w->fp) != 0 && rc == PF_OK) rc = werr(PF_ERR_IO, "close failed");
    delete w;
    return rc;
}

}  // extern "C"
