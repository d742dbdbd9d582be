// pf_meta.cpp — host-side Parquet metadata: footer FileMetaData + PageHeader walk.
//
// In the north-star deployment this is the Java side's job (parquet-mr's
// ParquetFileReader.open / readNextRowGroup, called at
// src/main/java/blue/strategic/parquet/ParquetReader.java:120 and :183); the Java bridge
// fills pf_chunk_desc from parquet-mr's own PageHeader objects. No JDK
// exists in this image, so this C++ parser produces the same descriptors for the C++/Python
// hosts and the tests. It reads Thrift compact protocol (parquet.thrift field ids) and
// never touches the GPU.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "pfloor.h"
#include "pf_host.h"

namespace pf {

namespace {

struct ThriftReader {
    const uint8_t* p;
    const uint8_t* end;

    [[noreturn]] static void fail(const char* what) { throw MetaError(what); }
    uint8_t byte() { if (p >= end) fail("truncated thrift"); return *p++; }
    uint64_t uvarint() {
        uint64_t v = 0;
        for (int sh = 0; sh < 70; sh += 7) {
            uint8_t c = byte();
            v |= uint64_t(c & 0x7f) << sh;
            if (!(c & 0x80)) return v;
        }
        fail("varint too long");
    }
    int64_t zigzag() { uint64_t v = uvarint(); return int64_t(v >> 1) ^ -int64_t(v & 1); }
    // Field iteration: returns false at STOP.
    bool field(int& last, int& id, int& type) {
        uint8_t h = byte();
        if (h == 0) return false;
        type = h & 0xf;
        int d = h >> 4;
        id = d ? last + d : int(zigzag());
        last = id;
        return true;
    }
    int64_t integer(int type) {
        if (type == 3) return int8_t(byte());
        if (type >= 4 && type <= 6) return zigzag();
        fail("expected integer");
    }
    bool boolean(int type) {
        if (type == 1) return true;
        if (type == 2) return false;
        fail("expected bool");
    }
    std::string str(int type) {
        if (type != 8) fail("expected binary");
        uint64_t n = uvarint();
        if (uint64_t(end - p) < n) fail("truncated string");
        std::string s(reinterpret_cast<const char*>(p), n);
        p += n;
        return s;
    }
    uint64_t list(int& etype) {
        uint8_t h = byte();
        uint64_t n = h >> 4;
        etype = h & 0xf;
        if (n == 15) n = uvarint();
        return n;
    }
    void skip(int type, int depth = 0) {
        if (depth > 64) fail("thrift nesting too deep");
        switch (type) {
        case 1: case 2: return;
        case 3: byte(); return;
        case 4: case 5: case 6: uvarint(); return;
        case 7: if (end - p < 8) fail("truncated double"); p += 8; return;
        case 8: { uint64_t n = uvarint(); if (uint64_t(end - p) < n) fail("truncated binary"); p += n; return; }
        case 9: case 10: {
            int et; uint64_t n = list(et);
            for (uint64_t i = 0; i < n; i++) { if (et == 1 || et == 2) byte(); else skip(et, depth + 1); }
            return;
        }
        case 11: {
            uint64_t n = uvarint();
            if (!n) return;
            uint8_t kv = byte();
            for (uint64_t i = 0; i < n; i++) { skip(kv >> 4, depth + 1); skip(kv & 0xf, depth + 1); }
            return;
        }
        case 12: {
            int last = 0, id, t;
            while (field(last, id, t)) skip(t, depth + 1);
            return;
        }
        default: fail("bad thrift type");
        }
    }
};

struct SchemaNode {
    std::string name;
    int type = -1, type_length = 0, repetition = 0, num_children = 0, converted = -1, logical = 0;
    int scale = 0, precision = 0;                 // SchemaElement 7/8, or LogicalType DECIMAL {1 scale, 2 precision}
};

SchemaNode read_schema_node(ThriftReader& r) {
    SchemaNode n;
    int last = 0, id, t;
    while (r.field(last, id, t)) {
        switch (id) {
        case 1: n.type = int(r.integer(t)); break;
        case 2: n.type_length = int(r.integer(t)); break;
        case 3: n.repetition = int(r.integer(t)); break;
        case 4: n.name = r.str(t); break;
        case 5: n.num_children = int(r.integer(t)); break;
        case 6: n.converted = int(r.integer(t)); break;
        case 7: n.scale = int(r.integer(t)); break;
        case 8: n.precision = int(r.integer(t)); break;
        case 10:
            if (t == 12) {   // LogicalType union: remember which member is set
                int l2 = 0, i2, t2;
                while (r.field(l2, i2, t2)) {
                    n.logical = i2;
                    if (i2 == 5 && t2 == 12) {   // DecimalType
                        int l3 = 0, i3, t3;
                        while (r.field(l3, i3, t3)) {
                            if (i3 == 1) n.scale = int(r.integer(t3));
                            else if (i3 == 2) n.precision = int(r.integer(t3));
                            else r.skip(t3);
                        }
                    } else r.skip(t2);
                }
            } else r.skip(t);
            break;
        default: r.skip(t);
        }
    }
    return n;
}

ChunkMeta read_column_chunk(ThriftReader& r) {
    ChunkMeta m;
    int last = 0, id, t;
    while (r.field(last, id, t)) {
        if (id == 3 && t == 12) {
            int l2 = 0, i2, t2;
            while (r.field(l2, i2, t2)) {
                switch (i2) {
                case 1: m.type = int(r.integer(t2)); break;
                case 4: m.codec = int(r.integer(t2)); break;
                case 5: m.num_values = r.integer(t2); break;
                case 6: m.total_uncompressed = r.integer(t2); break;
                case 7: m.total_compressed = r.integer(t2); break;
                case 9: m.data_page_offset = r.integer(t2); break;
                case 11: m.dictionary_page_offset = r.integer(t2); m.has_dict = true; break;
                default: r.skip(t2);
                }
            }
        } else r.skip(t);
    }
    return m;
}

}  // namespace

void FileMeta::parse_footer(const uint8_t* p, size_t n) {
    ThriftReader r{p, p + n};
    int last = 0, id, t;
    std::vector<SchemaNode> nodes;
    while (r.field(last, id, t)) {
        if (id == 2 && t == 9) {
            int et; uint64_t cnt = r.list(et);
            if (et != 12) ThriftReader::fail("schema list type");
            nodes.reserve(cnt);
            for (uint64_t i = 0; i < cnt; i++) nodes.push_back(read_schema_node(r));
        } else if (id == 3) {
            num_rows = r.integer(t);
        } else if (id == 4 && t == 9) {
            int et; uint64_t cnt = r.list(et);
            if (et != 12) ThriftReader::fail("row group list type");
            for (uint64_t g = 0; g < cnt; g++) {
                RowGroupMeta rg;
                int l2 = 0, i2, t2;
                while (r.field(l2, i2, t2)) {
                    if (i2 == 1 && t2 == 9) {
                        int e2; uint64_t nc = r.list(e2);
                        if (e2 != 12) ThriftReader::fail("column list type");
                        for (uint64_t c = 0; c < nc; c++) rg.columns.push_back(read_column_chunk(r));
                    } else if (i2 == 3) rg.num_rows = r.integer(t2);
                    else r.skip(t2);
                }
                row_groups.push_back(std::move(rg));
            }
        } else if (id == 6 && t == 8) {
            created_by = r.str(t);
        } else r.skip(t);
    }
    if (nodes.empty()) ThriftReader::fail("empty schema");
    // Leaf columns in schema order (MessageType.getColumns(); filtered at ParquetReader.java:126-128).
    size_t idx = 0;
    struct Frame { int def, rep, repeated_def, list_null_def; std::string path, top; };
    std::vector<std::pair<size_t, Frame>> stack;  // (remaining children, frame)
    std::function<void(int, Frame)> walk = [&](int depth, Frame f) {
        if (idx >= nodes.size() || depth > 100) ThriftReader::fail("schema tree");
        const SchemaNode& nd = nodes[idx++];
        Frame me = f;
        if (depth > 0) {
            if (nd.repetition == 1) me.def++;
            else if (nd.repetition == 2) { me.list_null_def = f.def; me.def++; me.rep++; me.repeated_def = me.def; }
            me.path = f.path.empty() ? nd.name : f.path + "." + nd.name;
            if (depth == 1) me.top = nd.name;
        }
        if (depth == 0 || nd.num_children > 0) {
            for (int c = 0; c < nd.num_children; c++) walk(depth + 1, me);
            return;
        }
        LeafMeta L;
        L.path = me.path; L.top = me.top;
        L.physical_type = nd.type; L.type_length = nd.type_length;
        L.max_def = me.def; L.max_rep = me.rep;
        L.repeated_def = me.rep ? me.repeated_def : 0;
        L.list_null_def = me.rep ? me.list_null_def : 0;
        L.converted_type = nd.converted; L.logical_type = nd.logical;
        L.scale = nd.scale; L.precision = nd.precision;
        leaves.push_back(std::move(L));
    };
    walk(0, Frame{0, 0, 0, 0, "", ""});
    for (auto& rg : row_groups)
        if (rg.columns.size() != leaves.size()) ThriftReader::fail("row group column count");
}

// Page headers of one chunk: parquet-mr Chunk.readAllPages reads pages until the chunk's
// num_values level entries have been seen; INDEX and unknown page types are skipped.
void FileMeta::walk_pages(const uint8_t* chunk, size_t size, const ChunkMeta& m, std::vector<pf_page_desc>& out) {
    out.clear();
    int64_t seen = 0;
    size_t off = 0;
    bool have_dict = false;
    while (seen < m.num_values) {
        ThriftReader r{chunk + off, chunk + size};
        pf_page_desc d{};
        d.is_compressed = 1;
        d.num_nulls = -1;   // v1 without page statistics: unknown
        d.page_type = -1;
        int last = 0, id, t;
        while (r.field(last, id, t)) {
            if (id == 1) d.page_type = int(r.integer(t));
            else if (id == 2) d.uncompressed_size = uint32_t(r.integer(t));
            else if (id == 3) d.compressed_size = uint32_t(r.integer(t));
            else if ((id == 5 || id == 7 || id == 8) && t == 12) {
                int l2 = 0, i2, t2;
                while (r.field(l2, i2, t2)) {
                    if (id == 5) {          // DataPageHeader
                        if (i2 == 1) d.num_values = int32_t(r.integer(t2));
                        else if (i2 == 2) d.encoding = int32_t(r.integer(t2));
                        else if (i2 == 3) d.def_encoding = int32_t(r.integer(t2));
                        else if (i2 == 4) d.rep_encoding = int32_t(r.integer(t2));
                        else if (i2 == 5 && t2 == 12) {   // Statistics: null_count (field 3), a routing hint
                            int l3 = 0, i3, t3;
                            while (r.field(l3, i3, t3)) {
                                if (i3 == 3) {
                                    const int64_t nn = r.integer(t3);
                                    d.num_nulls = nn >= 0 && nn <= INT32_MAX ? int32_t(nn) : -1;
                                } else r.skip(t3);
                            }
                        } else r.skip(t2);
                    } else if (id == 7) {   // DictionaryPageHeader
                        if (i2 == 1) d.num_values = int32_t(r.integer(t2));
                        else if (i2 == 2) d.encoding = int32_t(r.integer(t2));
                        else r.skip(t2);
                    } else {                // DataPageHeaderV2
                        if (i2 == 1) d.num_values = int32_t(r.integer(t2));
                        else if (i2 == 2) d.num_nulls = int32_t(r.integer(t2));
                        else if (i2 == 3) d.num_rows = int32_t(r.integer(t2));
                        else if (i2 == 4) d.encoding = int32_t(r.integer(t2));
                        else if (i2 == 5) d.def_bytes = int32_t(r.integer(t2));
                        else if (i2 == 6) d.rep_bytes = int32_t(r.integer(t2));
                        else if (i2 == 7) d.is_compressed = r.boolean(t2) ? 1 : 0;
                        else r.skip(t2);
                    }
                }
            } else r.skip(t);
        }
        size_t body = size_t(r.p - chunk);
        if (int32_t(d.compressed_size) < 0 || body + d.compressed_size > size) throw MetaError("page body exceeds chunk");
        d.offset = body;
        off = body + d.compressed_size;
        if (d.page_type == PF_PAGE_DICTIONARY) {
            if (have_dict || !out.empty()) throw MetaError("unexpected dictionary page");
            have_dict = true;
            out.push_back(d);
        } else if (d.page_type == PF_PAGE_DATA || d.page_type == PF_PAGE_DATA_V2) {
            if (d.num_values < 0) throw MetaError("negative num_values");
            if (d.page_type == PF_PAGE_DATA_V2 &&
                (d.def_bytes < 0 || d.rep_bytes < 0 ||
                 uint64_t(d.def_bytes) + uint64_t(d.rep_bytes) > d.compressed_size ||
                 uint64_t(d.def_bytes) + uint64_t(d.rep_bytes) > d.uncompressed_size))
                throw MetaError("v2 level lengths exceed page");
            out.push_back(d);
            seen += d.num_values;
        }
        if (off >= size && seen < m.num_values) throw MetaError("chunk ended before num_values");
    }
}

}  // namespace pf
