// pf_host.h — host-side metadata model (footer + page headers). Internal.
#pragma once
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "pfloor.h"

namespace pf {

struct MetaError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct ChunkMeta {
    int type = -1, codec = 0;
    int64_t num_values = 0, total_uncompressed = 0, total_compressed = 0;
    int64_t data_page_offset = 0, dictionary_page_offset = 0;
    bool has_dict = false;
    // ColumnChunkMetaData.getStartingPos(): the dictionary page offset when it precedes
    // the first data page, else the data page offset.
    int64_t start() const {
        if (has_dict && dictionary_page_offset > 0 && dictionary_page_offset < data_page_offset)
            return dictionary_page_offset;
        return data_page_offset;
    }
};

struct RowGroupMeta {
    int64_t num_rows = 0;
    std::vector<ChunkMeta> columns;
};

struct LeafMeta {
    std::string path, top;
    int physical_type = -1, type_length = 0, max_def = 0, max_rep = 0, repeated_def = 0, list_null_def = 0;
    int converted_type = -1, logical_type = 0;
    int scale = 0, precision = 0;
};

struct FileMeta {
    int64_t num_rows = 0;
    std::string created_by;
    std::vector<LeafMeta> leaves;
    std::vector<RowGroupMeta> row_groups;

    void parse_footer(const uint8_t* p, size_t n);
    static void walk_pages(const uint8_t* chunk, size_t size, const ChunkMeta& m, std::vector<pf_page_desc>& out);
};

// One page header of the write path (pf_write.cpp serialises it as a Thrift compact PageHeader).
struct PageHeaderOut {
    int32_t page_type = 0, uncompressed_size = 0, compressed_size = 0;
    int32_t num_values = 0, num_nulls = 0, num_rows = 0, encoding = 0, def_bytes = 0;
    bool is_compressed = true;
};
void write_page_header(std::vector<uint8_t>& out, const PageHeaderOut& h);

}  // namespace pf
