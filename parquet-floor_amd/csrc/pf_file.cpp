// pf_file.cpp — C ABI over the host metadata parser (pf_meta.cpp): open a file, read its
// footer (ParquetFileReader.open, ParquetReader.java:120), expose leaf columns in schema order
// (ParquetReader.java:126-128) and build pf_chunk_desc for a row group's chunks
// (readNextRowGroup, ParquetReader.java:183). No GPU calls.
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "pf_host.h"
#include "pfloor.h"

namespace {
thread_local std::string f_err;
int ferr(int code, const std::string& m) { f_err = m; return code; }
}  // namespace

struct pf_file {
    FILE* fp = nullptr;
    uint64_t size = 0;
    pf::FileMeta meta;
    std::map<std::pair<int, int>, std::vector<pf_page_desc>> pages;
};

extern "C" {

const char* pf_file_last_error(void) { return f_err.c_str(); }

int pf_file_open(const char* path, pf_file** out) {
    if (!path || !out) return ferr(PF_ERR_INVALID_ARG, "null arg");
    *out = nullptr;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return ferr(PF_ERR_IO, std::string("cannot open ") + path + ": " + std::strerror(errno));
    auto* f = new pf_file;
    f->fp = fp;
    std::fseek(fp, 0, SEEK_END);
    f->size = uint64_t(std::ftell(fp));
    try {
        if (f->size < 12) throw pf::MetaError("file too small to be parquet");
        uint8_t tail[8], head[4];
        std::fseek(fp, 0, SEEK_SET);
        if (std::fread(head, 1, 4, fp) != 4) throw pf::MetaError("read error");
        std::fseek(fp, long(f->size - 8), SEEK_SET);
        if (std::fread(tail, 1, 8, fp) != 8) throw pf::MetaError("read error");
        if (std::memcmp(head, "PAR1", 4) || std::memcmp(tail + 4, "PAR1", 4)) throw pf::MetaError("not a parquet file (magic)");
        uint32_t flen = uint32_t(tail[0]) | uint32_t(tail[1]) << 8 | uint32_t(tail[2]) << 16 | uint32_t(tail[3]) << 24;
        if (uint64_t(flen) + 12 > f->size) throw pf::MetaError("corrupt footer length");
        std::vector<uint8_t> foot(flen);
        std::fseek(fp, long(f->size - 8 - flen), SEEK_SET);
        if (flen && std::fread(foot.data(), 1, flen, fp) != flen) throw pf::MetaError("read error");
        f->meta.parse_footer(foot.data(), foot.size());
    } catch (const std::exception& e) {
        std::fclose(fp);
        delete f;
        return ferr(PF_ERR_IO, e.what());
    }
    *out = f;
    return PF_OK;
}

int pf_file_close(pf_file* f) {
    if (f) { if (f->fp) std::fclose(f->fp); delete f; }
    return PF_OK;
}

int pf_file_num_row_groups(pf_file* f, int* out) { if (!f || !out) return PF_ERR_INVALID_ARG; *out = int(f->meta.row_groups.size()); return PF_OK; }
int pf_file_num_columns(pf_file* f, int* out) { if (!f || !out) return PF_ERR_INVALID_ARG; *out = int(f->meta.leaves.size()); return PF_OK; }
int pf_file_num_rows(pf_file* f, int64_t* out) { if (!f || !out) return PF_ERR_INVALID_ARG; *out = f->meta.num_rows; return PF_OK; }
const char* pf_file_created_by(pf_file* f) { return f ? f->meta.created_by.c_str() : ""; }

int pf_file_column_meta(pf_file* f, int column, pf_column_meta* out) {
    if (!f || !out || column < 0 || column >= int(f->meta.leaves.size())) return ferr(PF_ERR_INVALID_ARG, "bad column");
    const pf::LeafMeta& L = f->meta.leaves[column];
    out->path = L.path.c_str();
    out->top_name = L.top.c_str();
    out->physical_type = L.physical_type; out->type_length = L.type_length;
    out->max_def = L.max_def; out->max_rep = L.max_rep;
    out->repeated_def = L.repeated_def; out->list_null_def = L.list_null_def;
    out->converted_type = L.converted_type; out->logical_type = L.logical_type;
    out->scale = L.scale; out->precision = L.precision;
    return PF_OK;
}

int pf_file_row_group_rows(pf_file* f, int rg, int64_t* out) {
    if (!f || !out || rg < 0 || rg >= int(f->meta.row_groups.size())) return ferr(PF_ERR_INVALID_ARG, "bad row group");
    *out = f->meta.row_groups[rg].num_rows;
    return PF_OK;
}

int pf_file_chunk_range(pf_file* f, int rg, int col, uint64_t* start, uint64_t* size) {
    if (!f || !start || !size || rg < 0 || rg >= int(f->meta.row_groups.size()) || col < 0 ||
        col >= int(f->meta.leaves.size()))
        return ferr(PF_ERR_INVALID_ARG, "bad index");
    const pf::ChunkMeta& m = f->meta.row_groups[rg].columns[col];
    if (m.num_values == 0) { *start = 0; *size = 0; return PF_OK; }
    int64_t s = m.start();
    if (s < 4 || m.total_compressed < 0 || uint64_t(s) + uint64_t(m.total_compressed) > f->size)
        return ferr(PF_ERR_IO, "column chunk outside the file");
    *start = uint64_t(s);
    *size = uint64_t(m.total_compressed);
    return PF_OK;
}

int pf_file_read(pf_file* f, uint64_t offset, uint64_t size, void* dst) {
    if (!f || (!dst && size)) return ferr(PF_ERR_INVALID_ARG, "null arg");
    if (offset + size > f->size) return ferr(PF_ERR_IO, "read past end of file");
    if (!size) return PF_OK;
    if (std::fseek(f->fp, long(offset), SEEK_SET) != 0) return ferr(PF_ERR_IO, "seek failed");
    if (std::fread(dst, 1, size, f->fp) != size) return ferr(PF_ERR_IO, "short read");
    return PF_OK;
}

int pf_file_chunk_desc(pf_file* f, int rg, int col, uint64_t chunk_offset_in_buffer, pf_chunk_desc* d) {
    if (!d) return ferr(PF_ERR_INVALID_ARG, "null desc");
    uint64_t start, size;
    int rc = pf_file_chunk_range(f, rg, col, &start, &size);
    if (rc) return rc;
    const pf::ChunkMeta& m = f->meta.row_groups[rg].columns[col];
    const pf::LeafMeta& L = f->meta.leaves[col];
    auto& pages = f->pages[{rg, col}];
    try {
        std::vector<uint8_t> buf(size);
        rc = pf_file_read(f, start, size, buf.data());
        if (rc) return rc;
        if (m.num_values > 0) pf::FileMeta::walk_pages(buf.data(), buf.size(), m, pages);
        else pages.clear();
    } catch (const std::exception& e) {
        return ferr(PF_ERR_CORRUPT_PAGE, e.what());
    }
    std::memset(d, 0, sizeof(*d));
    d->physical_type = L.physical_type;
    d->type_length = L.type_length;
    d->max_def = L.max_def;
    d->max_rep = L.max_rep;
    d->repeated_def = L.repeated_def;
    d->list_null_def = L.list_null_def;
    d->codec = m.codec;
    d->n_pages = int32_t(pages.size());
    d->pages = pages.empty() ? nullptr : pages.data();
    d->chunk_offset = chunk_offset_in_buffer;
    d->chunk_size = size;
    d->num_rows = f->meta.row_groups[rg].num_rows;
    return PF_OK;
}

}  // extern "C"
