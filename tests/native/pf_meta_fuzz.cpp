// Mutation fuzz driver for the host metadata parser (csrc/pf_meta.cpp + csrc/pf_file.cpp): the
// footer / PageHeader parse that stands in for parquet-mr's on the untrusted-input side of the
// boundary (ParquetFileReader.open + readNextRowGroup, ParquetReader.java:120, :183). Built with
// -fsanitize=address,undefined by tests/test_meta_fuzz.py; every mutated file must either parse or
// fail with a pf_status, with no sanitizer report.
//   pf_meta_fuzz SEED ITERATIONS TMPDIR FILE...
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "pfloor.h"

static std::vector<uint8_t> slurp(const char* path) {
    std::vector<uint8_t> b;
    FILE* f = std::fopen(path, "rb");
    if (!f) return b;
    std::fseek(f, 0, SEEK_END);
    b.resize(size_t(std::ftell(f)));
    std::fseek(f, 0, SEEK_SET);
    if (!b.empty() && std::fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
    std::fclose(f);
    return b;
}

// Parse everything the reader would: footer, columns, every chunk's page headers.
static int exercise(const char* path, long& ok, long& failed) {
    pf_file* f = nullptr;
    if (pf_file_open(path, &f) != PF_OK) { failed++; return 0; }
    int nrg = 0, nc = 0;
    int64_t rows = 0;
    pf_file_num_row_groups(f, &nrg);
    pf_file_num_columns(f, &nc);
    pf_file_num_rows(f, &rows);
    for (int c = 0; c < nc; c++) {
        pf_column_meta m;
        pf_file_column_meta(f, c, &m);
        if (m.path) (void)std::strlen(m.path);
    }
    for (int rg = 0; rg < nrg; rg++) {
        int64_t r = 0;
        pf_file_row_group_rows(f, rg, &r);
        for (int c = 0; c < nc; c++) {
            uint64_t s = 0, n = 0;
            if (pf_file_chunk_range(f, rg, c, &s, &n) != PF_OK) { failed++; continue; }
            pf_chunk_desc d;
            if (pf_file_chunk_desc(f, rg, c, 0, &d) != PF_OK) { failed++; continue; }
            uint64_t sum = 0;
            for (int i = 0; i < d.n_pages; i++) sum += d.pages[i].compressed_size;
            ok += sum > 0 || d.n_pages == 0;
        }
    }
    (void)pf_file_created_by(f);
    pf_file_close(f);
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 5) { std::fprintf(stderr, "usage: %s SEED ITER TMPDIR FILE...\n", argv[0]); return 2; }
    std::mt19937_64 rng(std::strtoull(argv[1], nullptr, 10));
    const long iters = std::strtol(argv[2], nullptr, 10);
    const std::string tmp = std::string(argv[3]) + "/fuzz.parquet";
    std::vector<std::vector<uint8_t>> files;
    for (int i = 4; i < argc; i++) files.push_back(slurp(argv[i]));
    long ok = 0, failed = 0, opened = 0;
    for (long it = 0; it < iters; it++) {
        std::vector<uint8_t> b = files[size_t(rng() % files.size())];
        if (b.size() < 16) continue;
        const uint32_t flen = uint32_t(b[b.size() - 8]) | uint32_t(b[b.size() - 7]) << 8 |
                              uint32_t(b[b.size() - 6]) << 16 | uint32_t(b[b.size() - 5]) << 24;
        const int nmut = 1 + int(rng() % 6);
        for (int k = 0; k < nmut; k++) {
            size_t at;
            const int where = int(rng() % 4);
            if (where == 0 && flen + 8 <= b.size()) at = b.size() - 8 - flen + size_t(rng() % flen);   // footer
            else if (where == 1) at = 4 + size_t(rng() % 4096) % (b.size() - 8);                      // first page headers
            else at = size_t(rng() % b.size());
            const int op = int(rng() % 4);
            if (op == 0) b[at] ^= uint8_t(1u << (rng() % 8));
            else if (op == 1) b[at] = uint8_t(rng());
            else if (op == 2) b[at] = uint8_t(rng() % 2 ? 0xff : 0x00);
            else if (at + 4 <= b.size()) std::memset(&b[at], 0xff, 4);
        }
        if (rng() % 16 == 0) b.resize(size_t(rng() % b.size()));   // truncation
        FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f) return 3;
        if (!b.empty()) std::fwrite(b.data(), 1, b.size(), f);
        std::fclose(f);
        opened += exercise(tmp.c_str(), ok, failed);
    }
    std::printf("iterations %ld opened %ld chunks_ok %ld failures %ld\n", iters, opened, ok, failed);
    return 0;
}
