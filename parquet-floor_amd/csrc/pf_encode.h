// pf_encode.h — device tables of the write path (pf_encode.hip <-> pf_runtime.hip). Internal.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pfloor.h"

namespace pf {

// Compression job: 8 KiB of input, compressed independently (copies never leave the job), so a
// 64 KiB Snappy block is eight jobs: 8x the waves of one wave per block (the kernel is latency-bound
// per job), for ~3 % larger output; tokens still never cross the 64 KiB output boundaries the read
// path's piece executor splits at. 64 KiB -> 16 KiB -> 8 KiB jobs: 33 -> 10 -> 6.6 ms per SF1 row group.
constexpr uint32_t SC_BLOCK = 8192;
// worst case of one compressed job (literal headers of <= 3 bytes per run): Google's bound
constexpr uint32_t SC_SLOT = ((32u + SC_BLOCK + SC_BLOCK / 6u) + 255u) & ~255u;

struct SnapCJob {
    const uint8_t* src;
    uint8_t* dst;      // SC_SLOT bytes
    uint32_t len;      // <= SC_BLOCK
    uint32_t pad;
};

struct EncPage {
    uint64_t out_off;  // values section in vals_out
    uint32_t d0, cnt;  // dense values [d0, d0 + cnt)
    uint32_t dict, bw;
};

// Every device array of one chunk's encode (one arena, laid out by the host).
struct EncArgs {
    int32_t ptype, width;
    int64_t n;                       // rows
    const uint8_t* values;           // row-indexed input
    const uint8_t* validity;         // nullptr: all present
    const int32_t* offsets;
    const uint8_t* chars;
    uint32_t* flag;                  // n + 1
    uint32_t* pos;                   // n + 1 (exclusive scan of flag)
    uint8_t* dense;                  // m x width (fixed, BOOLEAN)
    uint32_t* dsrc;                  // strings: chars offset of dense value
    uint32_t* dlen;                  // strings: length
    uint32_t* vsz;                   // strings: 4 + length (m + 1)
    uint32_t* vpre;                  // strings: exclusive scan of vsz (m + 1)
    uint64_t* key;                   // m
    uint64_t* skey;                  // m (sorted)
    uint32_t* didx;                  // m (0..m-1)
    uint32_t* sidx;                  // m (sorted)
    uint32_t* headpos;               // m
    uint32_t* head;                  // m
    uint32_t* mark;                  // m + 1
    uint32_t* did;                   // m + 1
    uint32_t* dsz;                   // m + 1
    uint32_t* doff;                  // m + 1
    uint32_t* ids;                   // m
    uint32_t* collide;               // 1
    uint8_t* dict_out;               // dictionary page (PLAIN)
    uint8_t* vals_out;               // data pages' values sections
};

hipError_t enc_scan_temp(size_t n, size_t& bytes);
hipError_t enc_dense(const EncArgs& a, void* temp, size_t temp_bytes, hipStream_t st);
hipError_t enc_plain_sizes(const EncArgs& a, uint32_t m, void* temp, size_t temp_bytes, hipStream_t st);
hipError_t enc_dictionary(const EncArgs& a, uint32_t m, int key_bits, void* temp, size_t temp_bytes, hipStream_t st);
void enc_dictionary_page_and_ids(const EncArgs& a, uint32_t m, hipStream_t st);
void enc_pages(const EncArgs& a, const EncPage* d_pages, int n_pages, hipStream_t st);
void launch_snappy_compress(const SnapCJob* d_jobs, int n_jobs, uint32_t* d_out_len, hipStream_t st);

}  // namespace pf
