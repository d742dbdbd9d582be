// pf_scan.hip — GPU page-header scan and page CRC32 verification.
//
// Replaces the per-page Thrift walk parquet-mr does inside ParquetFileReader.readNextRowGroup
// (called at src/main/java/blue/strategic/parquet/ParquetReader.java:183): Chunk.readAllPages reads
// PageHeaders back to back until the chunk's ColumnMetaData.num_values level entries have been seen,
// skipping INDEX and unknown page types; with page checksum verification on
// (ParquetReadOptions.usePageChecksumVerification) every page carrying PageHeader.crc (field 4) is
// checked against the CRC32 of its on-disk page bytes. The host walk this mirrors field by field is
// pf_meta.cpp FileMeta::walk_pages (same results, same errors).
//
//   k_page_scan  one wave per column chunk. Headers are staged 512 bytes at a time into LDS with
//                aligned dword loads; the Thrift compact reader runs uniformly on all lanes (every
//                lane parses the same bytes, so restaging mid-header is a uniform step). Nested
//                structs / lists / maps the reader does not need are skipped with a bounded explicit
//                stack (no recursion).
//   k_page_crc   one 256-thread workgroup per page: each thread takes a contiguous segment, computes
//                its raw CRC (zero init, table in LDS), shifts it to its place in the page
//                (multiplication by x^(8 * bytes after it) mod P, square-and-multiply over a table of
//                x^(2^k)), and the XOR over the workgroup plus the init / final-xor terms is the
//                page's standard CRC32 (zlib / java.util.zip.CRC32).
#include <hip/hip_runtime.h>

#include "pf_device.h"
#include "pf_internal.h"
#include "pfloor.h"

namespace pf {

constexpr uint32_t SCAN_STG = 512;     // staged header bytes
constexpr uint32_t SCAN_MARGIN = 16;   // restage when fewer staged bytes remain ahead (a varint is <= 10)
constexpr int SKIP_DEPTH = 16;

struct ThriftDev {
    uint8_t* stg;             // LDS
    const uint8_t* base;      // chunk start
    uint64_t size;            // chunk size
    uint64_t sbase;           // chunk offset of stg[0]
    uint64_t pos;             // chunk offset of the next byte
    bool err;

    __device__ void stage(uint64_t at) {
        __syncthreads();
        const int lane = threadIdx.x & 63;
        const uintptr_t b = reinterpret_cast<uintptr_t>(base);
        const uintptr_t lastw = (b + size - 1) & ~uintptr_t(3);
        for (uint32_t i = uint32_t(lane); i < SCAN_STG / 4; i += 64) {
            const uintptr_t a = b + at + 4 * i;
            const uintptr_t a0 = a & ~uintptr_t(3);
            const uint32_t lo = a0 <= lastw ? *(const PF_GLOBAL uint32_t*)a0 : 0u;
            const uint32_t hi = a0 + 4 <= lastw ? *(const PF_GLOBAL uint32_t*)(a0 + 4) : 0u;
            reinterpret_cast<uint32_t*>(stg)[i] = __builtin_amdgcn_alignbyte(hi, lo, uint32_t(a & 3u));
        }
        sbase = at;
        __syncthreads();
    }
    __device__ uint32_t byte() {
        if (pos >= size) { err = true; return 0; }
        if (pos - sbase >= SCAN_STG - SCAN_MARGIN) stage(pos);
        return stg[pos++ - sbase];
    }
    __device__ uint64_t uvarint() {
        uint64_t v = 0;
        for (int sh = 0; sh < 64 && !err; sh += 7) {
            const uint32_t c = byte();
            v |= uint64_t(c & 0x7f) << sh;
            if (!(c & 0x80)) return v;
        }
        err = true;
        return 0;
    }
    __device__ int64_t zigzag() { const uint64_t u = uvarint(); return int64_t(u >> 1) ^ -int64_t(u & 1); }
    // Field header: returns the field id (0 = stop); type in t.
    __device__ int field(int& last, int& t) {
        const uint32_t b = byte();
        if (err || b == 0) return 0;
        t = int(b & 0xf);
        const int d = int(b >> 4);
        last = d ? last + d : int(int16_t(zigzag()));
        return last;
    }
    __device__ int64_t integer(int t) {
        if (t == 3) return int64_t(int8_t(byte()));
        if (t == 4 || t == 5 || t == 6) return zigzag();
        err = true;
        return 0;
    }
    __device__ bool boolean(int t) { if (t == 1) return true; if (t == 2) return false; err = true; return false; }
    __device__ void advance(uint64_t n) {
        if (n > size - pos || pos > size) { err = true; pos = size; return; }
        pos += n;
    }
    // Skip a value of type t (containers with an explicit stack).
    __device__ void skip(int t) {
        struct Frame { int kind; uint64_t left; int et, vt, last; };   // kind 0 struct, 1 list/set, 2 map
        Frame st[SKIP_DEPTH];
        int sp = 0;
        int cur = t;
        for (;;) {
            if (err) return;
            bool push = false;
            switch (cur) {
            case 1: case 2: break;
            case 3: byte(); break;
            case 4: case 5: case 6: uvarint(); break;
            case 7: advance(8); break;
            case 8: advance(uvarint()); break;
            case 9: case 10: {
                const uint32_t h = byte();
                uint64_t n = h >> 4;
                if (n == 15) n = uvarint();
                st[sp] = Frame{1, n, int(h & 0xf), 0, 0};
                push = true;
                break;
            }
            case 11: {
                const uint64_t n = uvarint();
                const uint32_t kv = n ? byte() : 0u;
                st[sp] = Frame{2, 2 * n, int(kv >> 4), int(kv & 0xf), 0};
                push = true;
                break;
            }
            case 12: st[sp] = Frame{0, 0, 0, 0, 0}; push = true; break;
            default: err = true; return;
            }
            if (push && ++sp > SKIP_DEPTH - 1) { err = true; return; }
            // next value to skip: from the innermost open container
            for (;;) {
                if (sp == 0) return;
                Frame& f = st[sp - 1];
                if (f.kind == 0) {
                    int ft = 0;
                    if (field(f.last, ft) == 0) { sp--; if (err) return; continue; }
                    cur = ft;
                } else if (f.left == 0) {
                    sp--;
                    continue;
                } else {
                    const uint64_t k = f.left--;
                    cur = f.kind == 1 ? f.et : ((k & 1) == 0 ? f.et : f.vt);
                    if (f.kind == 1 && (cur == 1 || cur == 2)) { byte(); continue; }   // list bools are one byte
                }
                break;
            }
        }
    }
};

// One wave per chunk: PageHeaders until num_values level entries are seen (pf_meta.cpp walk_pages).
__global__ __launch_bounds__(64) void k_page_scan(const ScanChunk* __restrict__ chunks, pf_page_desc* __restrict__ pages,
                                                  ScanCrc* __restrict__ crcs, ScanResult* __restrict__ res) {
    __shared__ __attribute__((aligned(16))) uint8_t stg[SCAN_STG];
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    const ScanChunk ck = chunks[c];
    ThriftDev r{stg, ck.base, ck.size, 0, 0, false};
    int32_t np = 0, status = PF_OK, err_page = -1;
    int64_t seen = 0;
    uint64_t off = 0;
    bool have_dict = false;
    if (ck.num_values > 0 && ck.size > 0) r.stage(0);
    while (seen < ck.num_values) {
        if (off >= ck.size) { status = PF_ERR_CORRUPT_PAGE; err_page = np; break; }
        r.pos = off;
        if (off < r.sbase || off - r.sbase >= SCAN_STG - SCAN_MARGIN) r.stage(off);
        pf_page_desc d{};
        d.is_compressed = 1;
        d.num_nulls = -1;
        d.page_type = -1;
        uint32_t crc = 0;
        int has_crc = 0;
        int last = 0, t = 0, id;
        while ((id = r.field(last, t)) != 0) {
            if (id == 1) d.page_type = int32_t(r.integer(t));
            else if (id == 2) d.uncompressed_size = uint32_t(r.integer(t));
            else if (id == 3) d.compressed_size = uint32_t(r.integer(t));
            else if (id == 4 && t == 5) { crc = uint32_t(r.integer(t)); has_crc = 1; }
            else if ((id == 5 || id == 7 || id == 8) && t == 12) {
                int l2 = 0, t2 = 0, i2;
                while ((i2 = r.field(l2, t2)) != 0) {
                    if (id == 5) {
                        if (i2 == 1) d.num_values = int32_t(r.integer(t2));
                        else if (i2 == 2) d.encoding = int32_t(r.integer(t2));
                        else if (i2 == 3) d.def_encoding = int32_t(r.integer(t2));
                        else if (i2 == 4) d.rep_encoding = int32_t(r.integer(t2));
                        else if (i2 == 5 && t2 == 12) {   // Statistics.null_count: a routing hint
                            int l3 = 0, t3 = 0, i3;
                            while ((i3 = r.field(l3, t3)) != 0) {
                                if (i3 == 3) {
                                    const int64_t nn = r.integer(t3);
                                    d.num_nulls = nn >= 0 && nn <= 0x7fffffff ? int32_t(nn) : -1;
                                } else r.skip(t3);
                                if (r.err) break;
                            }
                        } else r.skip(t2);
                    } else if (id == 7) {
                        if (i2 == 1) d.num_values = int32_t(r.integer(t2));
                        else if (i2 == 2) d.encoding = int32_t(r.integer(t2));
                        else r.skip(t2);
                    } else {
                        if (i2 == 1) d.num_values = int32_t(r.integer(t2));
                        else if (i2 == 2) d.num_nulls = int32_t(r.integer(t2));
                        else if (i2 == 3) d.num_rows = int32_t(r.integer(t2));
                        else if (i2 == 4) d.encoding = int32_t(r.integer(t2));
                        else if (i2 == 5) d.def_bytes = int32_t(r.integer(t2));
                        else if (i2 == 6) d.rep_bytes = int32_t(r.integer(t2));
                        else if (i2 == 7) d.is_compressed = r.boolean(t2) ? 1 : 0;
                        else r.skip(t2);
                    }
                    if (r.err) break;
                }
            } else r.skip(t);
            if (r.err) break;
        }
        if (r.err) { status = PF_ERR_CORRUPT_PAGE; err_page = np; break; }
        const uint64_t body = r.pos;
        if (int32_t(d.compressed_size) < 0 || body + d.compressed_size > ck.size) { status = PF_ERR_CORRUPT_PAGE; err_page = np; break; }
        d.offset = body;
        off = body + d.compressed_size;
        bool keep = false;
        if (d.page_type == PF_PAGE_DICTIONARY) {
            if (have_dict || np > 0) { status = PF_ERR_CORRUPT_PAGE; err_page = np; break; }
            have_dict = true;
            keep = true;
        } else if (d.page_type == PF_PAGE_DATA || d.page_type == PF_PAGE_DATA_V2) {
            if (d.num_values < 0 ||
                (d.page_type == PF_PAGE_DATA_V2 &&
                 (d.def_bytes < 0 || d.rep_bytes < 0 ||
                  uint64_t(d.def_bytes) + uint64_t(d.rep_bytes) > d.compressed_size ||
                  uint64_t(d.def_bytes) + uint64_t(d.rep_bytes) > d.uncompressed_size))) {
                status = PF_ERR_CORRUPT_PAGE; err_page = np; break;
            }
            keep = true;
            seen += d.num_values;
        }
        if (keep) {
            if (np >= ck.page_cap) { status = PF_ERR_CAPACITY; err_page = np; break; }
            if (lane == 0) {
                pages[ck.page_base + np] = d;
                crcs[ck.page_base + np] = ScanCrc{ck.base + body, d.compressed_size, crc, has_crc, c};
            }
            np++;
        }
        if (off >= ck.size && seen < ck.num_values) { status = PF_ERR_CORRUPT_PAGE; err_page = np; break; }
    }
    if (lane == 0) res[c] = ScanResult{np, status, err_page, 0};
}

// ---- CRC32 (reflected polynomial 0xEDB88320, as zlib / java.util.zip.CRC32)
constexpr uint32_t CRC_POLY = 0xedb88320u;

// a * b mod P in the reflected representation (x^0 = bit 31).
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
    }
    return p;
}

// x^(8n) mod P from x2n[k] = x^(2^k) mod P.
__device__ uint32_t crc_x8n(uint64_t n, const uint32_t* x2n) {
    uint32_t p = 1u << 31;
    unsigned k = 3;
    while (n) {
        if (n & 1) p = crc_mulmod(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

constexpr int CRC_NT = 256;

__global__ __launch_bounds__(CRC_NT) void k_page_crc(const ScanCrc* __restrict__ crcs, const int* __restrict__ list,
                                                     ScanResult* __restrict__ res, int32_t* __restrict__ bad) {
    __shared__ uint32_t table[256];
    __shared__ uint32_t x2n[32];
    __shared__ uint32_t red[CRC_NT / 64];
    const int slot = list[blockIdx.x];
    const ScanCrc pc = crcs[slot];
    const int tid = threadIdx.x;
    if (!pc.has_crc) return;   // no PageHeader.crc: nothing to verify (parquet-mr skips the check)
    {
        uint32_t c = uint32_t(tid);
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ CRC_POLY : c >> 1;
        table[tid] = c;
    }
    if (tid == 0) {
        uint32_t p = 1u << 30;   // x^1
        x2n[0] = p;
        for (int k = 1; k < 32; k++) x2n[k] = p = crc_mulmod(p, p);
    }
    __syncthreads();
    const uint32_t len = pc.len;
    const uint32_t seg = (len + CRC_NT - 1) / CRC_NT;
    const uint32_t b0 = min(len, uint32_t(tid) * seg), b1 = min(len, b0 + seg);
    const PF_GLOBAL uint8_t* g = gptr(pc.body);
    uint32_t c = 0;   // raw CRC (zero init, no final xor): linear in the data
    for (uint32_t i = b0; i < b1; i++) c = table[(c ^ g[i]) & 0xffu] ^ (c >> 8);
    uint32_t part = b1 > b0 ? crc_mulmod(crc_x8n(len - b1, x2n), c) : 0u;
    #pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part ^= uint32_t(__shfl_xor(part, d, 64));
    if ((tid & 63) == 0) red[tid >> 6] = part;
    __syncthreads();
    if (tid == 0) {
        uint32_t raw = 0;
        for (int w = 0; w < CRC_NT / 64; w++) raw ^= red[w];
        // standard CRC32 = raw(data, init ~0) ^ ~0 = raw(data, 0) ^ (~0 * x^(8 len)) ^ ~0
        const uint32_t crc = raw ^ crc_mulmod(crc_x8n(len, x2n), 0xffffffffu) ^ 0xffffffffu;
        atomicAdd(&res[pc.chunk].crc_pages, 1);
        if (crc != pc.crc) atomicMin(&bad[pc.chunk], slot);
    }
}

void launch_page_scan(const ScanChunk* d_chunks, int n_chunks, pf_page_desc* d_pages, ScanCrc* d_crcs, ScanResult* d_res,
                      hipStream_t s) {
    if (n_chunks > 0) hipLaunchKernelGGL(k_page_scan, dim3(n_chunks), dim3(64), 0, s, d_chunks, d_pages, d_crcs, d_res);
}

void launch_page_crc(const ScanCrc* d_crcs, const int* d_list, int n, ScanResult* d_res, int32_t* d_bad, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_page_crc, dim3(n), dim3(CRC_NT), 0, s, d_crcs, d_list, d_res, d_bad);
}

}  // namespace pf
