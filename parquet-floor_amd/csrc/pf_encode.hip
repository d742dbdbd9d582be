// pf_encode.hip — write path kernels: the column encoding parquet-mr performs
// inside the reference's ParquetWriter (src/main/java/blue/strategic/parquet/ParquetWriter.java:61-68:
// SNAPPY, WriterVersion.PARQUET_2_0), on gfx950.
//
//   present rows -> dense values (exclusive scan of the validity flags)
//   dictionary   -> radix sort of (value key, dense index); segment heads; first occurrence of
//                   every distinct value marked; an exclusive scan of the marks numbers the
//                   dictionary in first-occurrence order — the order parquet-mr's
//                   DictionaryValuesWriter assigns ids (a hash map that appends new values)
//   data pages   -> values section per page: bit width byte + one bit-packed run of the ids
//                   (RLE_DICTIONARY), or PLAIN; definition levels (v2 pages, bit width 1) are the
//                   validity bits themselves, written by the host
//   Snappy       -> k_snappy_compress: one wave per 8 KiB job (hash table of 4-byte
//                   prefixes in LDS, 64 candidate positions per step, wave-parallel match
//                   extension); jobs are independent, so a page's stream is the varint length
//                   followed by its jobs' outputs; no token crosses a 64 KiB output boundary,
//                   the layout Google's compressor produces and the read path's executor uses.
// Byte/integer work throughout (HBM-bound; no MFMA).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "pf_encode.h"

namespace pf {

namespace {
constexpr int ENT = 256;

__device__ __forceinline__ uint64_t hash_bytes(const uint8_t* p, uint32_t n) {
    // FNV-1a over the bytes, then a 64-bit finaliser (collisions are detected, never trusted)
    uint64_t h = 0xcbf29ce484222325ull ^ n;
    for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
    return h;
}
}  // namespace

// flag[r] = row r present (flag[n] = 0 so the exclusive scan's last element is the count)
__global__ __launch_bounds__(ENT) void k_enc_flags(const uint8_t* __restrict__ validity, int64_t n, uint32_t* __restrict__ flag) {
    for (int64_t r = int64_t(blockIdx.x) * ENT + threadIdx.x; r <= n; r += int64_t(gridDim.x) * ENT)
        flag[r] = r == n ? 0u : (validity ? (validity[r >> 3] >> (r & 7)) & 1u : 1u);
}

// dense value d = the d-th present row: keys (fixed: value bits; strings: hash), dense index,
// string lengths / positions, PLAIN byte sizes (for the page plan)
__global__ __launch_bounds__(ENT) void k_enc_compact(EncArgs a) {
    for (int64_t r = int64_t(blockIdx.x) * ENT + threadIdx.x; r < a.n; r += int64_t(gridDim.x) * ENT) {
        if (a.flag[r] == 0) continue;
        const uint32_t d = a.pos[r];
        a.didx[d] = d;
        if (a.ptype == PF_BYTE_ARRAY) {
            const int32_t s = a.offsets[r], e = a.offsets[r + 1];
            const uint32_t len = e > s ? uint32_t(e - s) : 0u;
            a.dsrc[d] = uint32_t(s);
            a.dlen[d] = len;
            a.vsz[d] = 4u + len;
            a.key[d] = hash_bytes(a.chars + s, len);
        } else if (a.width == 8) {
            const uint64_t v = reinterpret_cast<const uint64_t*>(a.values)[r];
            reinterpret_cast<uint64_t*>(a.dense)[d] = v;
            a.key[d] = v;
        } else if (a.width == 4) {
            const uint32_t v = reinterpret_cast<const uint32_t*>(a.values)[r];
            reinterpret_cast<uint32_t*>(a.dense)[d] = v;
            a.key[d] = v;
        } else {   // BOOLEAN: one byte per row
            a.dense[d] = a.values[r] ? 1 : 0;
        }
    }
}

// Over the sorted (key, dense index) pairs: headpos[i] = i at a segment head (first of a run of
// equal keys; stable sort => its dense index is the value's first occurrence), else 0. Strings
// whose hashes are equal but bytes differ raise the collision flag (the chunk is then PLAIN).
__global__ __launch_bounds__(ENT) void k_enc_heads(EncArgs a, uint32_t m) {
    for (uint32_t i = blockIdx.x * ENT + threadIdx.x; i < m; i += gridDim.x * ENT) {
        const bool head = i == 0 || a.skey[i] != a.skey[i - 1];
        a.headpos[i] = head ? i : 0u;
        if (!head && a.ptype == PF_BYTE_ARRAY) {
            const uint32_t p = a.sidx[i], q = a.sidx[i - 1];
            bool same = a.dlen[p] == a.dlen[q];
            for (uint32_t k = 0; same && k < a.dlen[p]; k++) same = a.chars[a.dsrc[p] + k] == a.chars[a.dsrc[q] + k];
            if (!same) atomicOr(a.collide, 1u);
        }
    }
}

// mark[d] = dense value d is the first occurrence of its value; dict byte size per entry
__global__ __launch_bounds__(ENT) void k_enc_mark(EncArgs a, uint32_t m) {
    for (uint32_t i = blockIdx.x * ENT + threadIdx.x; i <= m; i += gridDim.x * ENT) {
        if (i == m) { a.mark[m] = 0; a.dsz[m] = 0; continue; }
        const uint32_t d = a.sidx[i];
        const uint32_t first = a.head[i] == i;
        a.mark[d] = first;
        a.dsz[d] = first ? (a.ptype == PF_BYTE_ARRAY ? 4u + a.dlen[d] : uint32_t(a.width)) : 0u;
    }
}

// ids[d] = dictionary id of dense value d; the dictionary page (PLAIN, first-occurrence order)
__global__ __launch_bounds__(ENT) void k_enc_ids(EncArgs a, uint32_t m) {
    for (uint32_t i = blockIdx.x * ENT + threadIdx.x; i < m; i += gridDim.x * ENT) {
        const uint32_t d = a.sidx[i];
        const uint32_t f = a.sidx[a.head[i]];
        const uint32_t id = a.did[f];
        a.ids[d] = id;
        if (f != d) continue;   // the first occurrence writes the dictionary entry
        uint8_t* o = a.dict_out + a.doff[d];
        if (a.ptype == PF_BYTE_ARRAY) {
            const uint32_t len = a.dlen[d];
            o[0] = uint8_t(len); o[1] = uint8_t(len >> 8); o[2] = uint8_t(len >> 16); o[3] = uint8_t(len >> 24);
            const uint8_t* s = a.chars + a.dsrc[d];
            for (uint32_t k = 0; k < len; k++) o[4 + k] = s[k];
        } else {
            const uint8_t* s = a.dense + uint64_t(d) * uint32_t(a.width);
            for (int k = 0; k < a.width; k++) o[k] = s[k];
        }
    }
}

// Values section of every data page: one workgroup per page (EncPage from the host plan).
__global__ __launch_bounds__(ENT) void k_enc_pages(EncArgs a, const EncPage* __restrict__ pages) {
    const EncPage pg = pages[blockIdx.x];
    const int tid = threadIdx.x;
    uint8_t* o = a.vals_out + pg.out_off;
    const uint32_t d0 = pg.d0, cnt = pg.cnt;
    if (pg.dict) {
        // bit width byte, then one bit-packed run: varint((groups << 1) | 1), groups of 8 ids
        const uint32_t bw = pg.bw;
        const uint32_t groups = (cnt + 7) / 8;
        uint32_t hdr = 1;
        if (tid == 0) {
            o[0] = uint8_t(bw);
            if (cnt) {
                uint32_t v = (groups << 1) | 1u;
                while (v >= 0x80) { o[hdr++] = uint8_t(v | 0x80); v >>= 7; }
                o[hdr++] = uint8_t(v);
            }
        }
        if (!cnt) return;
        hdr = 1;
        for (uint32_t v = (groups << 1) | 1u; v >= 0x80; v >>= 7) hdr++;
        hdr++;
        for (uint32_t g = tid; g < groups; g += ENT) {
            uint64_t w[5] = {0, 0, 0, 0, 0};   // 8 ids x <= 32 bits
            #pragma unroll
            for (uint32_t k = 0; k < 8; k++) {
                const uint32_t e = g * 8 + k;
                const uint64_t id = e < cnt ? a.ids[d0 + e] : 0u;
                const uint32_t bit = k * bw;
                w[bit >> 6] |= id << (bit & 63);
                if ((bit & 63) + bw > 64) w[(bit >> 6) + 1] |= id >> (64 - (bit & 63));
            }
            uint8_t* q = o + hdr + uint64_t(g) * bw;
            for (uint32_t b = 0; b < bw; b++) q[b] = uint8_t(w[b >> 3] >> (8 * (b & 7)));
        }
        return;
    }
    if (a.ptype == PF_BYTE_ARRAY) {   // PLAIN: 4-byte LE length + bytes
        const uint32_t base = a.vpre[d0];
        for (uint32_t e = tid; e < cnt; e += ENT) {
            const uint32_t d = d0 + e;
            uint8_t* q = o + (a.vpre[d] - base);
            const uint32_t len = a.dlen[d];
            q[0] = uint8_t(len); q[1] = uint8_t(len >> 8); q[2] = uint8_t(len >> 16); q[3] = uint8_t(len >> 24);
            const uint8_t* s = a.chars + a.dsrc[d];
            for (uint32_t k = 0; k < len; k++) q[4 + k] = s[k];
        }
    } else if (a.ptype == PF_BOOLEAN) {   // PLAIN: bit-packed LSB-first
        for (uint32_t b = tid; b < (cnt + 7) / 8; b += ENT) {
            uint32_t v = 0;
            for (uint32_t k = 0; k < 8; k++)
                if (b * 8 + k < cnt) v |= uint32_t(a.dense[d0 + b * 8 + k] & 1u) << k;
            o[b] = uint8_t(v);
        }
    } else {   // PLAIN fixed width: dense copy
        const uint64_t nb = uint64_t(cnt) * uint32_t(a.width);
        const uint8_t* s = a.dense + uint64_t(d0) * uint32_t(a.width);
        for (uint64_t k = tid; k < nb; k += ENT) o[k] = s[k];
    }
}

// ---------------------------------------------------------------- Snappy compression
// One wave per job of <= 8 KiB (SC_BLOCK): the job is staged in LDS with a 4096-entry table of the last
// position (+1) of each 4-byte prefix hash. Each step the 64 lanes look up positions ip..ip+63
// against the table as it stood before the step (so candidates always precede them); the first
// lane whose candidate matches starts a copy: literal [lit, q), match extended 64 bytes per
// ballot, emitted as copies of <= 64 bytes (copy-1 for 4..11 bytes at offsets < 2048, else
// copy-2); further matching lanes after that copy's end become tokens in the same step. No match
// in the step: its 64 positions are hashed in and the wave moves on.
namespace {
constexpr uint32_t SC_HBITS = 12;
__device__ __forceinline__ uint32_t sc_hash(uint32_t v) { return (v * 0x1e35a7bdu) >> (32 - SC_HBITS); }
__device__ __forceinline__ uint32_t sc_ld32(const uint8_t* b, uint32_t p) {
    return uint32_t(b[p]) | uint32_t(b[p + 1]) << 8 | uint32_t(b[p + 2]) << 16 | uint32_t(b[p + 3]) << 24;
}
__device__ __forceinline__ uint32_t sc_literal(uint8_t* dst, uint32_t op, const uint8_t* buf, uint32_t s, uint32_t n) {
    const int lane = threadIdx.x;
    const uint32_t l = n - 1;
    uint32_t h;
    if (l < 60) { if (lane == 0) dst[op] = uint8_t(l << 2); h = 1; }
    else if (l < 256) { if (lane == 0) { dst[op] = uint8_t(60 << 2); dst[op + 1] = uint8_t(l); } h = 2; }
    else { if (lane == 0) { dst[op] = uint8_t(61 << 2); dst[op + 1] = uint8_t(l); dst[op + 2] = uint8_t(l >> 8); } h = 3; }
    for (uint32_t j = lane; j < n; j += 64) dst[op + h + j] = buf[s + j];
    return op + h + n;
}
__device__ __forceinline__ uint32_t sc_copy(uint8_t* dst, uint32_t op, uint32_t off, uint32_t len) {
    if (len <= 11 && off < 2048) {
        if (threadIdx.x == 0) { dst[op] = uint8_t(1 | ((len - 4) << 2) | ((off >> 8) << 5)); dst[op + 1] = uint8_t(off); }
        return op + 2;
    }
    if (threadIdx.x == 0) { dst[op] = uint8_t(2 | ((len - 1) << 2)); dst[op + 1] = uint8_t(off); dst[op + 2] = uint8_t(off >> 8); }
    return op + 3;
}
}  // namespace

__global__ __launch_bounds__(64) void k_snappy_compress(const SnapCJob* __restrict__ jobs, uint32_t* __restrict__ out_len) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[SC_BLOCK + 16];
    __shared__ uint16_t tab[1u << SC_HBITS];
    const SnapCJob job = jobs[blockIdx.x];
    const int lane = threadIdx.x;
    const uint32_t len = job.len;
    for (uint32_t i = lane; i < len + 16; i += 64) buf[i] = i < len ? job.src[i] : 0;
    for (uint32_t i = lane; i < (1u << SC_HBITS); i += 64) tab[i] = 0;
    __syncthreads();
    uint8_t* dst = job.dst;
    uint32_t ip = 0, lit = 0, op = 0;
    while (ip + 4 <= len) {
        const uint32_t q = ip + uint32_t(lane);
        const bool valid = q + 4 <= len;
        const uint32_t v = valid ? sc_ld32(buf, q) : 0u;
        const uint32_t h = sc_hash(v);
        const uint32_t c = valid ? uint32_t(tab[h]) : 0u;
        const bool m = valid && c != 0 && sc_ld32(buf, c - 1) == v;
        const unsigned long long mask = __ballot(m);
        if (!mask) {
            if (valid) tab[h] = uint16_t(q + 1);
            ip += 64;
            continue;
        }
        // every match of this window, greedily: after a copy ending at e, the next token is the
        // first lane at or after e whose candidate matched (candidates all precede ip, so each is
        // valid); the lanes in between join the literal
        unsigned long long mk = mask;
        uint32_t e = ip;
        while (mk) {
            const uint32_t f = uint32_t(__ffsll(mk) - 1);
            const uint32_t qf = ip + f;
            const uint32_t cand = uint32_t(__builtin_amdgcn_readlane(int(c), int(f))) - 1u;
            uint32_t L = 4;
            for (;;) {   // extend the match 64 bytes per step
                const uint32_t x = qf + L + uint32_t(lane), y = cand + L + uint32_t(lane);
                const bool eq = x < len && buf[x] == buf[y];
                const unsigned long long ne = __ballot(!eq);
                if (!ne) { L += 64; continue; }
                L += uint32_t(__ffsll(ne) - 1);
                break;
            }
            if (qf > lit) op = sc_literal(dst, op, buf, lit, qf - lit);
            const uint32_t off = qf - cand;
            uint32_t rem = L;
            while (rem >= 68) { op = sc_copy(dst, op, off, 64); rem -= 64; }
            if (rem > 64) { op = sc_copy(dst, op, off, 60); rem -= 60; }
            op = sc_copy(dst, op, off, rem);
            e = qf + L;
            lit = e;
            mk = e - ip >= 64 ? 0ull : (mk & ~((1ull << (e - ip)) - 1ull));
        }
        if (valid && q < e) tab[h] = uint16_t(q + 1);   // positions passed by this window's tokens
        ip = e;   // lanes after the last copy had no match: rescanned with the table updated
    }
    if (len > lit) op = sc_literal(dst, op, buf, lit, len - lit);
    if (lane == 0) out_len[blockIdx.x] = op;
}

// ---------------------------------------------------------------- launchers
namespace {
inline unsigned grid_for(int64_t n) {
    const int64_t g = (n + ENT - 1) / ENT;
    return unsigned(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}
}  // namespace

hipError_t enc_scan_temp(size_t n, size_t& bytes) {
    bytes = 0;
    size_t b1 = 0, b2 = 0, b3 = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, b1, static_cast<uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr), int(n));
    if (e != hipSuccess) return e;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, b2, static_cast<const uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                                           static_cast<const uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr), int(n));
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::InclusiveScan(nullptr, b3, static_cast<uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr),
                                          hipcub::Max(), int(n));
    bytes = std::max(b1, std::max(b2, b3));
    return e;
}

// Dense stage: flags -> scan -> compaction (+ PLAIN size prefix for strings).
hipError_t enc_dense(const EncArgs& a, void* temp, size_t temp_bytes, hipStream_t st) {
    hipLaunchKernelGGL(k_enc_flags, dim3(grid_for(a.n + 1)), dim3(ENT), 0, st, a.validity, a.n, a.flag);
    size_t tb = temp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp, tb, a.flag, a.pos, int(a.n + 1), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_enc_compact, dim3(grid_for(a.n)), dim3(ENT), 0, st, a);
    return hipGetLastError();
}

// PLAIN string sizes: vpre = exclusive scan of vsz over m + 1 (vsz[m] = 0 set by the host).
hipError_t enc_plain_sizes(const EncArgs& a, uint32_t m, void* temp, size_t temp_bytes, hipStream_t st) {
    size_t tb = temp_bytes;
    return hipcub::DeviceScan::ExclusiveSum(temp, tb, a.vsz, a.vpre, int(m + 1), st);
}

// Dictionary stage over m dense values; key_bits = 32 for 4-byte types (radix passes halved).
hipError_t enc_dictionary(const EncArgs& a, uint32_t m, int key_bits, void* temp, size_t temp_bytes, hipStream_t st) {
    size_t tb = temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, tb, a.key, a.skey, a.didx, a.sidx, int(m), 0, key_bits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_enc_heads, dim3(grid_for(m)), dim3(ENT), 0, st, a, m);
    tb = temp_bytes;
    e = hipcub::DeviceScan::InclusiveScan(temp, tb, a.headpos, a.head, hipcub::Max(), int(m), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_enc_mark, dim3(grid_for(m + 1)), dim3(ENT), 0, st, a, m);
    tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(temp, tb, a.mark, a.did, int(m + 1), st);
    if (e != hipSuccess) return e;
    tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(temp, tb, a.dsz, a.doff, int(m + 1), st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

void enc_dictionary_page_and_ids(const EncArgs& a, uint32_t m, hipStream_t st) {
    if (m) hipLaunchKernelGGL(k_enc_ids, dim3(grid_for(m)), dim3(ENT), 0, st, a, m);
}

void enc_pages(const EncArgs& a, const EncPage* d_pages, int n_pages, hipStream_t st) {
    if (n_pages > 0) hipLaunchKernelGGL(k_enc_pages, dim3(n_pages), dim3(ENT), 0, st, a, d_pages);
}

void launch_snappy_compress(const SnapCJob* d_jobs, int n_jobs, uint32_t* d_out_len, hipStream_t st) {
    if (n_jobs > 0) hipLaunchKernelGGL(k_snappy_compress, dim3(n_jobs), dim3(64), 0, st, d_jobs, d_out_len);
}

}  // namespace pf
