// pf_device.h — device helpers shared by the decode kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pf_internal.h"

namespace pf {

constexpr int WAVE = 64;

// Global-memory view of a pointer loaded from a descriptor: without it the loads/stores are flat_*,
// which count against lgkmcnt as well and make the compiler drain vmcnt before LDS accesses.
#define PF_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ PF_GLOBAL T* gptr(T* p) { return (PF_GLOBAL T*)(p); }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // 16-byte access (POD, any address space)


// Status codes (pfloor.h pf_status); kept as constants so device code needs no header.
enum : int32_t {
    ST_OK = 0, ST_CORRUPT = -2, ST_ENCODING = -3, ST_CODEC = -4, ST_CAPACITY = -6, ST_TYPE = -7
};

__device__ __forceinline__ void set_status(DevChunkResult* res, int chunk, int32_t code, int page) {
    // the most negative code wins; any error is sticky
    int32_t prev = atomicMin(&res[chunk].status, code);
    if (code < prev) res[chunk].err_page = page;
}

// Bounds-checked byte read (bytes past `n` read as 0; callers validate lengths separately).
__device__ __forceinline__ uint32_t ld8(const uint8_t* p, uint64_t i, uint64_t n) {
    return i < n ? uint32_t(p[i]) : 0u;
}

__device__ __forceinline__ uint32_t ld32le(const uint8_t* p, uint64_t i, uint64_t n) {
    if (i + 4 <= n) {
        return uint32_t(p[i]) | uint32_t(p[i + 1]) << 8 | uint32_t(p[i + 2]) << 16 | uint32_t(p[i + 3]) << 24;
    }
    return ld8(p, i, n) | ld8(p, i + 1, n) << 8 | ld8(p, i + 2, n) << 16 | ld8(p, i + 3, n) << 24;
}

// Unsigned LEB128 varint; false on overrun / >10 bytes.
__device__ __forceinline__ bool uvarint(const uint8_t* p, uint64_t n, uint64_t& pos, uint64_t& v) {
    v = 0;
    for (int sh = 0; sh < 70; sh += 7) {
        if (pos >= n) return false;
        uint32_t c = p[pos++];
        v |= uint64_t(c & 0x7f) << sh;
        if (!(c & 0x80)) return true;
    }
    return false;
}

__device__ __forceinline__ int64_t unzigzag(uint64_t v) { return int64_t(v >> 1) ^ -int64_t(v & 1); }

// Little-endian (LSB-first) bit field of width w <= 32 at bit offset `bit` of p[0..n).
__device__ __forceinline__ uint32_t bits_le(const uint8_t* p, uint64_t n, uint64_t bit, int w) {
    if (w == 0) return 0;
    uint64_t by = bit >> 3;
    int sh = int(bit & 7);
    uint64_t acc = 0;
    int need = (sh + w + 7) >> 3;   // <= 5 bytes
    #pragma unroll
    for (int k = 0; k < 5; k++)
        if (k < need) acc |= uint64_t(ld8(p, by + k, n)) << (8 * k);
    uint64_t m = (w == 32) ? 0xffffffffull : ((1ull << w) - 1);
    return uint32_t((acc >> sh) & m);
}

// Same for w <= 64 (DELTA_BINARY_PACKED INT64 deltas).
__device__ __forceinline__ uint64_t bits_le64(const uint8_t* p, uint64_t n, uint64_t bit, int w) {
    if (w == 0) return 0;
    if (w <= 32) return bits_le(p, n, bit, w);
    uint64_t lo = bits_le(p, n, bit, 32);
    uint64_t hi = bits_le(p, n, bit + 32, w - 32);
    return lo | (hi << 32);
}

__device__ __forceinline__ int bit_width(uint32_t max_level) { return max_level ? 32 - __clz(max_level) : 0; }

// ---- 64-bit block-wide exclusive scan (lds_wave: NT / 64 words) ----------------------------
template <int NT>
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, unsigned long long* lds_wave, uint64_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = v;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up((unsigned long long)x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) lds_wave[wid] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
    #pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const uint64_t t = lds_wave[w];
        if (w < wid) base += t;
        tot += t;
    }
    __syncthreads();   // every wave has read lds_wave before a caller's next pass overwrites it
    total = tot;
    return base + x - v;
}

// ---- block-wide exclusive scan (blockDim.x == 256, 4 waves) -----------------------------
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds_wave /*[NT/64]*/, uint32_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) lds_wave[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    #pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        uint32_t t = lds_wave[w];
        if (w < wid) base += t;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

// ---- RLE / bit-packed hybrid run walker ---------------------------------------------------
// parquet-mr RunLengthBitPackingHybridDecoder: header varint; LSB=0 -> RLE run of (h>>1)
// copies of a ceil(bw/8)-byte LE value; LSB=1 -> (h>>1) groups of 8 bit-packed values.
// Bit-packed runs are truncated to the bytes left in the stream (parquet-mr reads
// min(bytes, available) and zero-pads); an RLE value that runs past the end is an error.
//
// The walker runs on ONE lane and emits "pieces" of <= PIECE values into LDS; all threads
// then expand pieces in parallel. State survives across tiles.
constexpr int PIECE = 32;

struct RleState {
    uint64_t pos;        // byte position of the next run header
    uint64_t run_left;   // values left in the current run
    uint64_t run_bit;    // bit-packed: bit offset of the next value (relative to stream start)
    uint32_t run_val;    // RLE value
    int32_t  run_packed; // current run kind
    int32_t  err;
};

struct Piece {           // 12 bytes
    uint32_t start;      // first value index within the tile
    uint32_t data;       // RLE value, or bit offset low 32 bits
    uint16_t count;      // values
    uint16_t packed;     // 1 = bit-packed (data = bit offset)
};

__device__ __forceinline__ void rle_init(RleState& s) {
    s.pos = 0; s.run_left = 0; s.run_bit = 0; s.run_val = 0; s.run_packed = 0; s.err = 0;
}

// Walk runs to cover up to `want` values (or until `max_pieces` pieces); returns values covered.
// The state lives in LDS in every caller and `pieces` does too: the walk runs on a register copy
// (otherwise every piece store forces the state to be re-read from LDS — ~10 dependent LDS round
// trips per piece) and writes it back once.
__device__ inline uint32_t rle_walk(RleState& s_io, const uint8_t* p, uint64_t n, int bw, uint32_t want,
                                    Piece* pieces, int max_pieces, int& npieces_io) {
    RleState s = s_io;
    uint32_t got = 0;
    int npieces = 0;
    while (got < want && npieces < max_pieces) {
        if (s.run_left == 0) {
            uint64_t h;
            if (!uvarint(p, n, s.pos, h)) { s.err = 1; break; }
            if (h & 1) {
                uint64_t groups = h >> 1;
                s.run_packed = 1;
                s.run_left = groups * 8;
                s.run_bit = s.pos * 8;
                uint64_t nb = groups * uint64_t(bw);
                uint64_t avail = n - s.pos;
                s.pos += nb < avail ? nb : avail;
            } else {
                s.run_packed = 0;
                s.run_left = h >> 1;
                int nbv = (bw + 7) >> 3;
                if (s.pos + nbv > n) { s.err = 1; break; }
                uint32_t v = 0;
                for (int b = 0; b < nbv; b++) v |= uint32_t(p[s.pos + b]) << (8 * b);
                s.pos += nbv;
                s.run_val = v;
            }
            if (s.run_left == 0) continue;
        }
        uint32_t c = uint32_t(min<uint64_t>(s.run_left, uint64_t(min<uint32_t>(want - got, PIECE))));
        Piece pc;
        pc.start = got;
        pc.count = uint16_t(c);
        pc.packed = uint16_t(s.run_packed);
        if (s.run_packed) { pc.data = uint32_t(s.run_bit); s.run_bit += uint64_t(c) * bw; }
        else pc.data = s.run_val;
        pieces[npieces++] = pc;
        s.run_left -= c;
        got += c;
    }
    s_io = s;
    npieces_io = npieces;
    return got;
}

// Expand pieces into out[0..covered) (one value per element). `bitbase` is the high part of
// the bit offset (pieces store the low 32 bits; streams are < 512 MiB so 32 bits suffice).
template <typename T>
__device__ __forceinline__ void rle_expand(const Piece* pieces, int npieces, const uint8_t* p, uint64_t n,
                                           int bw, T* out) {
    for (int i = threadIdx.x; i < npieces * PIECE; i += blockDim.x) {
        int pi = i / PIECE, k = i % PIECE;
        Piece pc = pieces[pi];
        if (k >= pc.count) continue;
        uint32_t v = pc.packed ? bits_le(p, n, uint64_t(pc.data) + uint64_t(k) * bw, bw) : pc.data;
        out[pc.start + k] = T(v);
    }
}

// Stage bytes [b0, b1) of stream p[0, n) into LDS words st: byte b0 + i of the stream is byte
// off + i of st (off = the 16-byte misalignment of p + b0); stream bytes at or past n read as zero
// (parquet-mr zero-pads a truncated bit-packed run), as do the 16 bytes after the range.
__device__ __forceinline__ uint32_t stage_bytes(uint32_t* st, const uint8_t* p, uint64_t n, uint32_t b0, uint32_t b1) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p) + b0;
    const uint32_t off = uint32_t(a & 15u);
    if (b1 <= b0) return off;
    const uint32_t nchunk = (off + (b1 - b0) + 15u) / 16u;
    const PF_GLOBAL u32x4* src = (const PF_GLOBAL u32x4*)(a - off);
    const int64_t base = int64_t(b0) - int64_t(off);   // stream offset of st byte 0
    for (uint32_t c = threadIdx.x; c <= nchunk; c += blockDim.x) {
        u32x4 v = {0u, 0u, 0u, 0u};
        const int64_t cb = base + 16 * int64_t(c);   // stream offset of the chunk
        if (c < nchunk && cb < int64_t(n)) {
            v = src[c];
            if (cb + 16 > int64_t(n)) {
                #pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int64_t keep = int64_t(n) - (cb + 4 * q);   // valid bytes of word q
                    const uint32_t mask = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
                    v[q] &= mask;
                }
            }
        }
        reinterpret_cast<u32x4*>(st)[c] = v;
    }
    return off;
}

}  // namespace pf
