// pf_pages.hip — K2..K7: page decode on gfx950.
//
// Replaces the per-value work parquet-mr 1.12.2 does behind ColumnReader (called from
// src/main/java/blue/strategic/parquet/ParquetReader.java:141-168 and :196-203):
//   K2 RLE/bit-packed hybrid expansion of def/rep levels and dictionary ids
//      (RunLengthBitPackingHybridDecoder, DictionaryValuesReader)
//   K3 dictionary gather (PlainValuesDictionary.decodeToX behind getX(), :151-161)
//   K4 PLAIN decode (Integer/Long/Float/Double/Boolean/Binary/FixedLen PlainValuesReader)
//   K5 DELTA_BINARY_PACKED (DeltaBinaryPackingValuesReader[ForLong]) — pf_delta.hip
//   K6 null scatter: def == maxDef test of ParquetReader.java:146 -> validity + slot positions
//   K7 repetition levels -> list offsets (ParquetReader.java:200's rep stream)
//
// Kernels (one 256-thread workgroup per page, entries processed in tiles of TILE):
//   k_ba_*        : PLAIN BYTE_ARRAY length walks (dictionary pages, PLAIN data pages), tile-parallel
//   k_count       : per data page of BYTE_ARRAY / nested chunks: slots, values, rows, chars
//                   (+ per-value positions or dictionary ids kept in the page's aux buffer)
//   k_scan        : per chunk: exclusive scans of the page counts -> output bases
//   k_decode      : per data page: levels -> validity / list offsets / levels; values -> slots
#include <hip/hip_runtime.h>

#include "pf_device.h"
#include "pf_snappy_par.h"

namespace pf {

constexpr int NT = 256;

#ifdef PF_STAMPS
__device__ unsigned long long pf_pstamps[16];
#define PSTAMP(i, v) atomicAdd(&pf_pstamps[i], (unsigned long long)(v))
extern "C" int pf_debug_pstamps(unsigned long long* out, int n, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_pstamps), sizeof(unsigned long long) * (n < 16 ? n : 16)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pf_pstamps), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define PSTAMP(i, v) ((void)0)
#endif
#ifndef PF_TILE
#define PF_TILE 512   // k_count / k_decode level tiles: 512 beat 1024 in 6 of 6 runs (~0.7 %), 2048 3 % slower
#endif
constexpr int TILE = PF_TILE;
constexpr int EPT = TILE / NT;   // entries per thread per tile (4 consecutive)

// ---- page section layout ------------------------------------------------------------------
struct Sections {
    const uint8_t* rep; uint64_t rep_n;
    const uint8_t* def; uint64_t def_n;
    const uint8_t* val; uint64_t val_n;
    int rep_rle, def_rle;    // 1 = RLE hybrid, 0 = BIT_PACKED (v1 deprecated)
};

// v1: [rep][def][values], each RLE level section prefixed by its 4-byte LE length;
//     BIT_PACKED levels take ceil(n*bw/8) bytes, no prefix.
// v2: levels in pg.lvl (rep_len + def_len bytes, no prefixes), values in pg.body.
__device__ inline bool page_sections(const DevPage& pg, const DevChunk& ck, Sections& s) {
    s.rep = s.def = nullptr; s.rep_n = s.def_n = 0; s.rep_rle = s.def_rle = 1;
    if (pg.flags & PG_V2) {
        s.rep = pg.lvl; s.rep_n = pg.rep_len;
        s.def = pg.lvl + pg.rep_len; s.def_n = pg.def_len;
        s.val = pg.body; s.val_n = pg.body_len;
        if (ck.max_rep == 0) s.rep_n = 0;
        if (ck.max_def == 0) s.def_n = 0;
        return true;
    }
    uint64_t pos = 0, n = pg.body_len;
    const uint8_t* b = pg.body;
    for (int which = 0; which < 2; which++) {
        int maxl = which == 0 ? ck.max_rep : ck.max_def;
        if (maxl == 0) continue;
        int enc = which == 0 ? pg.rep_enc : pg.def_enc;
        const uint8_t* p; uint64_t len;
        if (enc == 3) {
            if (pos + 4 > n) return false;
            len = ld32le(b, pos, n);
            pos += 4;
            if (len > n - pos) return false;
            p = b + pos;
        } else if (enc == 4) {
            len = (uint64_t(pg.num_values) * bit_width(maxl) + 7) / 8;
            if (len > n - pos) return false;
            p = b + pos;
        } else {
            return false;
        }
        pos += len;
        if (which == 0) { s.rep = p; s.rep_n = len; s.rep_rle = enc == 3; }
        else { s.def = p; s.def_n = len; s.def_rle = enc == 3; }
    }
    s.val = b + pos; s.val_n = n - pos;
    return true;
}

// ---- tile-wise level decoding ---------------------------------------------------------------
struct LevelLds {
    Piece prep[TILE];
    Piece pdef[TILE];
    uint8_t rep[TILE];
    uint8_t def[TILE];
    RleState srep, sdef;
    int nprep, npdef;
    uint32_t count;
    int err;
};

// BIT_PACKED (deprecated, big-endian bit order: ByteBitPackingValuesReader BE) level at index i
__device__ __forceinline__ uint32_t bitpacked_be(const uint8_t* p, uint64_t n, uint64_t i, int bw) {
    uint32_t v = 0;
    for (int b = 0; b < bw; b++) {
        uint64_t bit = i * bw + b;
        v = (v << 1) | ((ld8(p, bit >> 3, n) >> (7 - (bit & 7))) & 1);
    }
    return v;
}

// Decode the levels of entries [e0, e0 + want) into L.rep / L.def; returns count (== want) or
// sets L.err. Must be called by all threads (blockDim.x >= 128).
__device__ inline uint32_t decode_level_tile(LevelLds& L, const Sections& s, const DevChunk& ck,
                                             uint64_t e0, uint32_t want) {
    const int bwr = bit_width(ck.max_rep), bwd = bit_width(ck.max_def);
    // the two walks run concurrently on lanes of different waves
    if (threadIdx.x == 0) {
        L.nprep = 0;
        if (ck.max_rep > 0 && s.rep_rle) {
            uint32_t got = rle_walk(L.srep, s.rep, s.rep_n, bwr, want, L.prep, TILE, L.nprep);
            if (got != want || L.srep.err) L.err = 1;
        }
    } else if (threadIdx.x == 64) {
        L.npdef = 0;
        if (ck.max_def > 0 && s.def_rle) {
            uint32_t got = rle_walk(L.sdef, s.def, s.def_n, bwd, want, L.pdef, TILE, L.npdef);
            if (got != want || L.sdef.err) L.err = 1;
        }
    }
    __syncthreads();
    if (L.err) return 0;
    if (ck.max_rep > 0) {
        if (s.rep_rle) rle_expand<uint8_t>(L.prep, L.nprep, s.rep, s.rep_n, bwr, L.rep);
        else for (uint32_t i = threadIdx.x; i < want; i += NT) L.rep[i] = uint8_t(bitpacked_be(s.rep, s.rep_n, e0 + i, bwr));
    } else {
        for (uint32_t i = threadIdx.x; i < want; i += NT) L.rep[i] = 0;
    }
    if (ck.max_def > 0) {
        if (s.def_rle) rle_expand<uint8_t>(L.pdef, L.npdef, s.def, s.def_n, bwd, L.def);
        else for (uint32_t i = threadIdx.x; i < want; i += NT) L.def[i] = uint8_t(bitpacked_be(s.def, s.def_n, e0 + i, bwd));
    } else {
        for (uint32_t i = threadIdx.x; i < want; i += NT) L.def[i] = 0;
    }
    __syncthreads();
    // levels above their maximum are corrupt
    int bad = 0;
    for (uint32_t i = threadIdx.x; i < want; i += NT)
        bad |= (L.rep[i] > ck.max_rep) | (L.def[i] > ck.max_def);
    if (__syncthreads_or(bad)) { if (threadIdx.x == 0) L.err = 1; __syncthreads(); return 0; }
    return want;
}

// ---- PLAIN BYTE_ARRAY walk (one lane; v1) --------------------------------------------------
// BinaryPlainValuesReader: <4-byte LE length><bytes> repeated. Writes the chars start of
// value k into pos[k]; returns total chars or -1 on overrun.
__device__ inline int64_t plain_binary_walk(const uint8_t* p, uint64_t n, int64_t count, uint32_t* pos, uint32_t* len) {
    uint64_t i = 0;
    int64_t total = 0;
    for (int64_t k = 0; k < count; k++) {
        if (i + 4 > n) return -1;
        uint32_t l = ld32le(p, i, n);
        i += 4;
        if (l > n - i) return -1;
        pos[k] = uint32_t(i);
        if (len) len[k] = l;
        i += l;
        total += l;
    }
    return total;
}

// ---- workgroup-parallel PLAIN BYTE_ARRAY walk --------------------------------------------------
// The <len><bytes> chain is serial, but a 4-byte little-endian length is "plausible" at position q
// only if q + 4 + len <= n, and a true prefix is followed by another plausible prefix (or by the
// stream end). Inside text (or most payloads) only the true prefixes pass both tests: the second
// one drops the candidates text produces just before each true prefix (the previous value's last
// byte + the low bytes of the next length). Every thread tests BW_BPT positions of a tile staged
// in LDS; the true chain is then the tile's entry plus the candidates that are another
// candidate's successor, and it must chain exactly (q_next == q + 4 + len) from the entry. Any
// mismatch — a false candidate that got linked, overflow, too few values — falls back to the exact
// serial walk, so the result is always the chain parquet-mr's BinaryPlainValuesReader reads.
constexpr int BW_BPT = 4;                           // positions per thread per tile (4: 5.5 KiB of LDS, so the
                                                    // normally idle k_ba_fallback launch does not wait for
                                                    // CUs with 21 KiB free while other streams run)
constexpr int BW_TILE = NT * BW_BPT;                // bytes per tile
constexpr int BW_LOOK = 64;                         // staged lookahead for successor tests
constexpr int BW_STAGE = BW_TILE + BW_LOOK + 16;    // + alignment shift
constexpr int BW_CAP = BW_TILE / 4;                 // candidates per tile (true prefixes are >= 4 bytes apart)

struct BinWalkLds {
    __attribute__((aligned(16))) uint8_t stage[BW_STAGE];
    uint32_t cand[BW_CAP];
    uint32_t next[BW_CAP];
    uint8_t linked[BW_CAP];    // candidate is another candidate's successor
    uint32_t acand[BW_CAP];    // accepted chain, in order
    uint32_t anext[BW_CAP];
    uint32_t scan[NT / 64];
    unsigned long long chars;
    uint32_t found, carry, bad;
};

// 4 bytes from LDS at byte offset a (a + 8 must be staged when a is not 4-aligned).
__device__ __forceinline__ uint32_t lds_read4(const uint8_t* s, uint32_t a) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
    const uint32_t sh = 8u * (a & 3u);
    return sh ? (w[0] >> sh) | (w[1] << (32u - sh)) : w[0];
}

// Stage p[base - woff, base - woff + bytes) into LDS with 16-byte loads by the whole workgroup;
// 16-byte chunks wholly at or past n read as zero. Returns woff (base's 16-B misalignment).
__device__ __forceinline__ uint32_t wg_stage(uint8_t* stage, const uint8_t* p, uint64_t n, uint64_t base,
                                             uint32_t bytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + base);
    const uint32_t woff = uint32_t(a & 15u);
    const uint4* src = reinterpret_cast<const uint4*>(a - woff);
    const int64_t first = int64_t(base) - int64_t(woff);
    for (uint32_t c = threadIdx.x; c < bytes / 16; c += blockDim.x) {
        const int64_t q = first + int64_t(c) * 16;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (q < int64_t(n)) v = src[c];
        reinterpret_cast<uint4*>(stage)[c] = v;
    }
    return woff;
}

// The walk over candidates inside a tile: the true chain is the tile's entry E plus every
// candidate that is the successor of another candidate (a true value's successor is the next true
// value; a false candidate's successor is a random far position, so false candidates are almost
// never linked). The accepted list must still chain exactly from E and leave the tile; a false
// candidate that does get linked breaks that check and the page takes the serial walk.
constexpr int BW_CPT = BW_CAP / NT;                 // candidates owned by a thread (contiguous)

__device__ inline int64_t binary_walk_wg(const uint8_t* p, uint64_t n, int64_t count, uint32_t* pos, uint32_t* len,
                                         BinWalkLds& W) {
    const int tid = threadIdx.x;
    if (tid == 0) { W.found = 0; W.carry = 0; W.bad = 0; W.chars = 0; }
    __syncthreads();
    if (count == 0) return 0;
    if (n > 0x7fffffffull) return -1;
#ifdef PF_STAMPS
    const unsigned long long t_beg = __builtin_amdgcn_s_memtime();
    if (tid == 0) PSTAMP(0, 1);
#endif
    for (uint64_t t0 = 0; t0 < n; t0 += BW_TILE) {
        if (W.found >= uint64_t(count) || W.bad) break;
        const uint32_t E = W.carry;                 // true chain position entering this tile
        const uint64_t tend = min(t0 + BW_TILE, n);
        if (E >= tend) continue;                    // one value spans the whole tile
#ifdef PF_STAMPS
        unsigned long long t_ph = __builtin_amdgcn_s_memtime();
#endif
        const uint32_t woff = wg_stage(W.stage, p, n, t0, BW_STAGE);
        for (uint32_t i = tid; i < BW_CAP / 4; i += NT) reinterpret_cast<uint32_t*>(W.linked)[i] = 0;
        __syncthreads();
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(9, t_ - t_ph); t_ph = t_; }
#endif

        const uint64_t b0 = t0 + uint64_t(tid) * BW_BPT;
        uint32_t flags = 0, L[BW_BPT];
        #pragma unroll
        for (int i = 0; i < BW_BPT; i++) {
            const uint64_t q = b0 + i;
            L[i] = 0;
            if (q + 4 <= n && q >= E) {
                const uint32_t l = lds_read4(W.stage, woff + uint32_t(q - t0));
                if (uint64_t(l) <= n - q - 4) {
                    const uint64_t s = q + 4 + l;
                    bool ok = s == n;
                    if (!ok && s + 4 <= n) {
                        const uint32_t l2 = s + 8 <= t0 + BW_TILE + BW_LOOK ? lds_read4(W.stage, woff + uint32_t(s - t0))
                                                                              : ld32le(p, s, n);
                        ok = uint64_t(l2) <= n - s - 4;
                    }
                    if (ok) { flags |= 1u << i; L[i] = l; }
                }
            }
        }
        uint32_t tot;
        uint32_t idx = block_excl_scan<NT>(__popc(flags), W.scan, tot);
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(10, t_ - t_ph); t_ph = t_; }
#endif

        if (tot > BW_CAP || tot == 0) { if (tid == 0) { W.bad = 1; PSTAMP(5, 1); } __syncthreads(); break; }
#ifdef PF_STAMPS
        if (tid == 0) PSTAMP(1, 1);
#endif
        #pragma unroll
        for (int i = 0; i < BW_BPT; i++) {
            if ((flags >> i) & 1u) {
                const uint32_t q = uint32_t(b0 + i);
                W.cand[idx] = q;
                W.next[idx] = q + 4 + L[i];
                idx++;
            }
        }
        __syncthreads();
        // link: mark every candidate that is another candidate's successor
        for (uint32_t i = tid; i < tot; i += NT) {
            const uint32_t s = W.next[i];
            if (s >= tend) continue;
            uint32_t lo = i + 1, hi = tot;   // successors lie at higher indices
            while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (W.cand[m] < s) lo = m + 1; else hi = m; }
            if (lo < tot && W.cand[lo] == s) W.linked[lo] = 1;
        }
        __syncthreads();
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(11, t_ - t_ph); t_ph = t_; }
#endif

        // accepted = the entry + linked candidates, ranked in position order over contiguous ranges
        const uint32_t i0 = uint32_t(tid) * BW_CPT;
        uint32_t am = 0;
        #pragma unroll
        for (int k = 0; k < BW_CPT; k++) {
            const uint32_t i = i0 + k;
            am |= uint32_t(i < tot && (W.linked[i] || W.cand[i] == E)) << k;
        }
        uint32_t atot;
        uint32_t r = block_excl_scan<NT>(__popc(am), W.scan, atot);
        const uint32_t base = W.found;
        uint64_t my_chars = 0;
        #pragma unroll
        for (int k = 0; k < BW_CPT; k++) {
            if (!((am >> k) & 1u)) continue;
            const uint32_t q = W.cand[i0 + k], s = W.next[i0 + k];
            W.acand[r] = q;
            W.anext[r] = s;
            const uint64_t kk = uint64_t(base) + r;
            if (kk < uint64_t(count)) {
                pos[kk] = q + 4;
                if (len) len[kk] = s - q - 4;
                my_chars += s - q - 4;
            }
            r++;
        }
        __syncthreads();
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(12, t_ - t_ph); t_ph = t_; }
#endif

        // the accepted list chains exactly from E and its last value leaves the tile
        int bad = 0;
        for (uint32_t a = tid; a < atot; a += NT) {
            if (uint64_t(base) + a >= uint64_t(count)) continue;
            bad |= W.acand[a] != (a == 0 ? E : W.anext[a - 1]);
        }
        if (tid == 0 && (atot == 0 || (W.anext[atot - 1] < tend && uint64_t(base) + atot < uint64_t(count)))) bad = 1;
        if (my_chars) atomicAdd(&W.chars, (unsigned long long)my_chars);
        bad = __syncthreads_or(bad);
        if (tid == 0) {
            if (bad) { W.bad = 1; PSTAMP(7, 1); }
            else W.carry = W.anext[atot - 1];
            W.found = base + atot;
        }
        __syncthreads();
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(13, t_ - t_ph); t_ph = t_; }
#endif

    }
    __syncthreads();
#ifdef PF_STAMPS
    const unsigned long long t_mid = __builtin_amdgcn_s_memtime();
    if (tid == 0) PSTAMP(3, t_mid - t_beg);
#endif
    if (!W.bad && W.found >= uint64_t(count)) return int64_t(W.chars);
    // exact serial fallback (candidates the filters could not separate, or corrupt pages)
    __shared__ long long s_res;
    if (tid == 0) s_res = plain_binary_walk(p, n, count, pos, len);
    __syncthreads();
#ifdef PF_STAMPS
    if (tid == 0) { PSTAMP(2, 1); PSTAMP(4, __builtin_amdgcn_s_memtime() - t_mid); if (!W.bad) PSTAMP(8, 1); }
#endif
    return s_res;
}

// ---- tile-parallel PLAIN BYTE_ARRAY walk (k_ba_*) ----------------------------------------------
// BinaryPlainValuesReader reads <4-byte LE length><bytes> values one after another: a serial
// chain. Spread over the whole GPU instead of one workgroup per page:
//   k_ba_cand   every stream position q is a candidate if its length fits the stream, the
//               position after the value is the stream end or again a fitting length, and q + 1
//               is not plausible too (in text that pair is <char><len><0><0>: q is the char);
//   k_ba_link   (twice) link1 = successors of candidates, link2 = successors of link1 members
//               (position 0 is in both): a true value k >= 2 is in link2; a false candidate
//               needs two false predecessors lined up to get there;
//   k_ba_count / k_ba_scan  accepted = cand & link2, counted per tile, scanned per job; the total
//               must be the page's value count;
//   k_ba_emit   value k's chars start (and length) by rank;
//   k_ba_verify every accepted value's end must be the next accepted value's start, value 0 at 0;
//   k_ba_fallback  jobs that failed any check take the workgroup walk (binary_walk_wg, which ends
//               in the exact serial walk), so results never depend on the filters.
constexpr uint32_t BA_TILE = NT * 32;          // 8 KiB of stream per tile: one bitmap word per thread
constexpr uint32_t BA_STAGE = BA_TILE + 32;    // + alignment shift and the lookahead of a length

__device__ __forceinline__ uint32_t ba_stage(uint8_t* stg, const uint8_t* p, uint64_t n, uint64_t base) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + base);
    const uint32_t woff = uint32_t(a & 15u);
    const uint4* src = reinterpret_cast<const uint4*>(a - woff);
    const int64_t first = int64_t(base) - int64_t(woff);
    constexpr uint32_t NCH = BA_STAGE / 16, BU = (NCH + NT - 1) / NT;   // (all loads in flight, round 6)
    uint4 v[BU];
    #pragma unroll
    for (uint32_t u = 0; u < BU; u++) {
        const uint32_t c = threadIdx.x + NT * u;
        v[u] = make_uint4(0, 0, 0, 0);
        if (c < NCH && first + int64_t(c) * 16 < int64_t(n)) v[u] = src[c];
    }
    #pragma unroll
    for (uint32_t u = 0; u < BU; u++) {
        const uint32_t c = threadIdx.x + NT * u;
        if (c < NCH) reinterpret_cast<uint4*>(stg)[c] = v[u];
    }
    return woff;
}

__device__ __forceinline__ uint32_t lds_le32(const uint8_t* s, uint32_t a) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
    const uint32_t sh = 8u * (a & 3u);
    return sh ? ((w[0] >> sh) | (w[1] << (32u - sh))) : w[0];
}

__global__ __launch_bounds__(NT) void k_ba_cand(BaJob* __restrict__ jobs, const int2* __restrict__ tiles) {
    __shared__ __attribute__((aligned(16))) uint8_t stg[BA_STAGE];
    const int2 jt = tiles[blockIdx.x];
    const BaJob& J = jobs[jt.x];
    if (J.state != BA_OK) return;
    const uint32_t n = J.n;
    const uint32_t t0 = uint32_t(jt.y) * BA_TILE;
    if (t0 >= n) return;
    const uint8_t* p = J.p;
    const uint32_t woff = ba_stage(stg, p, n, t0);
    __syncthreads();
    const uint32_t wi = t0 / 32 + threadIdx.x;
    const uint32_t q0 = t0 + threadIdx.x * 32u;
    // lengths that fit the stream, for all 33 positions q0 .. q0 + 32 at once: the 36 bytes from q0
    // as 9 byte-aligned dwords, each position's little-endian length one v_alignbyte away (text
    // almost never passes: its "lengths" are 4 characters, far larger than the page)
    uint64_t fit = 0;
    {
        const uint32_t a = woff + threadIdx.x * 32u;
        const uint32_t* d = reinterpret_cast<const uint32_t*>(stg + (a & ~3u));
        const uint32_t s = a & 3u;
        uint32_t D[10], E[9];
        #pragma unroll
        for (int i = 0; i < 10; i++) D[i] = (a & ~3u) + 4u * i + 4u <= BA_STAGE ? d[i] : 0u;
        #pragma unroll
        for (int i = 0; i < 9; i++) E[i] = __builtin_amdgcn_alignbyte(D[i + 1], D[i], s);
        const int64_t room = int64_t(n) - int64_t(q0) - 4;   // a length at q0 + b fits if <= room - b
        #pragma unroll
        for (int b = 0; b <= 32; b++) {
            const uint32_t l = (b & 3) == 0 ? E[b >> 2] : __builtin_amdgcn_alignbyte(E[(b >> 2) + 1], E[b >> 2], b & 3);
            fit |= uint64_t(int64_t(l) <= room - b) << b;
        }
    }
    uint64_t m = 0;   // plausible positions: the length fits and the next value's length fits too
    for (uint64_t f = fit; f;) {
        const int b = __ffsll((unsigned long long)f) - 1;
        f &= f - 1;
        const uint32_t q = q0 + uint32_t(b);
        const uint32_t sv = q + 4 + lds_le32(stg, woff + (q - t0));
        bool ok = sv == n;
        if (!ok && uint64_t(sv) + 4 <= n) {
            const uint32_t ls = sv - t0 + 4 <= BA_TILE + 8 ? lds_le32(stg, woff + (sv - t0)) : ld32le(p, sv, n);
            ok = ls <= n - sv - 4;
        }
        m |= uint64_t(ok) << b;
    }
    // a plausible position followed by another is the byte before a true length prefix in text
    // (<char><len><0><0>): drop it (a true value that this drops fails the count check and takes
    // the exact fallback walk)
    J.cand[wi] = uint32_t(m & ~(m >> 1));
    J.link1[wi] = wi == 0 ? 1u : 0u;
    J.link2[wi] = wi == 0 ? 1u : 0u;
}

__global__ __launch_bounds__(NT) void k_ba_link(BaJob* __restrict__ jobs, const int2* __restrict__ tiles, int level) {
    __shared__ __attribute__((aligned(16))) uint8_t stg[BA_STAGE];
    const int2 jt = tiles[blockIdx.x];
    const BaJob& J = jobs[jt.x];
    if (J.state != BA_OK) return;
    const uint32_t n = J.n;
    const uint32_t t0 = uint32_t(jt.y) * BA_TILE;
    if (t0 >= n) return;
    const uint32_t woff = ba_stage(stg, J.p, n, t0);
    __syncthreads();
    const uint32_t wi = t0 / 32 + threadIdx.x;
    const uint32_t* cand = J.cand;
    uint32_t* to = level == 1 ? J.link1 : J.link2;
    uint32_t m = cand[wi];
    if (level == 2) m &= J.link1[wi];
    while (m) {
        const uint32_t q = wi * 32u + uint32_t(__ffs(m) - 1);
        m &= m - 1;
        const uint32_t sv = q + 4 + lds_le32(stg, woff + (q - t0));
        if (sv < n && ((cand[sv >> 5] >> (sv & 31u)) & 1u)) atomicOr(&to[sv >> 5], 1u << (sv & 31u));
    }
}

// k_ba_cand + k_ba_link (both levels) + k_ba_count + k_ba_verify's chain check in one kernel per tile
// (round 4). The links of a position come from candidates at most BA_HALO bytes before it, so a tile
// computes candidates over [t0 - 2 BA_HALO, t1 + BA_HALO), first links over [t0 - BA_HALO, t1 +
// BA_HALO) and second links over [t0, t1 + BA_HALO) from one staged window (LDS bitmaps, no global
// atomics); positions both tiles see get the same bits. It writes the tile's accepted words and count,
// and checks the chain locally: every accepted value of the tile must end exactly at the next accepted
// position (and the job's first accepted position is 0); with the count check of k_ba_scan that is
// k_ba_verify's test. A value longer than BA_HALO - 4 bytes is not linked here: its page fails the count
// or the chain check (BA_RELINK) and k_ba_fallback re-links it over the whole job (ba_relink_wg, any
// value length) before it would take the exact walk, so the emitted positions are always the verified
// true chain.
constexpr int BA_HALO = 128;
constexpr uint32_t BA_XW = (2 * BA_HALO) / 32;                       // halo words before the tile
constexpr uint32_t BA_NW = BA_XW + BA_TILE / 32 + BA_HALO / 32;        // words of the window
constexpr uint32_t BA_FSTAGE = 3 * BA_HALO + BA_TILE + 48;           // staged bytes from t0 - 2 BA_HALO
__global__ __launch_bounds__(NT) void k_ba_tile(BaJob* __restrict__ jobs, const int2* __restrict__ tiles) {
    __shared__ __attribute__((aligned(16))) uint8_t stg[BA_FSTAGE + 16];
    __shared__ uint32_t C[BA_NW], L1[BA_NW], L2[BA_NW];
    __shared__ uint32_t tmp[NT / 64];
    const int2 jt = tiles[blockIdx.x];
    BaJob& J = jobs[jt.x];
    // a job another tile already rejected (BA_RELINK) still needs this tile's candidate words:
    // ba_relink_wg re-links the job from the whole candidate bitmap
    const int32_t st0 = J.state;
    if (st0 == BA_SKIP || st0 == BA_FALLBACK) return;
    const uint32_t n = J.n;
    const uint32_t t0 = uint32_t(jt.y) * BA_TILE;
    if (t0 >= n) {
        if (threadIdx.x == 0) J.tile_cnt[jt.y] = 0;
        return;
    }
    const uint8_t* p = J.p;
    const int64_t sb = int64_t(t0) - 2 * BA_HALO;   // stream position of word 0 / stage byte woff
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(p) + uintptr_t(sb);
    const uint32_t woff = uint32_t(a0 & 15u);
    {   // 16-byte loads; chunks wholly before the stream start or at / past its end are zero (the chunk
        // holding byte 0 is read whole, as ba_stage does)
        const int64_t first = sb - int64_t(woff);
        const PF_GLOBAL u32x4* src = (const PF_GLOBAL u32x4*)(a0 - woff);
        constexpr uint32_t NCH = (BA_FSTAGE + 16) / 16, BU = (NCH + NT - 1) / NT;   // (all loads in flight, round 6)
        u32x4 v[BU];
        #pragma unroll
        for (uint32_t u = 0; u < BU; u++) {
            const uint32_t c = threadIdx.x + NT * u;
            const int64_t q = first + int64_t(c) * 16;
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (c < NCH && q + 16 > 0 && q < int64_t(n)) v[u] = src[c];
        }
        #pragma unroll
        for (uint32_t u = 0; u < BU; u++) {
            const uint32_t c = threadIdx.x + NT * u;
            if (c < NCH) reinterpret_cast<u32x4*>(stg)[c] = v[u];
        }
    }
    for (uint32_t i = threadIdx.x; i < BA_NW; i += NT) { C[i] = 0; L1[i] = 0; L2[i] = 0; }
    __syncthreads();
    auto len_at = [&](int64_t q) { return lds_le32(stg, woff + uint32_t(q - sb)); };   // q in the window
    // ---- candidates (k_ba_cand's rule)
    for (uint32_t w = threadIdx.x; w < BA_NW; w += NT) {
        const int64_t q0 = sb + int64_t(w) * 32;
        if (q0 + 32 <= 0 || q0 >= int64_t(n)) continue;
        const uint32_t a = woff + w * 32u;
        const uint32_t* d = reinterpret_cast<const uint32_t*>(stg + (a & ~3u));
        const uint32_t s = a & 3u;
        uint32_t D[10], E[9];
        #pragma unroll
        for (int i = 0; i < 10; i++) D[i] = d[i];
        #pragma unroll
        for (int i = 0; i < 9; i++) E[i] = __builtin_amdgcn_alignbyte(D[i + 1], D[i], s);
        const int64_t room = int64_t(n) - q0 - 4;
        uint64_t fit = 0;
        #pragma unroll
        for (int b = 0; b <= 32; b++) {
            const uint32_t l = (b & 3) == 0 ? E[b >> 2] : __builtin_amdgcn_alignbyte(E[(b >> 2) + 1], E[b >> 2], b & 3);
            fit |= uint64_t(int64_t(l) <= room - b && q0 + b >= 0) << b;
        }
        uint64_t m = 0;
        for (uint64_t f = fit; f;) {
            const int b = __ffsll((unsigned long long)f) - 1;
            f &= f - 1;
            const int64_t q = q0 + b;
            const uint32_t sv = uint32_t(q) + 4 + len_at(q);
            bool ok = sv == n;
            if (!ok && uint64_t(sv) + 4 <= n) {
                // a successor past the staged window is taken as plausible without reading it (round 5):
                // in text that is mostly the byte before a true length (<char><len><0><0> reads as a
                // length of a few thousand), which the adjacency rule below drops anyway, and the chain
                // and count checks decide the rest; the global read per value was k_ba_tile's 2.3x fetch
                const int64_t r = int64_t(sv) - sb;
                ok = r + 4 > int64_t(BA_FSTAGE) || lds_le32(stg, woff + uint32_t(r)) <= n - sv - 4;
            }
            m |= uint64_t(ok) << b;
        }
        C[w] = uint32_t(m & ~(m >> 1));
    }
    __syncthreads();
    const int64_t wend = sb + int64_t(BA_NW) * 32;   // end of the window
    // ---- first links: successors (within the halo) of candidates, over [t0 - BA_HALO, wend)
    for (uint32_t w = threadIdx.x; w < BA_NW; w += NT) {
        uint32_t mm = C[w];
        while (mm) {
            const uint32_t b = uint32_t(__ffs(mm) - 1);
            mm &= mm - 1;
            const int64_t q = sb + int64_t(w) * 32 + b;
            const int64_t sv = q + 4 + int64_t(len_at(q));
            if (sv - q <= BA_HALO && sv >= int64_t(t0) - BA_HALO && sv < wend && sv < int64_t(n)) {
                const uint32_t r = uint32_t(sv - sb);
                atomicOr(&L1[r >> 5], 1u << (r & 31u));
            }
        }
    }
    if (threadIdx.x == 0 && t0 == 0) atomicOr(&L1[BA_XW], 1u);   // position 0 starts the chain
    __syncthreads();
    // ---- second links: successors of candidates that are first links, over [t0, wend)
    for (uint32_t w = BA_XW / 2 + threadIdx.x; w < BA_NW; w += NT) {
        uint32_t mm = C[w] & L1[w];
        while (mm) {
            const uint32_t b = uint32_t(__ffs(mm) - 1);
            mm &= mm - 1;
            const int64_t q = sb + int64_t(w) * 32 + b;
            const int64_t sv = q + 4 + int64_t(len_at(q));
            if (sv - q <= BA_HALO && sv >= int64_t(t0) && sv < wend && sv < int64_t(n)) {
                const uint32_t r = uint32_t(sv - sb);
                atomicOr(&L2[r >> 5], 1u << (r & 31u));
            }
        }
    }
    if (threadIdx.x == 0 && t0 == 0) atomicOr(&L2[BA_XW], 1u);
    __syncthreads();
    // ---- accepted = candidates & second links: the tile's words, its count, the local chain check
    const uint32_t w = BA_XW + threadIdx.x;
    const uint32_t acc = C[w] & L2[w];
    const uint32_t wi = t0 / 32 + threadIdx.x;
    J.cand[wi] = C[w];
    J.link2[wi] = L2[w];
    bool bad = t0 == 0 && threadIdx.x == 0 && !(acc & 1u);   // the chain starts at position 0
    for (uint32_t mm = acc; mm && !bad;) {
        const uint32_t b = uint32_t(__ffs(mm) - 1);
        mm &= mm - 1;
        const int64_t q = sb + int64_t(w) * 32 + b;
        const int64_t sv = q + 4 + int64_t(len_at(q));
        // a value ending past the halo cannot be checked here (the exact walk takes the page)
        if (sv != int64_t(n) && sv - q > BA_HALO) { bad = true; break; }
        // the next accepted position after q must be sv: no accepted bit in (q, min(sv, wend)), bit sv set
        const int64_t stop = min(sv, wend);
        for (int64_t x = q + 1; x < stop;) {
            const uint32_t r = uint32_t(x - sb), ww = r >> 5;
            const uint32_t word = (C[ww] & L2[ww]) >> (r & 31u);
            const int64_t span = min(int64_t(32 - (r & 31u)), stop - x);
            if (word & (span >= 32 ? 0xffffffffu : ((1u << span) - 1u))) { bad = true; break; }
            x += span;
        }
        if (!bad && sv < wend && sv < int64_t(n)) {
            const uint32_t r = uint32_t(sv - sb);
            bad = !(((C[r >> 5] & L2[r >> 5]) >> (r & 31u)) & 1u);
        }
    }
    uint32_t tot;
    block_excl_scan<NT>(__popc(acc), tmp, tot);
    if (threadIdx.x == 0) J.tile_cnt[jt.y] = tot;
    if (__syncthreads_or(bad) && threadIdx.x == 0) atomicExch(&J.state, int32_t(BA_RELINK));
}

__global__ __launch_bounds__(NT) void k_ba_count(BaJob* __restrict__ jobs, const int2* __restrict__ tiles) {
    __shared__ uint32_t tmp[NT / 64];
    const int2 jt = tiles[blockIdx.x];
    const BaJob& J = jobs[jt.x];
    if (J.state != BA_OK) return;
    const uint32_t t0 = uint32_t(jt.y) * BA_TILE;
    if (t0 >= J.n) {
        if (threadIdx.x == 0) J.tile_cnt[jt.y] = 0;
        return;
    }
    const uint32_t wi = t0 / 32 + threadIdx.x;
    uint32_t tot;
    block_excl_scan<NT>(__popc(J.cand[wi] & J.link2[wi]), tmp, tot);
    if (threadIdx.x == 0) J.tile_cnt[jt.y] = tot;
}

__global__ __launch_bounds__(NT) void k_ba_scan(BaJob* __restrict__ jobs, int32_t fail_state) {
    __shared__ uint32_t tmp[NT / 64];
    BaJob& J = jobs[blockIdx.x];
    if (J.state != BA_OK) return;
    uint64_t run = 0;
    for (uint32_t b = 0; b < J.n_tiles; b += NT) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < J.n_tiles ? J.tile_cnt[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<NT>(v, tmp, tot);
        if (i < J.n_tiles) J.tile_cnt[i] = uint32_t(run) + ex;
        run += tot;
    }
    if (threadIdx.x == 0 && int64_t(run) != J.count) {
        J.state = fail_state;   // (fused: BA_RELINK; round-3 kernels: BA_FALLBACK)
        PSTAMP(14, 1);
        PSTAMP(15, run > uint64_t(J.count) ? run - uint64_t(J.count) : 0);
    }
}

__global__ __launch_bounds__(NT) void k_ba_emit(BaJob* __restrict__ jobs, const int2* __restrict__ tiles) {
    __shared__ uint32_t tmp[NT / 64];
    const int2 jt = tiles[blockIdx.x];
    const BaJob& J = jobs[jt.x];
    if (J.state != BA_OK) return;
    const uint32_t n = J.n;
    const uint32_t t0 = uint32_t(jt.y) * BA_TILE;
    if (t0 >= n) return;
    const uint32_t wi = t0 / 32 + threadIdx.x;
    uint32_t m = J.cand[wi] & J.link2[wi];
    uint32_t tot;
    uint64_t k = uint64_t(J.tile_cnt[jt.y]) + block_excl_scan<NT>(__popc(m), tmp, tot);
    const uint64_t count = uint64_t(J.count);
    while (m) {
        const uint32_t q = wi * 32u + uint32_t(__ffs(m) - 1);
        m &= m - 1;
        if (k < count) {
            J.pos[k] = q + 4;
            if (J.len || k + 1 == count) {
                const uint32_t l = ld32le(J.p, q, n);
                if (J.len) J.len[k] = l;
                if (k + 1 == count && J.chars_out) *J.chars_out = int64_t(q) + 4 + int64_t(l) - 4 * int64_t(count);
            }
        }
        k++;
    }
}

__global__ __launch_bounds__(NT) void k_ba_verify(BaJob* __restrict__ jobs, const int2* __restrict__ tiles) {
    __shared__ uint32_t tmp[NT / 64];
    const int2 jt = tiles[blockIdx.x];
    BaJob& J = jobs[jt.x];
    if (J.state != BA_OK) return;
    const uint32_t n = J.n;
    const uint32_t t0 = uint32_t(jt.y) * BA_TILE;
    if (t0 >= n) return;
    const uint32_t wi = t0 / 32 + threadIdx.x;
    uint32_t m = J.cand[wi] & J.link2[wi];
    uint32_t tot;
    uint64_t k = uint64_t(J.tile_cnt[jt.y]) + block_excl_scan<NT>(__popc(m), tmp, tot);
    const uint64_t count = uint64_t(J.count);
    int bad = 0;
    while (m) {
        const uint32_t q = wi * 32u + uint32_t(__ffs(m) - 1);
        m &= m - 1;
        const uint32_t nq = q + 4 + ld32le(J.p, q, n);
        if (k == 0 && q != 0) bad = 1;
        if (k + 1 < count) bad |= J.pos[k + 1] != nq + 4;
        else if (k + 1 == count) { if (J.chars_out) *J.chars_out = int64_t(nq) - 4 * int64_t(count); }
        else bad = 1;
        k++;
    }
    if (__syncthreads_or(bad) && threadIdx.x == 0) { atomicExch(&J.state, int32_t(BA_FALLBACK)); PSTAMP(6, 1); }
}

// A job k_ba_tile rejected (BA_RELINK), in one workgroup: k_ba_link's rule over the job's whole
// candidate bitmap (k_ba_tile wrote it; successors at any distance, so values of any length), then
// k_ba_count / k_ba_scan / k_ba_emit / k_ba_verify's count, emit and chain check over the job's words
// in order. Returns -1 on every thread when the chain does not verify (the exact walk takes the job);
// otherwise the job's chars on the thread holding its last value and 0 on the others.
// Link words are read back with agent-scope loads (their bits were set by global atomics).
__device__ int64_t ba_relink_wg(BaJob& J, uint32_t* tmp) {
    const uint32_t n = J.n;
    const int64_t count = J.count;
    if (n == 0 || count <= 0) return -1;
    const uint32_t nw = (n + 31u) / 32u;
    const uint8_t* p = J.p;
    const uint32_t* cand = J.cand;
    uint32_t* l1 = J.link1;
    uint32_t* l2 = J.link2;
    auto ld = [](const uint32_t* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (uint32_t w = threadIdx.x; w < nw; w += NT) { l1[w] = w == 0 ? 1u : 0u; l2[w] = w == 0 ? 1u : 0u; }
    __syncthreads();
    for (int level = 1; level <= 2; level++) {   // link1: successors of candidates; link2: of link1 members
        uint32_t* to = level == 1 ? l1 : l2;
        for (uint32_t w = threadIdx.x; w < nw; w += NT) {
            uint32_t m = cand[w];
            if (level == 2) m &= ld(l1 + w);
            while (m) {
                const uint32_t q = w * 32u + uint32_t(__ffs(m) - 1);
                m &= m - 1;
                const uint64_t sv = uint64_t(q) + 4 + ld32le(p, q, n);
                if (sv < n && ((cand[sv >> 5] >> (sv & 31u)) & 1u)) atomicOr(&to[sv >> 5], 1u << (sv & 31u));
            }
        }
        __syncthreads();
    }
    // accepted = cand & link2: emit by rank, then check the chain (value k + 1 starts where k ends)
    int64_t run = 0;
    for (uint32_t b = 0; b < nw; b += NT) {
        const uint32_t w = b + threadIdx.x;
        uint32_t m = w < nw ? cand[w] & ld(l2 + w) : 0u;
        uint32_t tot;
        int64_t k = run + block_excl_scan<NT>(__popc(m), tmp, tot);
        while (m) {
            const uint32_t q = w * 32u + uint32_t(__ffs(m) - 1);
            m &= m - 1;
            if (k < count) {
                J.pos[k] = q + 4;
                if (J.len) J.len[k] = ld32le(p, q, n);
            }
            k++;
        }
        run += tot;
    }
    if (run != count) return -1;   // (uniform: every thread ran the same scans)
    __syncthreads();
    int bad = 0;
    int64_t chars = 0;
    run = 0;
    for (uint32_t b = 0; b < nw; b += NT) {
        const uint32_t w = b + threadIdx.x;
        uint32_t m = w < nw ? cand[w] & ld(l2 + w) : 0u;
        uint32_t tot;
        int64_t k = run + block_excl_scan<NT>(__popc(m), tmp, tot);
        while (m) {
            const uint32_t q = w * 32u + uint32_t(__ffs(m) - 1);
            m &= m - 1;
            const uint64_t nq = uint64_t(q) + 4 + ld32le(p, q, n);
            if (k == 0 && q != 0) bad = 1;
            if (k + 1 < count) bad |= ld(J.pos + k + 1) != nq + 4;
            else chars = int64_t(nq) - 4 * count;   // (k + 1 == count: run == count)
            k++;
        }
        run += tot;
    }
    if (__syncthreads_or(bad)) return -1;
    return chars;   // (the thread that holds the last value; 0 on the others)
}

// Grid-stride over the jobs with a small grid: nearly every walk was accepted by the checks above,
// and a block per job (21 KB of LDS each) would wait for CUs held by other streams' kernels.
#ifdef PF_DIAG   // diagnostics build: jobs k_ba_fallback re-linked / walked exactly (tests)
__device__ unsigned long long pf_ba_counts[2];
extern "C" int pf_debug_ba_counts(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_ba_counts), sizeof(unsigned long long) * 2) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[2] = {0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pf_ba_counts), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#define BA_COUNT(i) (threadIdx.x == 0 ? (void)atomicAdd(&pf_ba_counts[i], 1ull) : (void)0)
#else
#define BA_COUNT(i) ((void)0)
#endif
__global__ __launch_bounds__(NT) void k_ba_fallback(BaJob* __restrict__ jobs, int n_jobs, DevChunkResult* res) {
    __shared__ BinWalkLds W;
    __shared__ long long s_chars;
    for (int j = blockIdx.x; j < n_jobs; j += gridDim.x) {
        BaJob& J = jobs[j];
        if (J.state == BA_RELINK) {
            if (threadIdx.x == 0) s_chars = 0;
            __syncthreads();
            const int64_t c = ba_relink_wg(J, W.scan);   // (c < 0 on every thread or on none)
            if (c > 0) atomicAdd(reinterpret_cast<unsigned long long*>(&s_chars), (unsigned long long)c);
            __syncthreads();
            if (c >= 0) {
                if (threadIdx.x == 0 && J.chars_out) *J.chars_out = s_chars;
                BA_COUNT(0);
                __syncthreads();
                continue;
            }
        } else if (J.state != BA_FALLBACK) {
            continue;
        }
        const int64_t t = binary_walk_wg(J.p, J.n, J.count, J.pos, J.len, W);
        BA_COUNT(1);
        if (threadIdx.x == 0) {
            if (t < 0) set_status(res, J.chunk, ST_CORRUPT, J.page);
            else if (J.chars_out) *J.chars_out = t;
        }
        __syncthreads();
    }
}

// ---- values helpers ------------------------------------------------------------------------
constexpr uint32_t DSTR_CAP = 256;   // string dictionaries up to this many entries: {pos, len} staged in LDS
constexpr uint32_t FBLK = 4096;      // entries per k_flat workgroup: pages are split into blocks

// BYTE_ARRAY data pages: chars of the entries before each FBLK block (k_count, dictionary pages),
// kept after the page's aux entries.
__device__ __forceinline__ uint64_t* flat_block_chars(const DevPage& pg) {
    if (!pg.aux) return nullptr;
    const uintptr_t a = reinterpret_cast<uintptr_t>(pg.aux + pg.aux_cap + 1);
    return reinterpret_cast<uint64_t*>((a + 7) & ~uintptr_t(7));
}
__device__ __forceinline__ bool is_dict_enc(int e) { return e == 2 || e == 8; }

// ---- k_count ---------------------------------------------------------------------------------
struct CountLds {
    LevelLds L;
    Piece pval[TILE];
    uint32_t ids[TILE];
    uint32_t scan_tmp[NT / 64];
    RleState sval;
    int npval, verr;
    unsigned long long chars_acc;
};

__device__ void count_page(const DevChunk* __restrict__ chunks, DevPage* pages, int pi, DevChunkResult* res, BaJob* bajobs,
                           CountLds& C) {
    LevelLds& L = C.L;
    Piece* pval = C.pval;
    uint32_t* ids = C.ids;
    uint32_t* scan_tmp = C.scan_tmp;
    RleState& sval = C.sval;
    int& npval = C.npval;
    int& verr = C.verr;
    unsigned long long& chars_acc = C.chars_acc;
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (res[pg.chunk].status != 0) return;   // an earlier stage failed this chunk
    if (pg.counted == 1 || pg.seg_ok == 1) return;   // counted by k_count_flat / k_count_seg
    Sections s;
    const bool ok = page_sections(pg, ck, s);
    if (threadIdx.x == 0) {
        rle_init(L.srep); rle_init(L.sdef); rle_init(sval);
        L.err = ok ? 0 : 1; verr = 0; chars_acc = 0;
        sval.pos = 1;    // dictionary ids: skip the bit-width byte
    }
    __syncthreads();
    if (L.err) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }

    const bool dict = is_dict_enc(pg.encoding);
    const bool binary = ck.ptype == 6;
    const int id_bw = (dict && s.val_n > 0) ? int(s.val[0]) : 0;
    uint64_t slots = 0, vals = 0, rows = 0;
    uint64_t* blk_chars = flat_block_chars(pg);
    for (uint64_t e0 = 0; e0 < uint64_t(pg.num_values); e0 += TILE) {
        uint32_t want = uint32_t(min<uint64_t>(TILE, uint64_t(pg.num_values) - e0));
        if (binary && dict && blk_chars && e0 % FBLK == 0 && threadIdx.x == 0) blk_chars[e0 / FBLK] = chars_acc;
        decode_level_tile(L, s, ck, e0, want);
        if (L.err) break;
        uint32_t ns = 0, nv = 0, nr = 0;
        for (uint32_t i = threadIdx.x; i < want; i += NT) {
            int d = L.def[i];
            ns += (ck.max_rep == 0 || d >= ck.repeated_def);
            nv += (d == ck.max_def);
            nr += (L.rep[i] == 0);
        }
        uint32_t t;
        block_excl_scan<NT>(ns, scan_tmp, t); slots += t;
        block_excl_scan<NT>(nr, scan_tmp, t); rows += t;
        block_excl_scan<NT>(nv, scan_tmp, t);
        // dictionary ids of this tile's present values: decode, keep in aux, sum lengths
        if (binary && dict && t > 0) {
            if (threadIdx.x == 0) {
                if (id_bw > 32 || !ck.dict_len) verr = 1;
                else {
                    uint32_t got = rle_walk(sval, s.val, s.val_n, id_bw, t, pval, TILE, npval);
                    if (got != t || sval.err) verr = 1;
                }
            }
            __syncthreads();
            if (verr) break;
            rle_expand<uint32_t>(pval, npval, s.val, s.val_n, id_bw, ids);
            __syncthreads();
            uint64_t acc = 0;
            int bad = 0;
            for (uint32_t i = threadIdx.x; i < t; i += NT) {
                uint32_t id = ids[i];
                if (int64_t(id) >= ck.dict_n) { bad = 1; continue; }
                acc += ck.dict_len[id];
                pg.aux[vals + i] = id;
            }
            if (__syncthreads_or(bad)) { if (threadIdx.x == 0) verr = 1; __syncthreads(); break; }
            atomicAdd(&chars_acc, (unsigned long long)acc);
        }
        vals += t;
        __syncthreads();
    }
    if (L.err || verr) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    if (binary && (pg.encoding == 6 || pg.encoding == 7) && pg.dx) {
        // DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY: lengths decoded by k_dlen (pf_delta.hip)
        if (threadIdx.x == 0) {
            if (int64_t(vals) > pg.dx_total || int64_t(vals) > pg.dx_bad) verr = 1;
            else chars_acc = pg.dx[vals];
        }
        __syncthreads();
        if (verr) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    } else if (binary && !dict) {
        if (pg.encoding != 0 || pg.ba_job < 0) {
            if (threadIdx.x == 0) set_status(res, pg.chunk, ST_ENCODING, pi);
            return;
        }
        if (threadIdx.x == 0) {   // the value chain is walked by the k_ba_* kernels
            BaJob& J = bajobs[pg.ba_job];
            J.p = s.val;
            J.n = uint32_t(min<uint64_t>(s.val_n, J.n_cap));
            J.count = int64_t(vals);
            J.state = vals > 0 ? BA_OK : BA_SKIP;
            chars_acc = 0;
        }
        __syncthreads();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        pg.n_slots = int64_t(slots);
        pg.n_values = int64_t(vals);
        pg.n_rows = int64_t(rows);
        pg.n_chars = int64_t(chars_acc);
    }
}

// Grid-stride over the BYTE_ARRAY / nested pages with a small grid: nearly every page is counted by
// k_count_flat or k_count_seg and skipped here, and a block per page (22 KiB of LDS each) waited for
// CUs held by the other streams' kernels (13-96 us per no-op launch in the r04 kernel trace).
// Grid-stride over a batch's page list for kernels most of whose pages are already done: a block
// tests NT of its pages at once (one round of loads instead of a few dependent loads per page in
// series) and runs `body` only on those `need` accepts, in turn (page order does not matter: each
// page writes its own outputs).
template <typename Need, typename Body>
__device__ __forceinline__ void stride_pages(const int* page_list, int n, Need need, Body body) {
    __shared__ int s_idx[NT];
    __shared__ int s_cnt;
    for (int c0 = 0; int(blockIdx.x) + c0 * int(gridDim.x) < n; c0 += NT) {
        const int i = int(blockIdx.x) + (c0 + int(threadIdx.x)) * int(gridDim.x);
        const int pi = i < n ? page_list[i] : -1;
        const bool w = pi >= 0 && need(pi);
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
        if (w) s_idx[atomicAdd(&s_cnt, 1)] = pi;
        __syncthreads();
        const int m = s_cnt;
        for (int k = 0; k < m; k++) {
            body(s_idx[k]);
            __syncthreads();
        }
        __syncthreads();   // (everyone has read s_cnt before the next round resets it)
    }
}

__global__ __launch_bounds__(NT) void k_count(const DevChunk* __restrict__ chunks, DevPage* pages,
                                              const int* page_list, int n, DevChunkResult* res, BaJob* bajobs) {
    __shared__ CountLds C;
    // (count_page's own early exits, tested for a block's pages at once)
    stride_pages(page_list, n,
                 [&](int pi) { const DevPage& pg = pages[pi]; return (res[pg.chunk].status == 0) & (pg.counted != 1) & (pg.seg_ok != 1); },
                 [&](int pi) { count_page(chunks, pages, pi, res, bajobs, C); });
}

// ---- k_scan (one wave per chunk) ------------------------------------------------------------
__global__ __launch_bounds__(64) void k_scan(DevChunk* chunks, DevPage* pages, const int* chunk_list,
                                             DevChunkResult* res, uint8_t* chars_arena, uint64_t arena_cap,
                                             unsigned long long* arena_used) {
    const int c = chunk_list[blockIdx.x];
    DevChunk& ck = chunks[c];
    const int lane = threadIdx.x;
    // page prefixes: 64 pages' counts loaded at once, wave scans (a serial loop put its loads in series)
    const int np = ck.n_pages, fp = ck.first_page;
    int64_t s = 0, v = 0, r = 0, ch = 0;
    for (int i0 = 0; i0 < np; i0 += 64) {
        const int i = i0 + lane;
        int64_t a[4] = {0, 0, 0, 0};
        if (i < np) { const DevPage& pg = pages[fp + i]; a[0] = pg.n_slots; a[1] = pg.n_values; a[2] = pg.n_rows; a[3] = pg.n_chars; }
        int64_t x[4] = {a[0], a[1], a[2], a[3]};
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            #pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t y = __shfl_up(x[q], d, 64);
                if (lane >= d) x[q] += y;
            }
        }
        if (i < np) {
            DevPage& pg = pages[fp + i];
            pg.slot_start = s + x[0] - a[0]; pg.value_start = v + x[1] - a[1];
            pg.row_start = r + x[2] - a[2]; pg.char_start = ch + x[3] - a[3];
        }
        s += __shfl(x[0], 63, 64); v += __shfl(x[1], 63, 64); r += __shfl(x[2], 63, 64); ch += __shfl(x[3], 63, 64);
    }
    if (lane != 0) return;
    res[c].num_slots = s; res[c].num_values = v; res[c].num_rows = r; res[c].num_chars = ch;
    if (ck.ptype == 6) {
        if (ch > int64_t(0x7fffffff)) { set_status(res, c, ST_CAPACITY, -1); ck.chars = nullptr; }
        else {
            unsigned long long need = (unsigned long long)((ch + 255) & ~int64_t(255));
            unsigned long long at = atomicAdd(arena_used, need);
            if (at + need > arena_cap) { set_status(res, c, ST_CAPACITY, -1); ck.chars = nullptr; }
            else ck.chars = chars_arena + at;
        }
        if (ck.offsets) ck.offsets[0] = 0;
    }
    if (ck.max_rep == 1 && ck.list_offsets) ck.list_offsets[r] = int32_t(s);
}

// Segment path (k_nest_*): the bytes of hybrid stream p[0, n) one segment reads, from the state at
// its first entry (a) to the next segment's (b: the header after the run holding the next segment's
// first entry; null or a sentinel = the stream's end), staged in LDS buffer buf of cap bytes. On
// success p / n become the LDS copy (stream byte lo + i at p[i]; bytes past the staged range read as
// zero but the segment's walk never needs them) and lo is returned: the caller rebases its walk
// state with rle_rebase. Returns 0 and leaves p / n alone when the range does not fit. All threads call.
__device__ __forceinline__ uint64_t stage_seg(uint32_t* buf, uint32_t cap, const uint8_t*& p, uint64_t& n,
                                              const RleState& a, const RleState* b) {
    if (a.err || n == 0 || n > 0xffffffffull) return 0;
    const uint64_t lo = (a.run_packed && a.run_left > 0) ? (a.run_bit >> 3) : a.pos;
    uint64_t hi = (b && !b->err) ? b->pos : n;
    if (lo >= n) return 0;
    hi = min<uint64_t>(n, hi + 16);
    if (hi <= lo || hi - lo + 48 > cap) return 0;
    const uint32_t off = stage_bytes(buf, p, n, uint32_t(lo), uint32_t(hi));
    __syncthreads();
    p = reinterpret_cast<const uint8_t*>(buf) + off;
    n = hi - lo;
    return lo;
}
__device__ __forceinline__ void rle_rebase(RleState& s, uint64_t lo) {
    if (lo == 0) return;
    s.pos -= lo;
    if (s.run_packed && s.run_left > 0) s.run_bit -= 8 * lo;
}

// ---- k_decode ----------------------------------------------------------------------------------
struct DecodeLds {
    LevelLds L;
    Piece pval[TILE];
    uint32_t ids[TILE];
    uint32_t vbits[TILE / 32 + 2];   // validity bits of the tile's slots (relative to aligned base)
    uint32_t lbits[TILE / 32 + 2];   // list validity bits (rows)
    uint32_t scan_tmp[NT / 64];
    RleState sval;
    int npval, verr;
};

template <typename T>
__device__ __forceinline__ void store_w(uint8_t* dst, const uint8_t* src) {
    T v;
    __builtin_memcpy(&v, src, sizeof(T));
    *reinterpret_cast<T*>(dst) = v;
}

// Copy one value of width w from `src` to `dst` (dst is aligned to w for w in {1,4,8}).
__device__ __forceinline__ void copy_value(uint8_t* dst, const uint8_t* src, int w) {
    if (w == 4) { uint32_t v = uint32_t(src[0]) | uint32_t(src[1]) << 8 | uint32_t(src[2]) << 16 | uint32_t(src[3]) << 24; *reinterpret_cast<uint32_t*>(dst) = v; }
    else if (w == 8) {
        uint64_t v = 0;
        #pragma unroll
        for (int k = 0; k < 8; k++) v |= uint64_t(src[k]) << (8 * k);
        *reinterpret_cast<uint64_t*>(dst) = v;
    } else {
        for (int k = 0; k < w; k++) dst[k] = src[k];
    }
}

__device__ __forceinline__ void zero_value(uint8_t* dst, int w) {
    if (w == 4) *reinterpret_cast<uint32_t*>(dst) = 0;
    else if (w == 8) *reinterpret_cast<uint64_t*>(dst) = 0;
    else for (int k = 0; k < w; k++) dst[k] = 0;
}

// Flush a bit array covering bits [b0, b0+nbits) (bit b0 stored at LDS bit (b0 & 31)) to words of
// `out` (bitmap, LSB-first). Edge words use atomicOr (neighbouring pages share them; the output
// bitmap is zeroed before the launch), inner words are plain stores.
__device__ inline void flush_bits(const uint32_t* bits, uint64_t b0, uint32_t nbits, uint8_t* out_bytes) {
    if (nbits == 0) return;
    uint32_t* out = reinterpret_cast<uint32_t*>(out_bytes);
    uint64_t w0 = b0 >> 5, w1 = (b0 + nbits - 1) >> 5;
    for (uint64_t w = w0 + threadIdx.x; w <= w1; w += blockDim.x) {
        uint32_t v = bits[w - w0];
        if (w == w0 || w == w1) { if (v) atomicOr(out + w, v); }
        else out[w] = v;
    }
}

// One segment of a nested page (k_decode_seg): its entries, where its slots / rows / chars / values
// start within the page and the rep, def and value stream states at its first entry.
struct DecodeRange {
    uint64_t e_b, e_e;
    uint64_t slot_base, row_base, char_base, vidx;
    const RleState* st;   // [3], segment-strided (st[k * nseg])
    const RleState* nx;   // the next segment's, or null
    int nseg;
    uint32_t* buf[3];     // LDS for the segment's rep / def / dictionary-id bytes (stage_seg)
};
#ifndef PF_SEG_LVL_CAP
#define PF_SEG_LVL_CAP 4096
#endif
// LDS for one segment's level / dictionary-id bytes (a segment whose bytes do not fit reads them from HBM)
constexpr uint32_t SEG_LVL_CAP = PF_SEG_LVL_CAP, SEG_VAL_CAP = 2 * PF_SEG_LVL_CAP;

__device__ __forceinline__ void decode_page(const DevChunk* __restrict__ chunks, DevPage* pages, const int pi, DevChunkResult* res,
                            DecodeLds& S, const DecodeRange* R = nullptr) {
    LevelLds& L = S.L;
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    if (pg.done != 0 || res[pg.chunk].status != 0) return;   // k_flat[_fixed] took it / an earlier stage failed this chunk
    if (!R && pg.seg_ok == 1) return;                         // k_decode_seg's
    Sections s;
    const bool ok = page_sections(pg, ck, s);
    if (tid == 0) {
        if (R) { L.srep = R->st[0]; L.sdef = R->st[R->nseg]; S.sval = R->st[2 * R->nseg]; }
        else { rle_init(L.srep); rle_init(L.sdef); rle_init(S.sval); }
        L.err = ok ? 0 : 1; S.verr = 0;
    }
    __syncthreads();
    if (L.err) { if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }

    const int enc = pg.encoding;
    const bool binary = ck.ptype == 6;
    const bool dict = is_dict_enc(enc);
    const bool boolean = ck.ptype == 0;
    const int w = ck.width;
    const bool counted = ck.needs_count != 0;
    // value-stream setup
    int id_bw = 0;
    if (dict) {
        id_bw = s.val_n > 0 ? int(s.val[0]) : 0;
        if (tid == 0 && !R) S.sval.pos = 1;
    } else if (boolean && enc == 3) {
        // RLE booleans: 4-byte length prefix, then a bit-width-1 hybrid stream
        if (tid == 0 && !R) S.sval.pos = 0;
    }
    const uint8_t* rle_bool_p = nullptr; uint64_t rle_bool_n = 0;
    if (boolean && enc == 3) {
        uint32_t ln = s.val_n >= 4 ? ld32le(s.val, 0, s.val_n) : 0;
        if (s.val_n < 4 || ln > s.val_n - 4) { if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
        rle_bool_p = s.val + 4; rle_bool_n = ln;
    }
    // encoding / type support check (PLAIN, dictionary, RLE bool, DELTA_BINARY_PACKED ints, BSS)
    bool supported = false;
    if (enc == 0) supported = true;
    else if (dict) supported = !boolean && (binary ? ck.dict_pos != nullptr : ck.dict_data != nullptr);
    else if (enc == 3) supported = boolean;
    else if (enc == 5) supported = (ck.ptype == 1 || ck.ptype == 2) && pg.aux != nullptr;
    else if (enc == 9) supported = (ck.ptype == 4 || ck.ptype == 5);
    else if (enc == 6 || enc == 7) supported = binary && pg.dx != nullptr;   // k_dlen lengths
    if (!supported) { if (tid == 0) set_status(res, pg.chunk, dict ? ST_CORRUPT : ST_ENCODING, pi); return; }
    if (dict && id_bw > 32) { if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    if (binary && !ck.chars) return;   // capacity error already recorded by k_scan
    if (R) {   // the segment's stream bytes in LDS: the walks below read one run header per dependent load
        const int n3 = R->nseg;
        const uint64_t lr = stage_seg(R->buf[0], SEG_LVL_CAP, s.rep, s.rep_n, R->st[0], R->nx ? &R->nx[0] : nullptr);
        const uint64_t ld = ck.max_def > 0 ? stage_seg(R->buf[1], SEG_LVL_CAP, s.def, s.def_n, R->st[n3], R->nx ? &R->nx[n3] : nullptr) : 0;
        const uint64_t lv = (dict && !binary) ? stage_seg(R->buf[2], SEG_VAL_CAP, s.val, s.val_n, R->st[2 * n3], R->nx ? &R->nx[2 * n3] : nullptr) : 0;
        if (tid == 0) { rle_rebase(L.srep, lr); rle_rebase(L.sdef, ld); rle_rebase(S.sval, lv); }
        __syncthreads();
    }

    // bases
    uint64_t slot_base = counted ? uint64_t(pg.slot_start) : uint64_t(pg.entry_start);
    uint64_t row_base = counted ? uint64_t(pg.row_start) : uint64_t(pg.entry_start);
    uint64_t char_base = counted ? uint64_t(pg.char_start) : 0;
    uint64_t vidx = 0;   // page-relative index of the next present value
    const uint64_t bss_total = (enc == 9 && w > 0) ? s.val_n / uint64_t(w) : 0;
    uint64_t e_b = 0, e_e = uint64_t(pg.num_values);
    if (R) {
        e_b = R->e_b; e_e = R->e_e;
        slot_base += R->slot_base; row_base += R->row_base; char_base += R->char_base; vidx = R->vidx;
    }

    for (uint64_t e0 = e_b; e0 < e_e; e0 += TILE) {
        uint32_t want = uint32_t(min<uint64_t>(TILE, e_e - e0));
        decode_level_tile(L, s, ck, e0, want);
        if (L.err) break;
        // per-thread: EPT consecutive entries
        const uint32_t eb = uint32_t(tid) * EPT;
        uint32_t fs = 0, fv = 0, fr = 0;   // bit flags per local entry
        #pragma unroll
        for (int k = 0; k < EPT; k++) {
            uint32_t e = eb + k;
            if (e < want) {
                int d = L.def[e];
                fs |= uint32_t(ck.max_rep == 0 || d >= ck.repeated_def) << k;
                fv |= uint32_t(d == ck.max_def) << k;
                fr |= uint32_t(L.rep[e] == 0) << k;
            }
        }
        uint32_t ts, tv, tr;
        uint32_t so = block_excl_scan<NT>(__popc(fs), S.scan_tmp, ts);
        uint32_t vo = block_excl_scan<NT>(__popc(fv), S.scan_tmp, tv);
        uint32_t ro = block_excl_scan<NT>(__popc(fr), S.scan_tmp, tr);

        // dictionary ids / RLE booleans for this tile's present values
        if ((dict || (boolean && enc == 3)) && tv > 0) {
            if (tid == 0) {
                const uint8_t* vp = dict ? s.val : rle_bool_p;
                uint64_t vn = dict ? s.val_n : rle_bool_n;
                int bw = dict ? id_bw : 1;
                if (binary && dict) S.npval = 0;   // ids were kept by k_count
                else {
                    uint32_t got = rle_walk(S.sval, vp, vn, bw, tv, S.pval, TILE, S.npval);
                    if (got != tv || S.sval.err) S.verr = 1;
                }
            }
            __syncthreads();
            if (S.verr) break;
            if (binary && dict) {
                for (uint32_t i = tid; i < tv; i += NT) S.ids[i] = pg.aux[vidx + i];
            } else {
                rle_expand<uint32_t>(S.pval, S.npval, dict ? s.val : rle_bool_p, dict ? s.val_n : rle_bool_n,
                                     dict ? id_bw : 1, S.ids);
            }
            __syncthreads();
        }
        // BYTE_ARRAY: per-slot lengths -> char offsets (scan over slots in entry order)
        uint32_t my_len[EPT];
        uint64_t my_src[EPT];
        uint32_t lsum = 0;
        if (binary) {
            uint32_t v = vo;
            #pragma unroll
            for (int k = 0; k < EPT; k++) {
                my_len[k] = 0; my_src[k] = 0;
                if ((fv >> k) & 1) {
                    uint64_t gv = vidx + v;
                    if (dict) {
                        uint32_t id = S.ids[v];
                        if (int64_t(id) < ck.dict_n) { my_src[k] = ck.dict_pos[id]; my_len[k] = ck.dict_len[id]; }
                        else S.verr = 1;
                    } else if (enc == 6 || enc == 7) {   // cpos: chars before value gv (checked by k_count)
                        my_src[k] = uint64_t(pg.dx_data) + pg.dx[gv];
                        my_len[k] = uint32_t(pg.dx[gv + 1] - pg.dx[gv]);
                    } else {
                        uint32_t p = pg.aux[gv];
                        uint32_t l = (p >= 4 && p <= s.val_n) ? ld32le(s.val, p - 4, s.val_n) : 0xffffffffu;
                        if (l <= s.val_n - p) { my_src[k] = p; my_len[k] = l; }
                        else S.verr = 1;
                    }
                    v++;
                }
                lsum += my_len[k];
            }
        }
        uint32_t tchars = 0;
        uint32_t lo = binary ? block_excl_scan<NT>(lsum, S.scan_tmp, tchars) : 0;
        if (binary && (S.verr || char_base + tchars > uint64_t(pg.char_start + pg.n_chars))) {
            S.verr = 1;   // inconsistent with k_count's sizing: never write past this page's chars
            break;
        }

        // validity / list-validity bit staging
        const uint64_t vb0 = slot_base + 0;      // first slot of this tile
        for (uint32_t i = tid; i < TILE / 32 + 2; i += NT) { S.vbits[i] = 0; S.lbits[i] = 0; }
        __syncthreads();

        // per-entry writes
        {
            uint32_t sidx = so, vv = vo, ridx = ro;
            uint64_t cpos = char_base + lo;
            #pragma unroll
            for (int k = 0; k < EPT; k++) {
                uint32_t e = eb + k;
                if (e >= want) break;
                const bool is_slot = (fs >> k) & 1, present = (fv >> k) & 1, rstart = (fr >> k) & 1;
                if (ck.max_rep > 0) {
                    uint64_t ge = uint64_t(pg.entry_start) + e0 + e;
                    if (ck.def_levels) ck.def_levels[ge] = L.def[e];
                    if (ck.rep_levels) ck.rep_levels[ge] = L.rep[e];
                    if (rstart && ck.max_rep == 1) {
                        uint64_t row = row_base + ridx;
                        if (ck.list_offsets) ck.list_offsets[row] = int32_t(slot_base + sidx);
                        if (L.def[e] >= ck.list_null_def) {
                            uint64_t rb = row - (row_base & ~uint64_t(31));
                            atomicOr(&S.lbits[rb >> 5], 1u << (rb & 31));
                        }
                    }
                }
                if (rstart) ridx++;
                if (!is_slot) continue;
                const uint64_t slot = slot_base + sidx;
                if (present && ck.max_def > 0) {
                    uint64_t rb = slot - (vb0 & ~uint64_t(31));
                    atomicOr(&S.vbits[rb >> 5], 1u << (rb & 31));
                }
                if (binary) {
                    if (present) {
                        const uint8_t* src = dict ? ck.dict_data + my_src[k] : s.val + my_src[k];
                        if (enc != 7)   // DELTA_BYTE_ARRAY chars: k_dba_chars (values depend on their predecessor)
                            for (uint32_t j = 0; j < my_len[k]; j++) ck.chars[cpos + j] = src[j];
                        cpos += my_len[k];
                    }
                    ck.offsets[slot + 1] = int32_t(cpos);
                } else if (present) {
                    const uint64_t gv = vidx + vv;
                    uint8_t* dst = ck.values + slot * uint64_t(w);
                    if (dict) {
                        uint32_t id = S.ids[vv];
                        if (int64_t(id) >= ck.dict_n) { S.verr = 1; }
                        else copy_value(dst, ck.dict_data + uint64_t(id) * w, w);
                    } else if (boolean) {
                        uint32_t b = (enc == 3) ? S.ids[vv] : ((ld8(s.val, gv >> 3, s.val_n) >> (gv & 7)) & 1);
                        if (enc == 0 && (gv >> 3) >= s.val_n) S.verr = 1;
                        dst[0] = uint8_t(b);
                    } else if (enc == 0) {
                        if ((gv + 1) * uint64_t(w) > s.val_n) S.verr = 1;
                        else copy_value(dst, s.val + gv * w, w);
                    } else if (enc == 5) {
                        const uint64_t* dv = reinterpret_cast<const uint64_t*>(pg.aux);
                        if (w == 8) *reinterpret_cast<uint64_t*>(dst) = dv[gv];
                        else *reinterpret_cast<uint32_t*>(dst) = uint32_t(dv[gv]);
                    } else if (enc == 9) {
                        if (gv >= bss_total) S.verr = 1;
                        else for (int b = 0; b < w; b++) dst[b] = s.val[uint64_t(b) * bss_total + gv];
                    }
                } else {
                    zero_value(ck.values + slot * uint64_t(w), w);
                }
                if (present) vv++;
                sidx++;
            }
        }
        __syncthreads();
        if (S.verr) break;
        if (ck.max_def > 0 && ck.validity) flush_bits(S.vbits, vb0, ts, ck.validity);
        if (ck.max_rep == 1 && ck.list_validity) flush_bits(S.lbits, row_base, tr, ck.list_validity);
        slot_base += ts;
        row_base += tr;
        char_base += tchars;
        vidx += tv;
        __syncthreads();
    }
    if (L.err || S.verr) { if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    if (!counted && tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&res[pg.chunk].num_values),
                                        (unsigned long long)vidx);
}

// Pages the flat kernels did not take (nested, DELTA_LENGTH / DELTA_BYTE_ARRAY, RLE booleans, BSS,
// anything they rejected). Grid-stride over the batch's page list with a grid sized by the host to
// the pages that will need it (listed first): most blocks find their pages done, and a launch of
// one large-LDS block per page would wait for CUs that other streams' kernels hold.
__global__ __launch_bounds__(NT) void k_decode(const DevChunk* __restrict__ chunks, DevPage* pages,
                                               const int* page_list, int n, DevChunkResult* res) {
    __shared__ DecodeLds S;
    // (decode_page's own early exits, tested for a block's pages at once)
    stride_pages(page_list, n,
                 [&](int pi) { const DevPage& pg = pages[pi]; return (pg.done == 0) & (pg.seg_ok != 1) & (res[pg.chunk].status == 0); },
                 [&](int pi) { decode_page(chunks, pages, pi, res, S); });
}

// ---- k_flat: data pages of flat columns (max_rep == 0) ------------------------------------------
// The same per-value work as k_decode, organised for throughput. The definition-level and
// dictionary-id run headers of the page are walked ONCE (one lane of wave 0 and one of wave 1,
// concurrently) into LDS run tables; tiles of FT entries then expand them by binary search with no
// serial section, one workgroup scan for the value index (none when the page has no nulls) and one
// for BYTE_ARRAY char offsets. BYTE_ARRAY chars are copied cooperatively, one 16-byte output chunk
// per thread step (coalesced stores), instead of a byte loop per value.
// Pages it does not take (run tables full, BIT_PACKED levels, RLE booleans, BYTE_STREAM_SPLIT,
// corrupt section layout) keep done == 0 and are decoded by k_decode.
#ifndef PF_FT
#define PF_FT 2048   // r04 (string path; the fixed-width path has FTX): SF1 2.896-2.899 vs 2.938-2.953 ms with
                     // 1024 (profiles/r04_ab/tune.txt). r02, one tile size for both paths: 1024 beat 2048 (3.82 vs 3.94)
#endif
constexpr int FT = PF_FT;            // entries per tile (fewer registers per thread, more blocks resident)
constexpr int FEPT = FT / NT;        // consecutive entries per thread
static_assert(FT <= int(FBLK) && FBLK % FT == 0 && FEPT <= 32, "tiles divide blocks; a thread's entries fit a 32-bit mask");
#ifndef PF_FTX
#define PF_FTX 2048   // SF1 2.936 / 2.936 ms vs 3.000-3.019 with 1024 (4096: 2.93, scratch for the arrays)
#endif
constexpr int FTX = PF_FTX;          // tile of the all-present fixed-width path (flat_present_fixed): its
                                     // tiles' id loads and gathers per thread in flight together
constexpr int FEPTX = FTX / NT;
static_assert(FTX <= int(FBLK) && FBLK % FTX == 0, "fixed-width tiles divide blocks");
#ifndef PF_RUN_CAP
#define PF_RUN_CAP 256
#endif
constexpr int RUN_CAP = PF_RUN_CAP;

struct Run {
    uint32_t first;    // index of the first value the run covers (entries for levels)
    uint32_t count;
    uint32_t data;     // RLE value, or absolute bit offset of the run's packed values
    uint32_t packed;
};

// Walk RLE/bit-packed hybrid run headers of p[0..n) (parquet-mr RunLengthBitPackingHybridDecoder)
// from the walker state (pos = next header, first = index of its first value) until `limit`
// values are covered. Runs that end at or before `lo` are skipped, the others are stored. Returns
// 0 covered (covered = limit), 1 stream ended or corrupt first, 2 table full (covered = end of the
// last stored run; the state points after it).
struct RunWalk {
    uint64_t pos;
    uint32_t first;
};

__device__ int walk_runs(const uint8_t* p, uint64_t n, int bw, uint32_t lo, uint32_t limit, Run* runs, int cap,
                         int& nruns, uint32_t& covered, RunWalk& st) {
    nruns = 0;
    covered = st.first;
    while (st.first < limit) {
        uint64_t pos = st.pos, h;
        if (!uvarint(p, n, pos, h)) return 1;
        Run r;
        uint64_t cnt;
        if (h & 1) {
            cnt = (h >> 1) * 8;
            const uint64_t nb = (h >> 1) * uint64_t(bw);
            r.data = uint32_t(pos * 8);
            r.packed = 1;
            pos += nb < n - pos ? nb : n - pos;   // truncated to what is left (zero-padded)
        } else {
            cnt = h >> 1;
            const int nbv = (bw + 7) >> 3;
            if (pos + nbv > n) return 1;
            uint32_t v = 0;
            for (int b = 0; b < nbv; b++) v |= uint32_t(p[pos + b]) << (8 * b);
            pos += nbv;
            r.data = v;
            r.packed = 0;
        }
        if (cnt == 0) { st.pos = pos; continue; }
        const uint32_t c = uint32_t(cnt < uint64_t(limit - st.first) ? cnt : uint64_t(limit - st.first));
        if (st.first + c > lo) {
            if (nruns == cap) return 2;
            r.first = st.first;
            r.count = c;
            runs[nruns++] = r;
            covered = st.first + c;
        } else {
            covered = st.first + c;
        }
        st.pos = pos;
        st.first += c;
    }
    return 0;
}

// ---- wave-parallel run discovery (north_star K2: run boundaries found by wavefront scans) ------
//
// The run headers of an RLE/bit-packed hybrid stream form a chain (each header's position follows
// from the previous run's length), and writers emit long stretches of identical headers: Arrow and
// parquet-mr cut bit-packed runs at 512 values (header 0x81 0x01), so a page of random dictionary
// ids or levels is ~40 runs with one byte stride. One round: every lane decodes the header at
// pos (the chain position, exact), then lane i decodes the header at pos + i * stride and votes
// whether it repeats lane 0's; the ballot's first failing lane ends the accepted prefix, and a
// prefix scan of the (equal) run lengths gives every accepted run's first value. A stretch of k
// equal runs costs one round instead of k dependent header loads; mixed runs still advance by
// one run per round. Called by all 64 lanes of one wave with wave-uniform arguments.
struct WaveRun {
    uint64_t pos;        // header position (uniform)
    uint32_t first;      // first value of the run at pos (uniform)
};
constexpr int WAVE_SERIAL_RUNS = 8;   // after a prediction fails at lane 1: this many runs without predicting

template <class Src>
__device__ __forceinline__ bool hdr_decode(const Src& B, uint64_t n, uint64_t p, int bw, uint64_t& h, uint32_t& hl,
                                           uint32_t& val) {
    h = 0;
    hl = 0;
    val = 0;
    #pragma unroll
    for (int k = 0; k < 5; k++) {
        if (p + uint64_t(k) >= n) return false;
        const uint32_t c = B(p + uint64_t(k));
        h |= uint64_t(c & 0x7fu) << (7 * k);
        if (!(c & 0x80u)) { hl = uint32_t(k) + 1u; break; }
    }
    if (hl == 0) return false;   // headers above 2^35 are not runs of a page
    if (!(h & 1)) {
        const uint32_t nbv = uint32_t(bw + 7) >> 3;
        if (p + hl + nbv > n) return false;
        for (uint32_t b = 0; b < nbv; b++) val |= uint32_t(B(p + hl + b)) << (8 * b);
    }
    return true;
}

// One discovery round from st (uniform). Returns the accepted runs k (lanes < k hold run `r`,
// with its count clipped at `limit`), 0 when the header at st.pos is an empty run (skipped), -1
// when the stream ends or is corrupt there. st advances past the accepted runs.
// spec = false: only the run at st.pos (no prediction; used after a round the prediction failed at
// lane 1, so streams of mixed runs cost one header decode per run instead of 64).
template <class Src>
__device__ int wave_run_round(const Src& B, uint64_t n, int bw, uint32_t limit, WaveRun& st, Run& r, bool& trunc,
                              bool spec = true) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t h0;
    uint32_t hl0, v0;
    if (!hdr_decode(B, n, st.pos, bw, h0, hl0, v0)) return -1;
    const bool packed = h0 & 1;
    const uint64_t cnt0 = packed ? (h0 >> 1) * 8 : (h0 >> 1);
    const uint64_t pay0 = packed ? (h0 >> 1) * uint64_t(bw) : uint64_t(uint32_t(bw + 7) >> 3);
    if (cnt0 == 0) {
        st.pos += hl0 + (packed ? 0 : pay0);
        return 0;
    }
    const uint64_t stride = uint64_t(hl0) + pay0;
    // lane i: the i-th run from st.pos, if the headers repeat
    const uint64_t p = st.pos + uint64_t(lane) * stride;
    bool ok = true;
    uint32_t v = v0;
    if (lane > 0) {
        uint64_t h;
        uint32_t hl;
        ok = spec && hdr_decode(B, n, p, bw, h, hl, v) && h == h0 && hl == hl0 && (!packed || p + hl + pay0 <= n);
    }
    const uint64_t fail = __ballot(!ok);
    uint32_t k = fail ? uint32_t(__ffsll((unsigned long long)fail) - 1) : 64u;
    // runs needed to reach `limit` (the last one clipped)
    const uint64_t left = uint64_t(limit - st.first);
    const uint64_t need = (left + cnt0 - 1) / cnt0;
    if (uint64_t(k) > need) k = uint32_t(need);
    const uint64_t f = uint64_t(st.first) + uint64_t(lane) * cnt0;
    r.first = uint32_t(f);
    r.count = uint32_t(min<uint64_t>(cnt0, f < limit ? uint64_t(limit) - f : 0));
    r.packed = packed ? 1u : 0u;
    r.data = packed ? uint32_t((p + hl0) * 8) : v;
    // a truncated final bit-packed run (lane 0 only: the others required the whole payload)
    uint64_t adv = uint64_t(k) * stride;
    trunc = packed && st.pos + stride > n;
    if (trunc) adv = n - st.pos;
    st.pos += adv;
    st.first = uint32_t(min<uint64_t>(uint64_t(st.first) + uint64_t(k) * cnt0, uint64_t(limit)));
    return int(k);
}

// walk_runs for a whole wave from state st0 (same contract; runs / nruns / covered / the final state
// are written by lane 0 or by the lanes holding the runs). All 64 lanes call it. The start state is
// a value, not shared memory: one lane's store to LDS is not ordered before the other lanes' loads
// without a barrier.
__device__ int wave_walk_runs(const uint8_t* p, uint64_t n, int bw, uint32_t lo, uint32_t limit, Run* runs, int cap,
                              int& nruns_out, uint32_t& covered_out, RunWalk& stw, RunWalk st0) {
    const uint32_t lane = threadIdx.x & 63u;
    const auto B = [p](uint64_t i) { return uint32_t(p[i]); };
    WaveRun st{st0.pos, st0.first};
    int nr = 0, ret = 0;
    uint32_t covered = st.first;
    int serial = 0;   // runs left to take one at a time after a failed prediction
    while (st.first < limit) {
        Run r;
        const uint64_t pos0 = st.pos;
        const uint32_t f0 = st.first;
        bool trunc;
        const int k = wave_run_round(B, n, bw, limit, st, r, trunc, serial == 0);
        if (k < 0) { ret = 1; break; }
        if (k == 0) continue;
        serial = serial > 0 ? serial - 1 : (k == 1 && st.first < limit ? WAVE_SERIAL_RUNS : 0);
        // stored: runs ending after lo (a prefix of the round's runs ends at or before lo)
        const bool keep = lane < uint32_t(k) && r.first + r.count > lo;
        const uint64_t km = __ballot(keep);
        const int nk = __popcll(km);
        const int rank = __popcll(km & ((1ull << lane) - 1ull));
        if (nr + nk > cap) {   // table full: store what fits, stop after the last stored run
            const int room = cap - nr;
            if (keep && rank < room) runs[nr + rank] = r;
            // the round's runs up to the last stored one: lanes [0, first kept lane + room)
            const uint32_t upto = uint32_t(__ffsll((unsigned long long)km) - 1) + uint32_t(room);
            const uint64_t stride = (st.pos - pos0) / uint64_t(k);
            st.pos = pos0 + uint64_t(upto) * stride;
            st.first = f0 + (upto ? __shfl(r.first + r.count, int(upto) - 1, 64) - f0 : 0u);
            covered = st.first;
            nr = cap;
            ret = 2;
            break;
        }
        if (keep) runs[nr + rank] = r;
        nr += nk;
        covered = st.first;
    }
    if (lane == 0) {
        nruns_out = nr;
        covered_out = covered;
        stw.pos = st.pos;
        stw.first = st.first;
    }
    return ret;
}

// Definition levels of p[0..n): 1 if every one of the `ne` levels is max_def (RLE runs only),
// 0 otherwise (or corrupt: the single-workgroup path reports it).
__device__ int all_present(const uint8_t* p, uint64_t n, int bw, uint32_t ne, uint32_t max_def) {
    uint64_t pos = 0;
    uint32_t covered = 0;
    while (covered < ne) {
        uint64_t h;
        if (!uvarint(p, n, pos, h)) return 0;
        if (h & 1) return 0;
        const int nbv = (bw + 7) >> 3;
        if (pos + nbv > n) return 0;
        uint32_t v = 0;
        for (int b = 0; b < nbv; b++) v |= uint32_t(p[pos + b]) << (8 * b);
        pos += nbv;
        if ((h >> 1) == 0) continue;
        if (v != max_def) return 0;
        covered += uint32_t(min<uint64_t>(h >> 1, uint64_t(ne - covered)));
    }
    return 1;
}

// Unaligned loads from global memory as aligned dwords + v_alignbyte (the dwords covering
// [p, p + 4 or 8) plus up to 3 following bytes must be readable).
__device__ __forceinline__ uint32_t ld_u32_any(const uint8_t* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3u);
    if (!sh) return q[0];
    return __builtin_amdgcn_alignbyte(q[1], q[0], sh);   // byte shift
}
__device__ __forceinline__ uint64_t ld_u64_any(const uint8_t* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3u);
    const uint32_t d0 = q[0], d1 = q[1];
    if (!sh) return uint64_t(d0) | (uint64_t(d1) << 32);
    const uint32_t d2 = q[2];
    return uint64_t(__builtin_amdgcn_alignbyte(d1, d0, sh)) | (uint64_t(__builtin_amdgcn_alignbyte(d2, d1, sh)) << 32);
}
__device__ __forceinline__ uint64_t ld64_bytes(const uint8_t* p) {
    uint64_t v = 0;
    #pragma unroll
    for (int k = 0; k < 8; k++) v |= uint64_t(p[k]) << (8 * k);
    return v;
}
// LSB-first bit field of width w <= 32 starting at bit `sh` (< 8) of p (12 bytes readable from p).
// Branch-free unaligned loads from global memory for callers that guarantee the extra readable
// bytes: all dwords are loaded unconditionally (no per-lane branch on the alignment, so a thread's
// loads of several values stay in flight together) and joined with v_alignbyte (shift 0 = dword).
__device__ __forceinline__ uint32_t gld_u32_8(const uint8_t* p) {   // p + 8 readable
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const PF_GLOBAL uint32_t* q = (const PF_GLOBAL uint32_t*)(a & ~uintptr_t(3));
    return __builtin_amdgcn_alignbyte(q[1], q[0], uint32_t(a & 3u));
}
__device__ __forceinline__ uint64_t gld_u64_12(const uint8_t* p) {   // p + 12 readable
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const PF_GLOBAL uint32_t* q = (const PF_GLOBAL uint32_t*)(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3u), d0 = q[0], d1 = q[1], d2 = q[2];
    return uint64_t(__builtin_amdgcn_alignbyte(d1, d0, sh)) | (uint64_t(__builtin_amdgcn_alignbyte(d2, d1, sh)) << 32);
}
__device__ __forceinline__ uint32_t bits_fast(const uint8_t* p, uint32_t sh, int w) {   // p + 12 readable
    const uint64_t v = gld_u64_12(p) >> sh;
    return uint32_t(v & (w == 32 ? 0xffffffffull : ((1ull << w) - 1ull)));
}

// Index of the run holding value i (runs sorted by `first`, runs[0].first == 0).
__device__ __forceinline__ int run_find(const Run* runs, int nr, uint32_t i) {
    int lo = 0, hi = nr;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (runs[mid].first <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t run_value(const Run& r, const uint8_t* p, uint64_t n, uint32_t i, int bw) {
    return r.packed ? bits_le(p, n, uint64_t(r.data) + uint64_t(i - r.first) * uint64_t(bw), bw) : r.data;
}

// One 128-thread workgroup per dictionary data page of a flat chunk: walks the page's
// dictionary-id run headers ONCE (wave 1) and checks whether every definition level is present
// (wave 0), so that k_flat's blocks of the page load a ready run table instead of each walking
// the headers from the page start.
__global__ __launch_bounds__(128) void k_runs(const DevChunk* __restrict__ chunks, DevPage* pages,
                                              const int* __restrict__ list, DevChunkResult* res) {
    __shared__ Run R[RUN_CAP];
    __shared__ int s_allp, s_nr, s_res;
    __shared__ uint32_t s_cov;
    const int pi = list[blockIdx.x];
    DevPage& pg = pages[pi];
    uint32_t* T = pg.runtab;
    if (!T) return;
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    Sections s;
    if (res[pg.chunk].status != 0 || !page_sections(pg, ck, s) || s.val_n == 0 || s.val[0] > 32) {
        if (tid == 0) T[3] = 0;
        return;
    }
    const uint32_t ne = uint32_t(pg.num_values);
    const int id_bw = int(s.val[0]);
    if (tid == 0) {
        s_allp = ck.max_def == 0 ? 1 : (s.def_rle ? all_present(s.def, s.def_n, bit_width(ck.max_def), ne, uint32_t(ck.max_def)) : 0);
    } else if (tid >= 64) {   // wave 1: the id runs, discovered wave-parallel
        __shared__ RunWalk s_st;
        int nr = 0;
        uint32_t cov = 0;
        const int rr = wave_walk_runs(s.val + 1, s.val_n - 1, id_bw, 0, ne, R, RUN_CAP, nr, cov, s_st, RunWalk{0, 0});
        if (tid == 64) { s_res = rr; s_nr = nr; s_cov = cov; }
    }
    __syncthreads();
    const int nr = s_nr;
    if (s_res == 2) {   // too many runs for the table: blocks walk themselves
        if (tid == 0) { T[2] = 0; T[3] = 0; }
        return;
    }
    for (int i = tid; i < nr; i += 128) {
        T[4 + 2 * i] = R[i].first | (R[i].packed << 31);
        T[5 + 2 * i] = R[i].data;
    }
    // T[2]: the id table is valid (indexed by value: pages with nulls hold fewer ids than entries, the
    // walk then ends with the stream); T[3]: valid and every level present (k_flat_fixed / k_flat split)
    if (tid == 0) { T[0] = uint32_t(nr); T[1] = s_cov; T[2] = 1u; T[3] = s_allp ? 1u : 0u; }
}

// Dictionary-string pages k_count_flat takes: flat, levels all present (k_runs: T[3]), a run table.
__device__ __forceinline__ bool count_dict_page(const DevPage& pg, const DevChunk& ck, const Sections& s) {
    const uint32_t* T = pg.runtab;
    return T != nullptr && T[3] == 1u && T[0] <= uint32_t(RUN_CAP) && T[1] >= uint32_t(pg.num_values) && ck.dict_len &&
           s.val_n > 0 && flat_block_chars(pg) != nullptr;
}
constexpr uint64_t BC_BAD = ~0ull;   // a block's chars word when one of its ids is out of the dictionary

// k_count_dict (round 5): the chars of one 4096-entry block of a flat dictionary BYTE_ARRAY page per
// workgroup -- the block's ids from the page's run table (k_runs), their dictionary lengths summed --
// into the page's per-block chars word bc[block]; k_count_flat scans those words into the blocks'
// chars bases and the page's chars. (Round 4 summed a page's blocks one after another in
// k_count_flat's one workgroup per page: SF1's pages of ~1M entries were 256 dependent rounds.)
__global__ __launch_bounds__(NT) void k_count_dict(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                   const int2* __restrict__ blocks, DevChunkResult* res) {
    __shared__ Run R[RUN_CAP];
    __shared__ uint32_t s_len[DSTR_CAP];   // lengths of small dictionaries
    __shared__ unsigned long long s_acc;
    const int2 pb = blocks[blockIdx.x];
    DevPage& pg = pages[pb.x];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    if (res[pg.chunk].status != 0 || ck.max_rep != 0 || ck.ptype != 6 || !is_dict_enc(pg.encoding)) return;
    Sections s;
    if (!page_sections(pg, ck, s) || !count_dict_page(pg, ck, s)) return;
    const uint32_t ne = uint32_t(pg.num_values);
    const uint32_t b0 = uint32_t(pb.y) * FBLK;
    if (pb.y > 0 && b0 >= ne) return;
    const uint32_t b1 = min(ne, b0 + FBLK);
    const uint32_t* T = pg.runtab;
    const uint32_t nr = T[0], cov = T[1];
    for (uint32_t i = tid; i < nr; i += NT) {
        const uint32_t f = T[4 + 2 * i];
        const uint32_t nf = i + 1 < nr ? (T[4 + 2 * (i + 1)] & 0x7fffffffu) : cov;
        Run r;
        r.first = f & 0x7fffffffu;
        r.count = nf - r.first;
        r.data = T[5 + 2 * i];
        r.packed = f >> 31;
        R[i] = r;
    }
    const bool lstage = ck.dict_n > 0 && ck.dict_n <= int64_t(DSTR_CAP);
    if (lstage)
        for (uint32_t i = tid; i < uint32_t(ck.dict_n); i += NT) s_len[i] = gptr(ck.dict_len)[i];
    if (tid == 0) s_acc = 0;
    __syncthreads();
    const uint8_t* ids = s.val + 1;
    const uint64_t ids_n = s.val_n - 1;
    const int id_bw = int(s.val[0]);
    constexpr int EPB = int(FBLK) / NT;   // entries of the block per thread
    int bad = 0;
    uint64_t acc = 0;
    // ids of the thread's EPB entries first (their loads in flight together), then the lengths
    uint32_t idk[EPB];
    int r = -1;
    #pragma unroll
    for (int k = 0; k < EPB; k++) {
        const uint32_t e = b0 + uint32_t(k) * NT + uint32_t(tid);
        idk[k] = 0xffffffffu;
        if (e >= b1) continue;
        if (r < 0) r = run_find(R, int(nr), e);
        while (e >= R[r].first + R[r].count) r++;
        const Run& Rr = R[r];
        uint32_t id = Rr.data;
        if (Rr.packed) {
            const uint64_t bit = uint64_t(Rr.data) + uint64_t(e - Rr.first) * uint64_t(id_bw);
            id = (bit >> 3) + 12 <= ids_n ? bits_fast(ids + (bit >> 3), uint32_t(bit & 7), id_bw)
                                          : bits_le(ids, ids_n, bit, id_bw);
        }
        if (int64_t(id) >= ck.dict_n) { bad = 1; continue; }
        idk[k] = id;
    }
    #pragma unroll
    for (int k = 0; k < EPB; k++)
        if (idk[k] != 0xffffffffu) acc += lstage ? s_len[idk[k]] : gptr(ck.dict_len)[idk[k]];
    if (acc) atomicAdd(&s_acc, (unsigned long long)acc);
    bad = __syncthreads_or(bad);
    if (tid == 0) flat_block_chars(pg)[pb.y] = bad ? BC_BAD : uint64_t(s_acc);
}

// k_count for flat BYTE_ARRAY pages whose levels are all present: slots = rows = values =
// entries; dictionary strings scan k_count_dict's per-block chars (k_flat's per-block chars bases,
// the page's chars); PLAIN pages hand their value chain to the k_ba walk. Marks the page counted
// (pg.counted) so k_count skips it; pages it leaves alone (nulls, corrupt) go through k_count.
__global__ __launch_bounds__(NT) void k_count_flat(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                   const int* __restrict__ page_list, DevChunkResult* res,
                                                   BaJob* bajobs) {
    __shared__ int s_ok;
    __shared__ unsigned long long s_scan[NT / 64];
    const int pi = page_list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    if (res[pg.chunk].status != 0 || ck.max_rep != 0 || ck.ptype != 6) return;
    Sections s;
    if (!page_sections(pg, ck, s)) return;
    const bool dict = is_dict_enc(pg.encoding);
    const uint32_t ne = uint32_t(pg.num_values);
    uint64_t total = 0;
    if (dict) {
        if (!count_dict_page(pg, ck, s)) return;
        // k_count_dict's block sums -> exclusive bases in place (a page of 1M entries: 256 words)
        uint64_t* bc = flat_block_chars(pg);
        const uint32_t nb = (ne + FBLK - 1) / FBLK;
        int bad = 0;
        for (uint32_t b = 0; b < nb; b += NT) {
            const uint32_t i = b + uint32_t(tid);
            uint64_t v = i < nb ? bc[i] : 0ull;
            if (v == BC_BAD) { bad = 1; v = 0; }
            uint64_t tot;
            const uint64_t ex = block_excl_scan64<NT>(v, s_scan, tot);
            if (i < nb) bc[i] = total + ex;
            total += tot;
        }
        if (__syncthreads_or(bad)) return;   // k_count reports the bad id
    } else {
        if (pg.encoding != 0 || pg.ba_job < 0) return;
        if (tid == 0)
            s_ok = ck.max_def == 0 ? 1
                                   : (s.def_rle ? all_present(s.def, s.def_n, bit_width(ck.max_def), ne, uint32_t(ck.max_def)) : 0);
        __syncthreads();
        if (!s_ok) return;
        if (tid == 0) {   // the value chain is walked by the k_ba_* kernels
            BaJob& J = bajobs[pg.ba_job];
            J.p = s.val;
            J.n = uint32_t(min<uint64_t>(s.val_n, J.n_cap));
            J.count = int64_t(ne);
            J.state = ne > 0 ? BA_OK : BA_SKIP;
        }
    }
    if (tid == 0) {
        pg.n_slots = int64_t(ne);
        pg.n_values = int64_t(ne);
        pg.n_rows = int64_t(ne);
        pg.n_chars = int64_t(total);
        pg.counted = 1;
    }
}

// One 16-byte output chunk at arena address c (tile chars start at a0, total bytes): chunks inside
// one value are one 16-byte source read (aligned dwords + v_alignbyte); a chunk spanning values is
// blended from one aligned window per value piece. v: a value at or before the chunk's first byte.
__device__ __forceinline__ void copy_chunk16(const uint32_t* coff, const uint32_t* csrc, uint32_t nv, uint32_t total,
                                    const uint8_t* sbase, const uint8_t* send, uintptr_t a0, uintptr_t c, uint32_t v) {
    const int64_t r0 = int64_t(c) - int64_t(a0);
    uint32_t vb = coff[v];
    uint32_t vend = v + 1 < nv ? coff[v + 1] : total;
    while (r0 >= 0 && uint32_t(r0) >= vend && v + 1 < nv) {   // zero-length values share a start
        v++;
        vb = coff[v];
        vend = v + 1 < nv ? coff[v + 1] : total;
    }
    uint8_t* dst = reinterpret_cast<uint8_t*>(c);
    if (r0 >= 0 && uint32_t(r0) >= vb && uint64_t(r0) + 16 <= vend) {
        const uint8_t* sp = sbase + csrc[v] + (uint32_t(r0) - vb);
        if (sp + 20 <= send) {
            const uintptr_t sa = reinterpret_cast<uintptr_t>(sp);
            const uint32_t* q = reinterpret_cast<const uint32_t*>(sa & ~uintptr_t(3));
            const uint32_t sh = uint32_t(sa & 3u);
            uint32_t d[5];
            #pragma unroll
            for (int k = 0; k < 5; k++) d[k] = q[k];
            uint4 o;
            if (sh) {
                o.x = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
                o.y = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
                o.z = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
                o.w = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
            } else {
                o = make_uint4(d[0], d[1], d[2], d[3]);
            }
            *reinterpret_cast<uint4*>(dst) = o;
            return;
        }
    }
    // the chunk spans values: one aligned 16-byte window per value piece, blended under a byte mask
    // (dword loads that overlap the piece's source bytes only, so every load stays in the source)
    uint32_t word[4] = {0, 0, 0, 0};
    for (;;) {
        const int64_t lo = max(max(r0, int64_t(vb)), int64_t(0)), hi = min(min(r0 + 16, int64_t(vend)), int64_t(total));
        if (lo < hi) {
            const uintptr_t need0 = reinterpret_cast<uintptr_t>(sbase) + csrc[v] + uint32_t(lo - vb);
            const uintptr_t need1 = need0 + uintptr_t(hi - lo);            // source bytes [need0, need1)
            const uintptr_t ws = need0 - uintptr_t(lo - r0);               // source of chunk byte 0
            const uintptr_t wa = ws & ~uintptr_t(3);
            const uint32_t sh = uint32_t(ws & 3u);
            uint32_t d[5];
            #pragma unroll
            for (int k = 0; k < 5; k++) {
                const uintptr_t da = wa + 4u * k;
                d[k] = (da + 4 > need0 && da < need1) ? *reinterpret_cast<const uint32_t*>(da) : 0u;
            }
            const uint32_t bm = (0xffffu >> (16 - uint32_t(hi - r0))) & ~((1u << uint32_t(lo - r0)) - 1u);
            #pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t w = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
                const uint32_t m = (((bm >> (4 * k)) & 0xfu) * 0x00204081u & 0x01010101u) * 0xffu;
                word[k] = (word[k] & ~m) | (w & m);
            }
        }
        if (int64_t(vend) >= r0 + 16 || v + 1 >= nv) break;
        v++;
        vb = coff[v];
        vend = v + 1 < nv ? coff[v + 1] : total;
    }
    if (r0 >= 0 && r0 + 16 <= int64_t(total)) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(word[0], word[1], word[2], word[3]);
    } else {
        #pragma unroll
        for (int k = 0; k < 16; k++) {
            const int64_t r = r0 + k;
            if (r >= 0 && r < int64_t(total)) dst[k] = uint8_t(word[k >> 2] >> (8 * (k & 3)));
        }
    }
}

// Chars copy with a chunk -> value table (no per-chunk binary search) and 16-byte source reads
// (aligned dwords + v_alignbyte) for chunks inside one value; other chunks blended per value piece.
// cv: LDS table of CV_CAP u16; send: end of the readable source buffer.
constexpr uint32_t CV_CAP = 2048;   // (round 5: 4096 -> 2048 brought k_flat_all under 32 KiB of LDS, five workgroups per CU)
__device__ __forceinline__ void copy_chars_fast(const uint32_t* coff, const uint32_t* csrc, uint32_t nv, uint32_t total,
                                       const uint8_t* sbase, const uint8_t* send, uint8_t* obase, uint16_t* cv) {
    if (total == 0 || nv == 0) return;
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(obase);
    const uintptr_t c0 = a0 & ~uintptr_t(15);
    const uint32_t nch = uint32_t(((a0 + total + 15) & ~uintptr_t(15)) - c0) / 16u;
    // value v owns the chunks whose first byte lies inside it (chunk 0 may start before the tile: 0);
    // tiles of more than CV_CAP chunks in passes of CV_CAP (round 5: the per-chunk search before)
    for (uint32_t p0 = 0; p0 < nch; p0 += CV_CAP) {
        const uintptr_t lo = c0 + uintptr_t(p0) * 16u, hi = c0 + uintptr_t(min(nch, p0 + CV_CAP)) * 16u;
        if (p0 > 0) __syncthreads();   // the previous pass's table reads are done
        if (threadIdx.x == 0 && p0 == 0) cv[0] = 0;
        for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
            const uint32_t b = coff[v], e = v + 1 < nv ? coff[v + 1] : total;
            if (e <= b) continue;
            const uintptr_t ab = max(a0 + b, lo), ae = min(a0 + e, hi);
            for (uintptr_t c = (ab + 15) & ~uintptr_t(15); c < ae; c += 16) cv[(c - lo) >> 4] = uint16_t(v);
        }
        __syncthreads();
        for (uint32_t ci = threadIdx.x; ci < uint32_t((hi - lo) >> 4); ci += blockDim.x)
            copy_chunk16(coff, csrc, nv, total, sbase, send, a0, lo + uintptr_t(ci) * 16u, cv[ci]);
    }
}

// PLAIN BYTE_ARRAY chars (round 4): the tile's values are consecutive in the page body, each after its
// 4-byte length, so output byte r of value v comes from csrc[0] + r + 4 v: the chars are the source
// range with a 4-byte hole before every value. A thread copies one 64-byte output span with ONE round
// of source loads (the span's bytes plus 4 per value starting inside it: <= 21 aligned dwords), then
// assembles each output dword from the two shifted source dwords around a hole (v_perm). copy_chars_fast
// issued one dependent round of loads per 16-byte chunk, and its chunks spanning values (most of them
// for ~27-byte comments) blended one value piece at a time. Spans at the tile's ends, and spans where
// more than SP_K values start (or two holes fall in one dword), take copy_chunk16 per chunk.
constexpr uint32_t SP_K = 4;
__device__ __forceinline__ uint32_t sp_pick(const uint32_t* Z, int d, uint32_t h) {   // Z[d + h], h <= SP_K
    uint32_t r = Z[d];
    #pragma unroll
    for (uint32_t k = 1; k <= SP_K; k++) r = h >= k ? Z[d + int(k)] : r;
    return r;
}
__device__ __forceinline__ void copy_chars_plain(const uint32_t* coff, const uint32_t* csrc, uint32_t nv, uint32_t total,
                                        const uint8_t* sbase, const uint8_t* send, uint8_t* obase, uint16_t* cv) {
    if (total == 0 || nv == 0) return;
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(obase);
    const uintptr_t s0 = a0 & ~uintptr_t(63);
    const uint32_t nsp = uint32_t(((a0 + total + 63) & ~uintptr_t(63)) - s0) / 64u;
    // more spans than the table holds (values averaging over 64 bytes): the chunk copy, in passes
    if (nsp > CV_CAP) { copy_chars_fast(coff, csrc, nv, total, sbase, send, obase, cv); return; }
    // value v owns the spans whose first byte lies inside it
    if (threadIdx.x == 0) cv[0] = 0;
    for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
        const uint32_t b = coff[v], e = v + 1 < nv ? coff[v + 1] : total;
        if (e <= b) continue;
        const uintptr_t ab = a0 + b, ae = a0 + e;
        for (uintptr_t c = (ab + 63) & ~uintptr_t(63); c < ae; c += 64) cv[(c - s0) >> 6] = uint16_t(v);
    }
    __syncthreads();
    const uint32_t base0 = csrc[0] - coff[0];   // (coff[0] == 0)
    for (uint32_t si = threadIdx.x; si < nsp; si += blockDim.x) {
        const uintptr_t c = s0 + uintptr_t(si) * 64u;
        const int64_t r0 = int64_t(c) - int64_t(a0);
        const uint32_t v = si == 0 ? 0u : uint32_t(cv[si]);
        bool wide = r0 >= 0 && r0 + 64 <= int64_t(total);
        uint64_t M = 0;   // bit b: a value starts at span byte b (0 < b < 64)
        uint32_t K = 0;
        if (wide) {
            uint32_t u = v + 1, prev = 0;
            #pragma unroll
            for (uint32_t k = 0; k <= SP_K; k++) {
                const uint32_t b = u < nv ? coff[u] - uint32_t(r0) : 64u;
                if (b < 64u) {
                    wide &= k < SP_K && b != prev;   // (a zero-length value: two holes at one byte)
                    M |= 1ull << b;
                    K++;
                    prev = b;
                    u++;
                }
            }
        }
        const uintptr_t src = reinterpret_cast<uintptr_t>(sbase) + base0 + uint32_t(r0) + 4u * v;
        if (wide) wide = src + 64u + 4u * K + 4u <= reinterpret_cast<uintptr_t>(send);
        if (wide) {   // a dword holding two holes (values of 1-3 bytes) is not one v_perm
            #pragma unroll
            for (int d = 0; d < 16; d++) wide &= __popcll((M >> (4 * d + 1)) & 7ull) <= 1;
        }
        if (!wide) {
            #pragma unroll
            for (int k = 0; k < 4; k++) copy_chunk16(coff, csrc, nv, total, sbase, send, a0, c + 16u * uint32_t(k), v);
            continue;
        }
        const uint32_t sh = uint32_t(src & 3u);
        const PF_GLOBAL uint32_t* q = (const PF_GLOBAL uint32_t*)(src & ~uintptr_t(3));
        const uint32_t nd = (sh + 64u + 4u * K + 3u) >> 2;   // <= 21 dwords hold the span's source bytes
        uint32_t W[21];   // (all issued together: dwords past nd re-read the last one, never past send)
        #pragma unroll
        for (int k = 0; k < 21; k++) W[k] = q[min(uint32_t(k), nd - 1u)];
        uint32_t Z[20];   // Z[j]: the 4 source bytes at src + 4 j
        #pragma unroll
        for (int k = 0; k < 20; k++) Z[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], sh);
        uint32_t o[16];
        #pragma unroll
        for (int d = 0; d < 16; d++) {
            const uint32_t h0 = uint32_t(__popcll(M & ((2ull << (4 * d)) - 1ull)));   // holes before byte 4 d + 1
            const uint32_t m3 = uint32_t(M >> (4 * d + 1)) & 7u;                          // a hole at byte 4 d + 1..3
            const uint32_t A = sp_pick(Z, d, h0);
            const uint32_t B = sp_pick(Z, d, min(h0 + 1u, SP_K));
            const uint32_t t = uint32_t(__ffs(m3));                                         // 1..3, 0: none
            const uint32_t sel = 0x03020100u | (t ? (0x04040404u & (0xffffffffu << (8u * t))) : 0u);
            o[d] = __builtin_amdgcn_perm(B, A, sel);
        }
        PF_GLOBAL u32x4* d4 = (PF_GLOBAL u32x4*)c;
        #pragma unroll
        for (int k = 0; k < 4; k++) d4[k] = u32x4{o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
    }
}

#ifndef PF_SHORT_AVG
#define PF_SHORT_AVG 32   // r05: SF1 2.624-2.626 vs 2.630-2.643 ms at 16 (24: 2.610-2.631), configs 1 / 5 unchanged
#endif
constexpr uint32_t SHORT_AVG = PF_SHORT_AVG;   // tiles averaging at most this many chars per value: copy_chars_short
// Short values (dictionary strings such as flags and modes: 1-16 chars): one value per thread,
// lane-consecutive values, so a wave's byte stores cover one contiguous run of the chars arena.
// Each 8-byte piece of a value is read as the aligned dwords around it (+ v_alignbyte); a chunk
// copy (copy_chars_fast) would blend up to 16 values into every 16-byte chunk one at a time.
__device__ inline void copy_chars_short(const uint32_t* coff, const uint32_t* csrc, uint32_t nv, uint32_t total,
                                        const uint8_t* sbase, uint8_t* obase) {
    for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
        const uint32_t b = coff[v], e = v + 1 < nv ? coff[v + 1] : total;
        const uint8_t* sp = sbase + csrc[v];
        uint8_t* dp = obase + b;
        for (uint32_t o = 0; o < e - b; o += 8) {
            const uint32_t len = min(8u, e - b - o);
            const uintptr_t a = reinterpret_cast<uintptr_t>(sp + o);
            const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
            const uint32_t sh = uint32_t(a & 3u);
            const uint32_t d0 = q[0];
            const uint32_t d1 = sh + len > 4u ? q[1] : 0u;
            const uint32_t d2 = sh + len > 8u ? q[2] : 0u;
            const uint64_t x = uint64_t(__builtin_amdgcn_alignbyte(d1, d0, sh)) |
                               (uint64_t(__builtin_amdgcn_alignbyte(d2, d1, sh)) << 32);
            for (uint32_t i = 0; i < len; i++) dp[o + i] = uint8_t(x >> (8 * i));
        }
    }
}

struct FlatLds {
    uint32_t dpos[DSTR_CAP], dlen[DSTR_CAP];
    Run drun[RUN_CAP];
    Run vrun[RUN_CAP];
    uint32_t coff[FT];
    uint32_t csrc[FT];
    uint16_t cv[CV_CAP];
    uint32_t vbits[FT / 32 + 2];
    uint32_t scan_tmp[NT / 64];
    RunWalk dst, vst;
    int ndrun, nvrun, dres, vres, allp;
    uint32_t dcover, vcover, vlo;
};

// ---- k_snappy_head: pages whose Snappy stream needs no executor or no scratch ----------------
//
// One thread per Snappy job of a data page, before the parse kernels (DecompressorStream.java:101-173
// hands every page to snappy-java; here two common shapes skip work):
//  * INPLACE: the stream is a single literal (incompressible pages: bit-packed dictionary ids,
//    dictionary pages of random data): the decompressed body IS the literal's bytes in the
//    compressed input. The page's body points there and every Snappy kernel skips the job
//    (FB_INPLACE): no index / chain / repair / splits / executor work, no scratch copy.
//  * VALUES: a PLAIN fixed-width page of a flat chunk whose levels are all present (v2: the level
//    section; v1: the first literal must hold the level section, as it does for parquet-mr and
//    Arrow pages) and whose values section is exactly num_values * width bytes: the executor
//    writes the values straight into the column (SnappyJob.ddst) and k_flat_fixed only sets the
//    validity bits of the page (north_star's fusion of decompression with the PLAIN decode).
// Anything else, and every page whose stream turns out not to parse, takes the normal path.
__global__ __launch_bounds__(64) void k_snappy_head(SnappyJob* __restrict__ jobs, int n_jobs, DevPage* __restrict__ pages,
                                                    const DevChunk* __restrict__ chunks, int* __restrict__ fb,
                                                    const DevChunkResult* __restrict__ res) {
    const int j = int(blockIdx.x) * 64 + int(threadIdx.x);
    if (j >= n_jobs || fb[j] != FB_OK) return;
    SnappyJob& J = jobs[j];
    DevPage& pg = pages[J.page];
    const DevChunk& ck = chunks[pg.chunk];
    if (res[pg.chunk].status != 0) return;
    const uint8_t* in = J.src;
    const uint64_t n = J.src_len;
    uint64_t pos = 0, ulen = 0;
    if (!uvarint(in, n, pos, ulen) || ulen != J.dst_len || pos >= n) return;
    const SnapTok t = snap_tok(glb_read8(in, n, pos));
    if (t.kind != 0) return;
    const uint64_t data = pos + t.arg;   // the first literal's bytes: in[data, data + t.ol)
    if (data + t.ol > n) return;
    const bool one = pos + t.tl == n && t.ol == J.dst_len;   // one literal covers the page
    if ((J.dflags & 2u) && !(one && !(pg.flags & PG_DICT))) {
        // a stream of literals only (incompressible data: Snappy emits one literal per 64 KiB block,
        // e.g. a 400 KB dictionary of random values is 7): copied to the scratch body by
        // k_snappy_litcopy from a table {data offset, output offset} per literal, kept in the job's
        // token bitmap (unused: no index pass runs on the job), without any parse. Dictionary pages
        // always take this (their decoded pointers were set from the scratch body, and gathers want it
        // aligned); data pages only when flagged by the host (compressed size >= uncompressed).
        uint32_t* tab = J.tokmap;
        uint64_t p = pos, o = 0;
        uint32_t cnt = 0;
        while (p < n && cnt < LC_MAX) {
            const SnapTok u = snap_tok(glb_read8(in, n, p));
            const uint64_t d = p + u.arg;
            if (u.kind != 0 || d + u.ol > n) break;
            tab[2 * cnt] = uint32_t(d);
            tab[2 * cnt + 1] = uint32_t(o);
            o += u.ol;
            p = d + u.ol;
            cnt++;
        }
        if (p == n && o == J.dst_len && cnt > 0) {
            J.lit = cnt;
            fb[j] = FB_LITCOPY;
            return;
        }
        // not a literal-only stream after all (a copy token, or more than LC_MAX literals): a data
        // page still gets the VALUES setup below (the partial table is overwritten by k_snappy_index)
    }
    if (pg.flags & PG_DICT) return;
    if (one) {
        pg.body = in + data;
        pg.direct = DIRECT_INPLACE;
        fb[j] = FB_INPLACE;
        return;
    }
    // PLAIN fixed width, flat, all present
    const int w = ck.width;
    if (pg.encoding != 0 || ck.max_rep != 0 || ck.ptype == 0 || ck.ptype == 6 || w <= 0 || !ck.values) return;
    const uint32_t ne = uint32_t(pg.num_values);
    uint32_t L = 0;
    if (ck.max_def > 0) {
        const int bw = bit_width(uint32_t(ck.max_def));
        if (pg.flags & PG_V2) {
            if (!all_present(pg.lvl + pg.rep_len, pg.def_len, bw, ne, uint32_t(ck.max_def))) return;
        } else {
            if (pg.def_enc != 3 || t.ol < 4) return;
            const uint32_t lv = ld32le(in + data, 0, 4);
            if (lv > 60u || 4u + lv > t.ol) return;   // the level section must sit in the first literal
            if (!all_present(in + data + 4, lv, bw, ne, uint32_t(ck.max_def))) return;
            L = 4u + lv;
        }
    }
    if (uint64_t(J.dst_len) != uint64_t(L) + uint64_t(ne) * uint64_t(w)) return;
    uint8_t* dd = ck.values + uint64_t(pg.entry_start) * uint64_t(w) - L;
    const uintptr_t al = reinterpret_cast<uintptr_t>(dd);
    const uint32_t gran = (al & 15u) == 0 ? 16u : ((al & 7u) == 0 ? 8u : ((al & 3u) == 0 ? 4u : 0u));
    if (gran == 0) return;
    J.ddst = dd;
    J.dlo = L;
    J.dgran = gran;
    pg.direct = DIRECT_VALUES;
}

// k_flat, all levels present, fixed-width values: value index = entry index, lane-consecutive
// entries so every load and store of a wave is one contiguous run of memory. Returns err.
#ifndef PF_DICT_LDS
#define PF_DICT_LDS 16384   // 16 KiB: 0.8 % faster SF1 step than 32 KiB (occupancy), 64 KiB 8 % slower (tools/gpu_ab_libs.sh)
#endif
constexpr uint32_t DICT_LDS = PF_DICT_LDS;   // bytes of a fixed-width dictionary staged in LDS (k_flat_fixed)
#ifndef PF_FIX_IDS
#define PF_FIX_IDS 0   // extra LDS bytes behind the dictionary for a block's ids (6144, which fits the date
                       // columns' 10 + 12 KB, costs a workgroup per CU: SF1 2.660-2.663 vs 2.632-2.655 ms)
#endif
struct FixedLds {
    uint64_t dict[(DICT_LDS + PF_FIX_IDS) / 8 + 2];   // the dictionary, then the block's id bytes when they fit
    Run vrun[RUN_CAP];
    uint32_t coff[FTX / 64];
    RunWalk vst;
    int nvrun, vres, allp;
    uint32_t vcover, vlo;
    uint32_t ib[2];                   // the block's id byte range [ib[0], ib[1])
};

template <class Lds>
__device__ __forceinline__ int flat_present_fixed(Lds& S, const DevChunk& ck, const DevPage& pg, const Sections& s, bool dict,
                                  bool boolean, int enc, int w, const uint8_t* ids, uint64_t ids_n, int id_bw,
                                  uint64_t slot_base, uint32_t e_begin, uint32_t e_end, bool direct = false) {
    const int tid = threadIdx.x;
    const uint8_t* vend = s.val + s.val_n;
    const bool dalign = dict && (reinterpret_cast<uintptr_t>(ck.dict_data) & uintptr_t(w - 1)) == 0;
    // dictionary gather from LDS when the whole dictionary fits (north_star: K3 LDS / global)
    const bool dlds = DICT_LDS > 0 && dict && dalign && (w == 4 || w == 8) && ck.dict_data != nullptr &&
                      ck.dict_n > 0 && uint64_t(ck.dict_n) * uint64_t(w) <= DICT_LDS;
    // The block's dictionary ids, when the run table covers the block and their bytes fit behind the
    // dictionary: staged in LDS with the dictionary's loads (round 5), so the tiles read ids from LDS
    // instead of issuing a round of id loads per tile batch. Page id byte k is staged byte k - idd.
    const uint32_t dbytes = dlds ? (uint32_t(ck.dict_n) * uint32_t(w) + 15u) & ~15u : 0u;
    uint8_t* const sid = reinterpret_cast<uint8_t*>(S.dict) + dbytes;
    int64_t idd = 0;
    bool ilds = false;
    if (dict && dalign && (w == 4 || w == 8) && id_bw > 0 && id_bw <= 32 && s.val_n > 0 && S.vres != 2 &&
        S.vlo <= e_begin && e_end <= S.vcover) {
        if (tid == 0) { S.ib[0] = 0xffffffffu; S.ib[1] = 0u; }
        __syncthreads();
        for (int r = tid; r < S.nvrun; r += NT) {
            const Run R = S.vrun[r];
            const uint32_t f = max(R.first, e_begin), l = min(R.first + R.count, e_end);
            if (!R.packed || f >= l) continue;
            atomicMin(&S.ib[0], uint32_t((uint64_t(R.data) + uint64_t(f - R.first) * uint64_t(id_bw)) >> 3));
            atomicMax(&S.ib[1], uint32_t((uint64_t(R.data) + uint64_t(l - R.first) * uint64_t(id_bw) + 7u) >> 3));
        }
        __syncthreads();
        const uint32_t lo = S.ib[0], hi = S.ib[1];
        if (lo < hi && hi <= ids_n) {
            const uintptr_t a0 = (reinterpret_cast<uintptr_t>(ids) + lo) & ~uintptr_t(15);
            const uintptr_t aend = reinterpret_cast<uintptr_t>(ids) + ids_n;     // readable source end
            const uint32_t nb = (uint32_t(reinterpret_cast<uintptr_t>(ids) + hi - a0) + 8u + 15u) & ~15u;
            if (dbytes + nb <= uint32_t(sizeof(S.dict))) {
                ilds = true;
                idd = int64_t(a0) - int64_t(reinterpret_cast<uintptr_t>(ids));
                for (uint32_t c = tid; c < nb / 16u; c += NT) {
                    const uintptr_t a = a0 + 16u * c;
                    u32x4 x;
                    if (a + 16u <= aend) {
                        x = *reinterpret_cast<const PF_GLOBAL u32x4*>(a);
                    } else {   // the section's last bytes: no read past it
                        uint32_t q[4] = {0, 0, 0, 0};
                        for (uint32_t b = 0; b < 16u && a + b < aend; b++)
                            q[b >> 2] |= uint32_t(*reinterpret_cast<const PF_GLOBAL uint8_t*>(a + b)) << (8 * (b & 3));
                        x = u32x4{q[0], q[1], q[2], q[3]};
                    }
                    reinterpret_cast<u32x4*>(sid)[c] = x;
                }
            }
        }
    }
    if (dlds) {   // eight loads a thread in flight per round (a 2,526-entry date dictionary: 2 rounds, not 10)
        const uint32_t dn = uint32_t(ck.dict_n);
        if (w == 8) {
            const PF_GLOBAL uint64_t* g = (const PF_GLOBAL uint64_t*)(ck.dict_data);
            for (uint32_t i0 = tid; i0 < dn; i0 += 8u * NT) {
                uint64_t v[8];
                #pragma unroll
                for (uint32_t k = 0; k < 8; k++) v[k] = i0 + k * NT < dn ? g[i0 + k * NT] : 0ull;
                #pragma unroll
                for (uint32_t k = 0; k < 8; k++) if (i0 + k * NT < dn) S.dict[i0 + k * NT] = v[k];
            }
        } else {
            const PF_GLOBAL uint32_t* g = (const PF_GLOBAL uint32_t*)(ck.dict_data);
            uint32_t* d32 = reinterpret_cast<uint32_t*>(S.dict);
            for (uint32_t i0 = tid; i0 < dn; i0 += 8u * NT) {
                uint32_t v[8];
                #pragma unroll
                for (uint32_t k = 0; k < 8; k++) v[k] = i0 + k * NT < dn ? g[i0 + k * NT] : 0u;
                #pragma unroll
                for (uint32_t k = 0; k < 8; k++) if (i0 + k * NT < dn) d32[i0 + k * NT] = v[k];
            }
        }
    }
    if (dlds || ilds) __syncthreads();
    for (uint32_t e0 = e_begin, want = 0; e0 < e_end; e0 += want) {
        want = min(uint32_t(FTX), e_end - e0);
        int bad = 0;
        if (dict) {
            if ((S.vlo > e0 || e0 + want > S.vcover) && S.vres == 2) {
                __syncthreads();
                if (tid < 64) {   // next window of runs (re-walk from the page start), wave 0
                    if (tid == 0) { S.vst = RunWalk{0, 0}; S.vlo = e0; }
                    const int rr = wave_walk_runs(ids, ids_n, id_bw, e0, e_end, S.vrun, RUN_CAP, S.nvrun, S.vcover, S.vst, RunWalk{0, 0});
                    if (tid == 0) S.vres = rr;
                }
                __syncthreads();
                // a tile whose ids need more runs than the table holds (runs shorter than FTX / RUN_CAP
                // values): this tile is the part the table covers, the next window starts after it
                if (S.vres == 2 && S.vcover > e0 && e0 + want > S.vcover) want = S.vcover - e0;
            }
            if (id_bw > 32 || s.val_n == 0 || ck.dict_data == nullptr || e0 + want > S.vcover || S.vlo > e0) bad = 1;
            if (!bad && uint32_t(tid) < (want + 63) / 64) S.coff[tid] = uint32_t(run_find(S.vrun, S.nvrun, e0 + tid * 64));
            __syncthreads();
        }
        const bool wide = w == 4 || w == 8;
        if (direct) {
            // the executor wrote this page's values into the column (k_snappy_head): validity only
        } else if (!bad && wide && ((dict && dalign) || enc == 0 || enc == 5)) {
            // batched: the loads of FB entries per thread are in flight together
#ifndef PF_FB_DIV
#define PF_FB_DIV 2
#endif
            constexpr uint32_t FB = FEPTX / PF_FB_DIV;   // entries per thread per load batch
            for (uint32_t kb = 0; kb < FEPTX; kb += FB) {
            uint64_t v[FB];
            uint32_t id[FB];
            #pragma unroll
            for (uint32_t k = 0; k < FB; k++) {
                const uint32_t e = e0 + (kb + k) * NT + uint32_t(tid);
                id[k] = 0;
                v[k] = 0;
                if (e >= e0 + want) continue;
                if (dict) {
                    int r = int(S.coff[(e - e0) >> 6]);
                    while (e >= S.vrun[r].first + S.vrun[r].count) r++;
                    const Run R = S.vrun[r];
                    id[k] = R.data;
                    if (R.packed) {
                        const uint64_t bit = uint64_t(R.data) + uint64_t(e - R.first) * uint64_t(id_bw);
                        if (ilds) {
                            const uint32_t rb = uint32_t(int64_t(bit) - 8 * idd);
                            const uint32_t* q = reinterpret_cast<const uint32_t*>(sid) + (rb >> 5);
                            const uint64_t x = (uint64_t(q[0]) | (uint64_t(q[1]) << 32)) >> (rb & 31u);
                            id[k] = uint32_t(x & (id_bw == 32 ? 0xffffffffull : ((1ull << id_bw) - 1ull)));
                        } else {
                            id[k] = (bit >> 3) + 12 <= ids_n ? bits_fast(ids + (bit >> 3), uint32_t(bit & 7), id_bw)
                                                             : bits_le(ids, ids_n, bit, id_bw);
                        }
                    }
                } else if (enc == 0) {
                    if ((uint64_t(e) + 1) * uint64_t(w) > s.val_n) { bad = 1; continue; }
                    const uint8_t* src = s.val + uint64_t(e) * uint64_t(w);
                    if (w == 8) v[k] = src + 12 <= vend ? gld_u64_12(src) : ld64_bytes(src);
                    else v[k] = src + 8 <= vend ? gld_u32_8(src) : ld32le(src, 0, 4);
                } else {
                    v[k] = reinterpret_cast<const uint64_t*>(pg.aux)[e];
                }
            }
            if (dict) {   // all FB gathers issued together (entries past the tile / bad ids load element 0)
                const int64_t dn = ck.dict_n;
                #pragma unroll
                for (uint32_t k = 0; k < FB; k++) {
                    const uint32_t e = e0 + (kb + k) * NT + uint32_t(tid);
                    if (e < e0 + want && int64_t(id[k]) >= dn) bad = 1;
                    id[k] = int64_t(id[k]) < dn ? id[k] : 0u;
                }
                if (dlds) {
                    #pragma unroll
                    for (uint32_t k = 0; k < FB; k++)
                        v[k] = w == 8 ? S.dict[id[k]] : reinterpret_cast<const uint32_t*>(S.dict)[id[k]];
                } else if (w == 8) {
                    const PF_GLOBAL uint64_t* g = (const PF_GLOBAL uint64_t*)ck.dict_data;
                    #pragma unroll
                    for (uint32_t k = 0; k < FB; k++) v[k] = g[id[k]];
                } else {
                    const PF_GLOBAL uint32_t* g = (const PF_GLOBAL uint32_t*)ck.dict_data;
                    #pragma unroll
                    for (uint32_t k = 0; k < FB; k++) v[k] = g[id[k]];
                }
            }
            #pragma unroll
            for (uint32_t k = 0; k < FB; k++) {
                const uint32_t e = e0 + (kb + k) * NT + uint32_t(tid);
                if (e >= e0 + want) continue;
                uint8_t* dst = ck.values + (slot_base + e) * uint64_t(w);
                if (w == 8) *reinterpret_cast<uint64_t*>(dst) = v[k];
                else *reinterpret_cast<uint32_t*>(dst) = uint32_t(v[k]);
            }
            }
        } else if (!bad) {
            #pragma unroll 2
            for (uint32_t k = 0; k < FEPTX; k++) {
                const uint32_t e = e0 + k * NT + uint32_t(tid);
                if (e >= e0 + want) break;
                uint8_t* dst = ck.values + (slot_base + e) * uint64_t(w);
                if (dict) {
                    int r = int(S.coff[(e - e0) >> 6]);
                    while (e >= S.vrun[r].first + S.vrun[r].count) r++;
                    const Run R = S.vrun[r];
                    uint32_t id = R.data;
                    if (R.packed) {
                        const uint64_t bit = uint64_t(R.data) + uint64_t(e - R.first) * uint64_t(id_bw);
                        id = (bit >> 3) + 12 <= ids_n ? bits_fast(ids + (bit >> 3), uint32_t(bit & 7), id_bw)
                                                      : bits_le(ids, ids_n, bit, id_bw);
                    }
                    if (int64_t(id) >= ck.dict_n) { bad = 1; continue; }
                    const uint8_t* src = ck.dict_data + uint64_t(id) * uint64_t(w);
                    if (w == 8 && dalign) *reinterpret_cast<uint64_t*>(dst) = *reinterpret_cast<const uint64_t*>(src);
                    else if (w == 4 && dalign) *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(src);
                    else copy_value(dst, src, w);
                } else if (boolean) {
                    if ((e >> 3) >= s.val_n) { bad = 1; continue; }
                    dst[0] = uint8_t((s.val[e >> 3] >> (e & 7)) & 1u);
                } else if (enc == 0) {
                    if ((uint64_t(e) + 1) * uint64_t(w) > s.val_n) { bad = 1; continue; }
                    const uint8_t* src = s.val + uint64_t(e) * uint64_t(w);
                    if (w == 8 && src + 12 <= vend) *reinterpret_cast<uint64_t*>(dst) = gld_u64_12(src);
                    else if (w == 4 && src + 8 <= vend) *reinterpret_cast<uint32_t*>(dst) = gld_u32_8(src);
                    else copy_value(dst, src, w);
                } else {   // DELTA_BINARY_PACKED, decoded by k_delta into aux
                    const uint64_t* dv = reinterpret_cast<const uint64_t*>(pg.aux);
                    if (w == 8) *reinterpret_cast<uint64_t*>(dst) = dv[e];
                    else *reinterpret_cast<uint32_t*>(dst) = uint32_t(dv[e]);
                }
            }
        }
        if (ck.max_def > 0 && ck.validity) {   // all present: the tile's validity bits are ones
            const uint64_t b0 = slot_base + e0, b1 = b0 + want;
            uint32_t* vw = reinterpret_cast<uint32_t*>(ck.validity);
            for (uint64_t wd = (b0 >> 5) + tid; wd <= ((b1 - 1) >> 5); wd += NT) {
                const uint64_t lo = max(b0, wd << 5), hi = min(b1, (wd + 1) << 5);
                const uint32_t m = uint32_t((hi - lo >= 32 ? 0xffffffffull : ((1ull << (hi - lo)) - 1ull)) << (lo & 31));
                if (lo == (wd << 5) && hi == ((wd + 1) << 5)) vw[wd] = m;
                else atomicOr(vw + wd, m);
            }
        }
        if (__syncthreads_or(bad)) return 1;
    }
    return 0;
}

// k_flat for fixed-width pages whose levels are all present (the common case), with a small LDS
// footprint and its own register budget: one workgroup per (page, FBLK block). Marks the page
// done; k_flat decodes everything else (strings, pages with nulls).
// Returns whether the block took its (page, block) (block-uniform); false: k_flat's body decodes it.
__device__ __forceinline__ bool flat_fixed_block(FixedLds& S, const DevChunk* __restrict__ chunks, DevPage* pages, const int2 pbk,
                                 DevChunkResult* res) {
    if (pbk.x < 0) return true;   // padding of the XCD-grouped block list (runtime)
    const int pi = pbk.x;
    const uint32_t blk = uint32_t(pbk.y) & 0x0fffffffu;
    const uint32_t bsz = FBLK << (uint32_t(pbk.y) >> 28);   // entries per block (runtime: wide blocks for no-null pages)
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    // the page's, chunk's and result's words are read in one round (bitwise ors: a short-circuit
    // chain puts a wait between each load)
    const int* jfb = pg.jfb;
    const bool dval = pg.direct == DIRECT_VALUES;
    const int jf = jfb != nullptr ? *jfb : FB_WHOLE + 1;
    if ((res[pg.chunk].status != 0) | (ck.max_rep != 0) | (ck.ptype == 6) | ((pg.done & DONE_NULL) != 0)) return false;
    if (dval & (jf <= FB_WHOLE)) {
        // the executor wrote the values (k_snappy_head checked the levels): this block's validity bits
        const uint32_t ne = uint32_t(pg.num_values), e_begin = blk * bsz;
        if (e_begin >= ne && blk > 0) return true;
        const uint32_t e_end = min(ne, e_begin + bsz);
        if (ck.max_def > 0 && ck.validity && e_end > e_begin) {
            const uint64_t b0 = uint64_t(pg.entry_start) + e_begin, b1 = uint64_t(pg.entry_start) + e_end;
            uint32_t* vw = reinterpret_cast<uint32_t*>(ck.validity);
            for (uint64_t wd = (b0 >> 5) + threadIdx.x; wd <= ((b1 - 1) >> 5); wd += NT) {
                const uint64_t lo = max(b0, wd << 5), hi = min(b1, (wd + 1) << 5);
                const uint32_t m = uint32_t((hi - lo >= 32 ? 0xffffffffull : ((1ull << (hi - lo)) - 1ull)) << (lo & 31));
                if (lo == (wd << 5) && hi == ((wd + 1) << 5)) vw[wd] = m;
                else atomicOr(vw + wd, m);
            }
        }
        if (threadIdx.x == 0) {
            if (ck.needs_count == 0)
                atomicAdd(reinterpret_cast<unsigned long long*>(&res[pg.chunk].num_values), (unsigned long long)(e_end - e_begin));
            atomicOr(&pg.done, DONE_FIXED);
        }
        return true;
    }
    Sections s;
    if (!page_sections(pg, ck, s)) return false;
    const int enc = pg.encoding;
    const bool boolean = ck.ptype == 0, dict = is_dict_enc(enc);
    const int w = ck.width;
    bool take = ck.max_def == 0 || s.def_rle;
    if (enc == 0) {
    } else if (dict) take = take && !boolean;
    else if (enc == 5) take = take && (ck.ptype == 1 || ck.ptype == 2) && pg.aux != nullptr;
    else take = false;
    if (!take) return false;
    const uint32_t ne = uint32_t(pg.num_values);
    if (blk > 0 && blk * bsz >= ne) return true;
    const int id_bw = (dict && s.val_n > 0) ? int(s.val[0]) : 0;
    const uint8_t* ids = dict && s.val_n > 0 ? s.val + 1 : s.val;
    const uint64_t ids_n = dict && s.val_n > 0 ? s.val_n - 1 : 0;
    const uint32_t* T = pg.runtab;
    uint32_t t0 = 0, t3 = 0;
    if (T != nullptr) { t0 = T[0]; t3 = T[3]; }
    const bool tab = (t3 == 1u) & (t0 <= uint32_t(RUN_CAP));   // k_runs: levels all present
    if (tid == 0)
        S.allp = tab ? 1 : (ck.max_def == 0 ? 1 : all_present(s.def, s.def_n, bit_width(ck.max_def), ne, uint32_t(ck.max_def)));
    __syncthreads();
    if (!S.allp) return false;
    const uint32_t e_begin = blk * bsz;
    const uint32_t e_end = min(ne, e_begin + bsz);
#ifdef PF_STAMPS
    const unsigned long long ft0 = __builtin_amdgcn_s_memtime();
#endif
    if (dict) {
        if (tab) {
            const uint32_t nr = T[0], cov = T[1];
            for (uint32_t i = tid; i < nr; i += NT) {
                const uint32_t f = T[4 + 2 * i];
                const uint32_t nf = i + 1 < nr ? (T[4 + 2 * (i + 1)] & 0x7fffffffu) : cov;
                Run r;
                r.first = f & 0x7fffffffu;
                r.count = nf - r.first;
                r.data = T[5 + 2 * i];
                r.packed = f >> 31;
                S.vrun[i] = r;
            }
            if (tid == 0) { S.nvrun = int(nr); S.vcover = cov; S.vlo = 0; S.vres = cov >= ne ? 0 : 1; }
        } else if (tid < 64) {   // wave 0 walks the id runs of this block
            if (tid == 0) { S.nvrun = 0; S.vcover = 0; S.vres = 0; S.vlo = e_begin; S.vst = RunWalk{0, 0}; }
            if (s.val_n > 0 && id_bw <= 32) {
                const int rr = wave_walk_runs(ids, ids_n, id_bw, e_begin, e_end, S.vrun, RUN_CAP, S.nvrun, S.vcover, S.vst, RunWalk{0, 0});
                if (tid == 0) S.vres = rr;
            }
        }
        __syncthreads();
    }
    // values already in place: the executor decoded the page without falling back (a redo / serial
    // fallback writes the body to scratch instead, and the page is decoded from there)
    const bool direct = dval & (jf <= FB_WHOLE);
    const int err = flat_present_fixed(S, ck, pg, s, dict, boolean, enc, w, ids, ids_n, id_bw,
                                       uint64_t(pg.entry_start), e_begin, e_end, direct);
#ifdef PF_STAMPS
    if (tid == 0) { const unsigned long long dt_ = __builtin_amdgcn_s_memtime() - ft0; PSTAMP(1, dt_); PSTAMP(0, 1); atomicMax(&pf_pstamps[9], dt_); }
#endif
    if (tid == 0) {
        if (err) set_status(res, pg.chunk, ST_CORRUPT, pi);
        else if (ck.needs_count == 0)
            atomicAdd(reinterpret_cast<unsigned long long*>(&res[pg.chunk].num_values), (unsigned long long)(e_end - e_begin));
        atomicOr(&pg.done, DONE_FIXED);
    }
    return true;
}

// Fallback queue (device, zeroed with the batch metadata): word 0 counts the (page, block) pairs that
// start at word 4; k_flat_null and k_flat_fixed append the blocks they do not take, the last workgroups of k_flat_all decode them.
__device__ __forceinline__ void null_fallback(int* fbq, int2 pbk) {
    if (threadIdx.x == 0) reinterpret_cast<int2*>(fbq + 4)[atomicAdd(fbq, 1)] = pbk;
}

// k_flat_fixed (round 5): the blocks of flat fixed-width pages, in a list of their own. Its register
// budget is the fixed-width body's (73 VGPRs, 21 KiB LDS: six workgroups per CU, against four of
// k_flat_all's 127-VGPR union of both bodies); blocks it does not take (a page with nulls that
// k_flat_null did not take, levels that are not RLE, ...) go to the fallback queue (k_flat_all's last workgroups).
#ifndef PF_FIXED_OCC
#define PF_FIXED_OCC 6
#endif
__global__ __launch_bounds__(NT, PF_FIXED_OCC) void k_flat_fixed(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                              const int2* __restrict__ blocks, DevChunkResult* res, int* fbq) {
    __shared__ FixedLds S;
    const int2 pbk = blocks[blockIdx.x];
    if (!flat_fixed_block(S, chunks, pages, pbk, res)) null_fallback(fbq, pbk);
}

// One workgroup per (page, FBLK block of entries). Pages whose levels are all present (max_def
// == 0 or RLE runs of max_def) are decoded block by block in parallel: value index = entry
// index, each block walks the dictionary-id run headers up to its own range (windowed when a
// block needs more than RUN_CAP runs) and takes its chars base from k_count's block table or,
// for PLAIN BYTE_ARRAY, from the value positions. Pages with nulls are decoded by block 0 alone.
__device__ __forceinline__ void flat_block(FlatLds& S, const DevChunk* __restrict__ chunks, DevPage* pages, const int2 pbk,
                           DevChunkResult* res) {
    if (pbk.x < 0) return;   // padding of the XCD-grouped block list (runtime)
    const int pi = pbk.x;
    const uint32_t blk = uint32_t(pbk.y) & 0x0fffffffu;
    const uint32_t bsz = FBLK << (uint32_t(pbk.y) >> 28);   // (wide blocks: fixed-width pages only)
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    // DONE_FIXED: k_flat_fixed took the page. Never test DONE_FLAT here: this kernel's own blocks of
    // the same page set it when they finish, and a block that starts later must still run.
    if ((res[pg.chunk].status != 0) | (ck.max_rep != 0) | ((pg.done & (DONE_FIXED | DONE_NULL)) != 0)) return;
    Sections s;
    if (!page_sections(pg, ck, s)) return;                 // k_decode reports it
    const int enc = pg.encoding;
    const bool binary = ck.ptype == 6, boolean = ck.ptype == 0, dict = is_dict_enc(enc);
    const int w = ck.width;
    bool take = ck.max_def == 0 || s.def_rle;
    if (enc == 0) {
    } else if (dict) take = take && !boolean;
    else if (enc == 5) take = take && (ck.ptype == 1 || ck.ptype == 2) && pg.aux != nullptr;
    else take = false;
    if (!take) return;

    const int bwd = bit_width(ck.max_def);
    const uint32_t ne = uint32_t(pg.num_values);
    const int id_bw = (dict && s.val_n > 0) ? int(s.val[0]) : 0;
    const uint8_t* ids = dict && s.val_n > 0 ? s.val + 1 : s.val;
    const uint64_t ids_n = dict && s.val_n > 0 ? s.val_n - 1 : 0;
    const bool counted = ck.needs_count != 0;
    const uint64_t slot_base = uint64_t(pg.entry_start);   // flat: slot == entry
    if (blk > 0 && blk * bsz >= ne) return;
    const uint32_t* T = pg.runtab;
    uint32_t t0 = 0, t3 = 0;
    if (T != nullptr) { t0 = T[0]; t3 = T[3]; }
    const bool tab = (t3 == 1u) & (t0 <= uint32_t(RUN_CAP));   // k_runs: levels all present
    if (tid == 0) S.allp = tab ? 1 : (ck.max_def == 0 ? 1 : all_present(s.def, s.def_n, bwd, ne, uint32_t(ck.max_def)));
    __syncthreads();
    const bool split = S.allp;
    if (!split && blk > 0) return;                          // block 0 decodes the whole page
    const uint32_t e_begin = split ? blk * bsz : 0u;
    const uint32_t e_end = split ? min(ne, e_begin + bsz) : ne;
#ifdef PF_STAMPS
    const unsigned long long ft0 = __builtin_amdgcn_s_memtime();
    if (tid == 0) { PSTAMP(0, 1); if (dict) PSTAMP(6, 1); if (binary) PSTAMP(7, 1); }
#endif
    if (tid < 64) {   // wave 0: definition-level runs (pages with nulls)
        if (tid == 0) { S.ndrun = 0; S.dcover = ne; S.dres = 0; S.dst = RunWalk{0, 0}; }
        if (!split && ck.max_def > 0) {
            const int rr = wave_walk_runs(s.def, s.def_n, bwd, 0, ne, S.drun, RUN_CAP, S.ndrun, S.dcover, S.dst, RunWalk{0, 0});
            if (tid == 0) S.dres = rr;
        }
    } else if (tid < 128 && !(split && tab)) {   // wave 1: dictionary-id runs
        if (tid == 64) { S.nvrun = 0; S.vcover = 0; S.vres = 0; S.vlo = e_begin; S.vst = RunWalk{0, 0}; }
        if (dict && s.val_n > 0 && id_bw <= 32) {
            const int rr = wave_walk_runs(ids, ids_n, id_bw, e_begin, split ? e_end : ne, S.vrun, RUN_CAP, S.nvrun,
                                          S.vcover, S.vst, RunWalk{0, 0});
            if (tid == 64) S.vres = rr;
        }
    }
    if (split && tab) {   // the page's run table (k_runs), loaded by all threads
        const uint32_t nr = T[0], cov = T[1];
        for (uint32_t i = tid; i < nr; i += NT) {
            const uint32_t f = T[4 + 2 * i];
            const uint32_t nf = i + 1 < nr ? (T[4 + 2 * (i + 1)] & 0x7fffffffu) : cov;
            Run r;
            r.first = f & 0x7fffffffu;
            r.count = nf - r.first;
            r.data = T[5 + 2 * i];
            r.packed = f >> 31;
            S.vrun[i] = r;
        }
        if (tid == 0) { S.nvrun = int(nr); S.vcover = cov; S.vlo = 0; S.vres = cov >= ne ? 0 : 1; }
    }
    // small string dictionaries: {pos, len} from LDS (visible after the tile loop's first barrier)
    const bool dstage = binary && dict && ck.dict_pos != nullptr && ck.dict_n > 0 && ck.dict_n <= int64_t(DSTR_CAP);
    if (dstage) {
        const PF_GLOBAL uint32_t* gp = gptr(ck.dict_pos);
        const PF_GLOBAL uint32_t* gl = gptr(ck.dict_len);
        for (uint32_t i = uint32_t(tid); i < uint32_t(ck.dict_n); i += NT) { S.dpos[i] = gp[i]; S.dlen[i] = gl[i]; }
    }
    __syncthreads();
#ifdef PF_STAMPS
    unsigned long long ft1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) PSTAMP(2, ft1 - ft0);
#endif
    if (!split && (S.dres == 2 || S.vres == 2)) return;    // too many runs: k_decode takes the page
    bool allp = true, lvl_bad = S.dres != 0;
    if (!split) {
        for (int r = 0; r < S.ndrun; r++) {
            const Run& R = S.drun[r];
            if (R.packed || R.data != uint32_t(ck.max_def)) allp = false;
            if (!R.packed && R.data > uint32_t(ck.max_def)) lvl_bad = true;
        }
    }
    if (lvl_bad) {
        if (tid == 0) { set_status(res, pg.chunk, ST_CORRUPT, pi); atomicOr(&pg.done, DONE_FLAT); }
        return;
    }
    uint64_t char_base = 0;
    if (binary && counted) {
        char_base = uint64_t(pg.char_start);
        if (e_begin > 0) {
            if (dict) char_base += flat_block_chars(pg)[blk];
            else char_base += uint64_t(pg.aux[e_begin]) - 4ull * (uint64_t(e_begin) + 1);
        }
    }
    uint64_t vidx = e_begin;                                // page-relative index of the next present value
    int err = 0;
#ifdef PF_STAMPS   // tile sub-phases (tools/probe_flat_all.py): 11 levels, 12 values, 13 scan, 14 offsets, 15 chars
    unsigned long long fs_ = __builtin_amdgcn_s_memtime();
#define FSTAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(i, t_ - fs_); fs_ = t_; } while (0)
#else
#define FSTAMP(i) ((void)0)
#endif


    for (uint32_t e0 = e_begin, want = 0; e0 < e_end; e0 += want) {
        want = min(uint32_t(FT), e_end - e0);
        if (split && dict && S.vres == 2 && (uint64_t(S.vlo) > uint64_t(e0) || e0 + want > S.vcover)) {
            // all levels present: value index = entry index. Next window of id runs before the levels,
            // and a tile needing more runs than the table holds shrinks to what it covers
            __syncthreads();
            if (tid < 64) {
                if (tid == 0) { S.vst = RunWalk{0, 0}; S.vlo = e0; }
                const int rr = wave_walk_runs(ids, ids_n, id_bw, e0, e_end, S.vrun, RUN_CAP, S.nvrun, S.vcover, S.vst,
                                              RunWalk{0, 0});
                if (tid == 0) S.vres = rr;
            }
            __syncthreads();
            if (S.vres == 2 && S.vcover > e0 && e0 + want > S.vcover) want = S.vcover - e0;
        }
        const uint32_t eb = uint32_t(tid) * FEPT;
        for (uint32_t i = tid; i < FT / 32 + 2; i += NT) S.vbits[i] = 0;
        // ---- definition levels -> present bits of this thread's entries
        uint32_t fv = 0;
        int bad = 0;
        if (eb < want) {
            const uint32_t m = min(uint32_t(FEPT), want - eb);
            if (allp) {
                fv = m >= 32 ? 0xffffffffu : (1u << m) - 1u;
            } else {
                const uint32_t e = e0 + eb;
                int r = run_find(S.drun, S.ndrun, e);
                for (uint32_t k = 0; k < m; k++) {
                    while (e + k >= S.drun[r].first + S.drun[r].count) r++;
                    const uint32_t d = run_value(S.drun[r], s.def, s.def_n, e + k, bwd);
                    bad |= d > uint32_t(ck.max_def);
                    fv |= uint32_t(d == uint32_t(ck.max_def)) << k;
                }
            }
        }
        uint32_t tv;
        uint32_t vo;
        if (allp) { vo = min(eb, want); tv = want; }
        else vo = block_excl_scan<NT>(__popc(fv), S.scan_tmp, tv);
        // ---- dictionary: this tile's values [vidx, vidx + tv) must be in the run table
        if (tv > 0 && dict) {
            if (split && (uint64_t(S.vlo) > vidx || vidx + tv > uint64_t(S.vcover)) && S.vres == 2) {
                __syncthreads();
                if (tid < 64) {   // next window of runs (re-walk from the page start), wave 0
                    if (tid == 0) { S.vst = RunWalk{0, 0}; S.vlo = uint32_t(vidx); }
                    const int rr = wave_walk_runs(ids, ids_n, id_bw, uint32_t(vidx), e_end, S.vrun, RUN_CAP, S.nvrun,
                                                  S.vcover, S.vst, RunWalk{0, 0});
                    if (tid == 0) S.vres = rr;
                }
                __syncthreads();
            }
            if (id_bw > 32 || s.val_n == 0 || (binary ? ck.dict_pos == nullptr : ck.dict_data == nullptr) ||
                vidx + tv > uint64_t(S.vcover) || uint64_t(S.vlo) > vidx)
                bad = 1;
        }
        if (__syncthreads_or(bad)) { err = 1; break; }
        FSTAMP(11);
        // ---- values
        uint32_t lsum = 0;
        uint32_t my_src[FEPT], my_len[FEPT];   // indexed by entry k (static after unrolling)
        {
            uint32_t j = 0;
            int vr = -1;
            #pragma unroll
            for (uint32_t k = 0; k < FEPT; k++) {
                my_src[k] = 0;
                my_len[k] = 0;
                if (eb + k >= want) continue;
                const uint64_t slot = slot_base + e0 + eb + k;
                const bool present = (fv >> k) & 1u;
                if (!binary) {
                    uint8_t* dst = ck.values + slot * uint64_t(w);
                    if (!present) { zero_value(dst, w); continue; }
                    const uint64_t gv = vidx + vo + j++;
                    if (dict) {
                        if (vr < 0) vr = run_find(S.vrun, S.nvrun, uint32_t(gv));
                        while (gv >= uint64_t(S.vrun[vr].first) + S.vrun[vr].count) vr++;
                        const uint32_t id = run_value(S.vrun[vr], ids, ids_n, uint32_t(gv), id_bw);
                        if (int64_t(id) >= ck.dict_n) { bad = 1; continue; }
                        copy_value(dst, ck.dict_data + uint64_t(id) * uint64_t(w), w);
                    } else if (boolean) {
                        if ((gv >> 3) >= s.val_n) { bad = 1; continue; }
                        dst[0] = uint8_t((s.val[gv >> 3] >> (gv & 7)) & 1u);
                    } else if (enc == 0) {
                        if ((gv + 1) * uint64_t(w) > s.val_n) { bad = 1; continue; }
                        copy_value(dst, s.val + gv * uint64_t(w), w);
                    } else {   // DELTA_BINARY_PACKED, decoded by k_delta into aux
                        const uint64_t* dv = reinterpret_cast<const uint64_t*>(pg.aux);
                        if (w == 8) *reinterpret_cast<uint64_t*>(dst) = dv[gv];
                        else *reinterpret_cast<uint32_t*>(dst) = uint32_t(dv[gv]);
                    }
                } else if (present) {
                    // strings: ids / positions of all FEPT entries first (their loads in flight
                    // together), the dictionary {pos, len} gathers in a second pass
                    const uint64_t gv = vidx + vo + j;
                    if (dict) {
                        if (vr < 0) vr = run_find(S.vrun, S.nvrun, uint32_t(gv));
                        while (gv >= uint64_t(S.vrun[vr].first) + S.vrun[vr].count) vr++;
                        const Run R = S.vrun[vr];
                        uint32_t id = R.data;
                        if (R.packed) {
                            const uint64_t bit = uint64_t(R.data) + uint64_t(uint32_t(gv) - R.first) * uint64_t(id_bw);
                            id = (bit >> 3) + 12 <= ids_n ? bits_fast(ids + (bit >> 3), uint32_t(bit & 7), id_bw)
                                                          : bits_le(ids, ids_n, bit, id_bw);
                        }
                        my_src[k] = id;
                        my_len[k] = 1;   // present (the length comes from the dictionary)
                    } else {   // PLAIN: value positions from the k_ba walk; a value's length is the
                               // distance to the next position (the walk checked the chain), the
                               // page's last value reads its length prefix
                        const PF_GLOBAL uint32_t* ax = gptr(pg.aux);
                        const uint32_t p = ax[gv];
                        uint32_t ln;
                        if (split && gv + 1 < uint64_t(ne)) {
                            const uint32_t nx = ax[gv + 1];
                            ln = nx >= p + 4 ? nx - p - 4 : 0xffffffffu;
                        } else {
                            ln = (p >= 4 && p <= s.val_n) ? ld32le(s.val, p - 4, s.val_n) : 0xffffffffu;
                        }
                        if (p >= 4 && p <= s.val_n && ln <= s.val_n - p) { my_src[k] = p; my_len[k] = ln; lsum += ln; }
                        else bad = 1;
                    }
                    j++;
                }
            }
            if (binary && dict) {
                const PF_GLOBAL uint32_t* gp = gptr(ck.dict_pos);
                const PF_GLOBAL uint32_t* gl = gptr(ck.dict_len);
                #pragma unroll
                for (uint32_t k = 0; k < FEPT; k++) {
                    if (!my_len[k]) continue;
                    const uint32_t id = my_src[k];
                    uint32_t src = 0, l = 0;
                    if (int64_t(id) >= ck.dict_n) bad = 1;
                    else if (dstage) { src = S.dpos[id]; l = S.dlen[id]; }
                    else { src = gp[id]; l = gl[id]; }
                    my_src[k] = src;
                    my_len[k] = l;
                    lsum += l;
                }
            }
        }
        FSTAMP(12);
        uint32_t tchars = 0;
        const uint32_t lo = binary ? block_excl_scan<NT>(lsum, S.scan_tmp, tchars) : 0;
        if (binary && char_base + tchars > uint64_t(pg.char_start + pg.n_chars)) bad = 1;   // k_count disagrees
        if (__syncthreads_or(bad)) { err = 1; break; }
        FSTAMP(13);
        if (binary) {
            uint32_t c = lo, j = 0;
            #pragma unroll
            for (uint32_t k = 0; k < FEPT; k++) {
                if (eb + k >= want) continue;
                if ((fv >> k) & 1u) {
                    S.coff[vo + j] = c;
                    S.csrc[vo + j] = my_src[k];
                    c += my_len[k];
                    j++;
                }
                ck.offsets[slot_base + e0 + eb + k + 1] = int32_t(char_base + c);
            }
        }
        // validity bits of this thread's entries
        if (ck.max_def > 0 && fv) {
            const uint64_t abase = (slot_base + e0) & ~uint64_t(31);
            const uint64_t rb = slot_base + e0 + eb - abase;
            const uint32_t sh = uint32_t(rb & 31);
            atomicOr(&S.vbits[rb >> 5], fv << sh);
            if (sh + FEPT > 32 && sh) atomicOr(&S.vbits[(rb >> 5) + 1], fv >> (32 - sh));
        }
        __syncthreads();
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) { PSTAMP(4, t_ - ft1); PSTAMP(3, 1); PSTAMP(14, t_ - fs_); } ft1 = t_; fs_ = t_; }
#endif
        if (binary) {
            const uint8_t* sb = dict ? ck.dict_data : s.val;
            const uint8_t* se = dict ? pages[ck.dict_page].body + pages[ck.dict_page].body_len : s.val + s.val_n;
            if (tchars <= SHORT_AVG * tv) copy_chars_short(S.coff, S.csrc, tv, tchars, sb, ck.chars + char_base);
            else if (!dict) copy_chars_plain(S.coff, S.csrc, tv, tchars, sb, se, ck.chars + char_base, S.cv);
            else copy_chars_fast(S.coff, S.csrc, tv, tchars, sb, se, ck.chars + char_base, S.cv);
        }
        FSTAMP(15);
        if (ck.max_def > 0 && ck.validity) flush_bits(S.vbits, slot_base + e0, want, ck.validity);
        vidx += tv;
        char_base += tchars;
        __syncthreads();
#ifdef PF_STAMPS
        { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(5, t_ - ft1); ft1 = t_; }
#endif
    }
#ifdef PF_STAMPS
    if (tid == 0) {
        const unsigned long long dt_ = __builtin_amdgcn_s_memtime() - ft0;
        PSTAMP(1, dt_);
        atomicMax(&pf_pstamps[binary ? 8 : 9], dt_);
        if (!split) PSTAMP(10, 1);
    }
#endif
    if (tid == 0) {
        if (err) set_status(res, pg.chunk, ST_CORRUPT, pi);
        else if (!counted) atomicAdd(reinterpret_cast<unsigned long long*>(&res[pg.chunk].num_values),
                                     (unsigned long long)(vidx - e_begin));
        atomicOr(&pg.done, DONE_FLAT);
    }
}


// k_flat_fixed and k_flat in one launch over the same (page, block) list: a block decodes its page
// with the fixed-width body when that applies, else with the general body. One stage instead of
// two in stream order (the fixed-width columns' blocks no longer wait for the string blocks or the
// other way round); the LDS of the two bodies is shared (they never run in one block together).
#ifndef PF_FLAT_OCC
#define PF_FLAT_OCC 5   // round 5 (with CV_CAP 2048 and the chars copies inlined): SF1 2.74 -> 2.69 ms; 4 before
#endif
// Workgroups n.. of the grid take the fallback queue (round 6: k_flat_fb's launch folded in; the producers
// of the queue, k_flat_fixed and k_flat_null, are earlier in stream order): a grid stride over the queued
// blocks, nearly always none.
__global__ __launch_bounds__(NT, PF_FLAT_OCC) void k_flat_all(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                 const int2* __restrict__ blocks, int n, const int* __restrict__ fbq,
                                                 DevChunkResult* res) {
    __shared__ union FlatAllLds {
        FixedLds f;
        FlatLds g;
    } S;
    if (int(blockIdx.x) >= n) {
        const int nq = fbq[0], g = int(gridDim.x) - n;
        for (int i = int(blockIdx.x) - n; i < nq; i += g) {
            const int2 pq = reinterpret_cast<const int2*>(fbq + 4)[i];
            if (!flat_fixed_block(S.f, chunks, pages, pq, res)) {
                __syncthreads();
                flat_block(S.g, chunks, pages, pq, res);
            }
            __syncthreads();   // the block's LDS reads are done before the next one reuses it
        }
        return;
    }
    const int2 pbk = blocks[blockIdx.x];
    if (flat_fixed_block(S.f, chunks, pages, pbk, res)) return;
    __syncthreads();   // the fixed body's LDS reads are done before the general body reuses it
    flat_block(S.g, chunks, pages, pbk, res);
}

// ---- nullable flat pages: definition-level run table + block-parallel decode ------------------
//
// north_star K2/K6: "RLE/bit-packed-hybrid expansion of definition levels ... using prefix scans to
// find run boundaries" and null scatter. k_lvl walks a page's level run headers once (they are few:
// ~300 per 20,000 entries at 30 % random nulls), counts the present values of every run in parallel
// and scans them, so that every 4096-entry block of the page knows the value index of its first
// present entry. k_flat_null then decodes the blocks in parallel: levels -> present bits -> block
// scan -> value index -> dictionary gather / PLAIN load; null slots are zero.
constexpr uint32_t LVL_STAGE = 4096;   // level sections up to this size are decoded from LDS (k_lvl)

// Bits [bit, bit + k) (k <= 32) of an LDS byte array (LSB-first), from the two aligned dwords around it.
__device__ __forceinline__ uint32_t lds_bits(const uint8_t* st, uint32_t bit, uint32_t k) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(st);
    const uint32_t wi = bit >> 5, sh = bit & 31u;
    const uint64_t v = uint64_t(w[wi]) | (uint64_t(w[wi + 1]) << 32);
    return uint32_t(v >> sh) & (k >= 32 ? 0xffffffffu : ((1u << k) - 1u));
}

// Last level run with first entry <= e (runs: k_lvl table rows of 4 words, runs[0].first == 0).
__device__ __forceinline__ uint32_t lvl_run_at(const uint32_t* runs, uint32_t nr, uint32_t e) {
    uint32_t lo = 0, hi = nr;
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (runs[4 * m] <= e) lo = m; else hi = m;
    }
    return lo;
}
// Present values before entry e, which lies in run r (its present-before count plus the present
// levels of the run before e, from the staged level section).
__device__ inline uint32_t lvl_values_before(const uint32_t* runs, uint32_t r, uint32_t e, const uint8_t* stage,
                                             uint32_t woff, int bw, uint32_t maxd) {
    const uint32_t first = runs[4 * r], data = runs[4 * r + 1], cw = runs[4 * r + 2];
    const uint32_t before = e - first;
    uint32_t vb = runs[4 * r + 3];
    if (!(cw >> 31)) return vb + (data == maxd ? before : 0u);
    if (bw == 1) {
        for (uint32_t i = 0; i < before; i += 32) {
            const uint32_t k = min(32u, before - i), bb = woff * 8u + data + i;
            if (bb + k <= LVL_STAGE * 8u) vb += __popc(lds_bits(stage, bb, k));
        }
    } else {
        for (uint32_t i = 0; i < before; i++) {
            const uint32_t bb = woff * 8u + data + i * uint32_t(bw);
            if (bb + uint32_t(bw) <= LVL_STAGE * 8u) vb += lds_bits(stage, bb, uint32_t(bw)) == maxd;
        }
    }
    return vb;
}
// Dictionary-id run (k_runs table T: {nruns, covered, valid, -}, then {first | packed << 31, data})
// holding value v.
__device__ __forceinline__ uint32_t id_run_at(const uint32_t* T, uint32_t nr, uint32_t v) {
    uint32_t lo = 0, hi = nr;
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if ((T[4 + 2 * m] & 0x7fffffffu) <= v) lo = m; else hi = m;
    }
    return lo;
}

constexpr int LT_NT = 256;                // k_lvl: four waves per page
constexpr uint32_t LVL_RUNS_LDS = 512;    // level runs k_lvl keeps in LDS (pages with more read them from HBM)
constexpr uint32_t LVL_NXT = 4096;        // = LVL_STAGE: k_lvl's all-positions header tables cover its sections
constexpr uint32_t LVL_JUMP = 8;          // runs per step of k_lvl's chain walk (jump table: 3 doubling passes)
constexpr uint32_t LVL_S8 = LVL_NXT / LVL_JUMP;   // walk steps (a run is at least one byte)
constexpr uint32_t LVL_PPT = LVL_NXT / LT_NT;     // section positions per thread in the table passes
static_assert(LVL_PPT == 16, "k_lvl's mark words: two threads per 32 positions");
#ifndef PF_LVL_OCC
#define PF_LVL_OCC 1   // k_lvl workgroups per CU the register budget must allow (1: the compiler's choice, 114 VGPRs;
                       // 5: 96 VGPRs + 80 B scratch, config 4 3.70-3.75 vs 3.68-3.74 ms, not kept)
#endif
__global__ __launch_bounds__(LT_NT, PF_LVL_OCC) void k_lvl(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list,
                                               DevChunkResult* res, uint32_t dcap, uint32_t icap) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[LVL_STAGE + 48];
    __shared__ uint32_t scan_tmp[LT_NT / 64];
    __shared__ uint32_t s_ns8;
    // next-header positions of every byte position (0xffff: not a header, or its run passes the
    // section end; dn: the chain ends there), then the page's dictionary-id runs (k_runs) for the
    // block table
    __shared__ union { uint16_t nxt[LVL_NXT]; uint32_t T[4 + 2 * RUN_CAP]; } s_u;
    // the 8-run jump table during the chain walk, then the LDS copy of the level runs
    __shared__ union { uint16_t jmp[LVL_NXT]; uint32_t runs[4 * LVL_RUNS_LDS]; } s_a;
    __shared__ uint16_t s_s8[LVL_S8];         // chain positions of runs 0, 8, 16, ...
    __shared__ uint32_t s_mark[LVL_NXT / 32];  // chain positions (run headers)
    static_assert(sizeof(uint16_t) * LVL_NXT >= sizeof(uint32_t) * (4 + 2 * RUN_CAP), "s_u sized by the header table");
    uint16_t* const s_nxt = s_u.nxt;
    uint32_t* const s_T = s_u.T;
    uint16_t* const s_jmp = s_a.jmp;
    uint32_t* const s_runs = s_a.runs;
    const int pi = list[blockIdx.x];
    DevPage& pg = pages[pi];
    uint32_t* LT = pg.lvltab;
    if (!LT) return;
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    Sections s;
    if (pg.done & DONE_PAGE) {   // k_page_null decoded the page
        if (tid == 0) LT[1] = 0;
        return;
    }
    if (res[pg.chunk].status != 0 || ck.max_rep != 0 || ck.max_def <= 0 || !page_sections(pg, ck, s) || !s.def_rle ||
        s.def_n > LVL_STAGE) {   // (longer level sections: k_flat / k_decode)
        if (tid == 0) LT[1] = 0;
        return;
    }
    const uint32_t ne = uint32_t(pg.num_values);
    const int bw = bit_width(uint32_t(ck.max_def));
    const uint32_t maxd = uint32_t(ck.max_def);
    const uint32_t dn = uint32_t(s.def_n);
#ifdef PF_STAMPS   // phase cycles per page (tools/probe_wide.py): 8 pages, 9 stage, 10 header table, 11 chain,
                   // 12 run decode, 13 present counts, 14 block table, 15 total; 6 runs, 7 level bytes
    unsigned long long lt_ = __builtin_amdgcn_s_memtime(), lt0_ = lt_;
#define LTS(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tid == 0) PSTAMP(i, t_ - lt_); lt_ = t_; } while (0)
    if (tid == 0) { PSTAMP(8, 1); PSTAMP(7, dn); }
#else
#define LTS(i) ((void)0)
#endif
    // stage the level section with aligned 16-byte loads: section byte i is stage[woff + i]; bytes
    // past the section read as zero (parquet-mr zero-pads a truncated bit-packed run)
    const uintptr_t sa = reinterpret_cast<uintptr_t>(s.def);
    const uint32_t woff = uint32_t(sa & 15u);
    if (woff + dn > LVL_STAGE) {
        if (tid == 0) LT[1] = 0;
        return;
    }
    {
        const PF_GLOBAL u32x4* src = (const PF_GLOBAL u32x4*)(sa - woff);
        const uint32_t nchunk = (woff + dn + 15u) / 16u;
        for (uint32_t c = tid; c < nchunk; c += LT_NT) reinterpret_cast<u32x4*>(stage)[c] = src[c];
        if (uint32_t(tid) < LVL_NXT / 32) s_mark[tid] = 0;
        __syncthreads();
        for (uint32_t i = woff + dn + uint32_t(tid); i < nchunk * 16u + 16u; i += LT_NT) stage[i] = 0;
        __syncthreads();
    }
    LTS(9);
    uint32_t* runs = LT + 4;
    const uint32_t cap = pg.lvl_cap;
    const uint8_t* const stw = stage + woff;
    // (1) every byte position decoded as a run header: the position of the next header
    for (uint32_t p = tid; p < dn; p += LT_NT) {
        uint32_t h = 0, hl = 0, nx = 0xffffu;
        #pragma unroll
        for (uint32_t k = 0; k < 3; k++) {   // headers over 2^21 are no runs of a <= 4 KiB section
            const uint32_t c = p + k < dn ? uint32_t(stw[p + k]) : 0x80u;
            h |= (c & 0x7fu) << (7 * k);
            if (!(c & 0x80u)) { hl = k + 1; break; }
        }
        if (hl) {
            const uint32_t pay = (h & 1u) ? (h >> 1) * uint32_t(bw) : (uint32_t(bw) + 7u) >> 3;
            if (p + hl + pay <= dn) nx = p + hl + pay;   // a truncated run ends the chain
        }
        s_nxt[p] = uint16_t(nx);
    }
    __syncthreads();
    LTS(10);
    // (2) the chain from position 0 (north_star K2: run boundaries by wavefront passes). The 8-run jump
    // table by three doubling passes, one thread walks it eight runs a step, then one thread per
    // 8-run stretch walks the runs in between and marks their headers. Terminal values stay put:
    // 0xffff (broken chain) and positions >= dn (the section end).
    {
        uint32_t J[LVL_PPT];
        #pragma unroll
        for (uint32_t k = 0; k < LVL_PPT; k++) {
            const uint32_t p = uint32_t(tid) + k * LT_NT;
            const uint32_t q = p < dn ? uint32_t(s_nxt[p]) : 0xffffu;
            J[k] = q < dn ? uint32_t(s_nxt[q]) : q;
        }
        #pragma unroll
        for (uint32_t k = 0; k < LVL_PPT; k++) s_jmp[uint32_t(tid) + k * LT_NT] = uint16_t(J[k]);
        __syncthreads();
        for (int pass = 0; pass < 2; pass++) {   // 2 -> 4 -> 8 runs
            #pragma unroll
            for (uint32_t k = 0; k < LVL_PPT; k++) J[k] = J[k] < dn ? uint32_t(s_jmp[J[k]]) : J[k];
            __syncthreads();
            #pragma unroll
            for (uint32_t k = 0; k < LVL_PPT; k++) s_jmp[uint32_t(tid) + k * LT_NT] = uint16_t(J[k]);
            __syncthreads();
        }
    }
    if (tid == 0) {
        uint32_t p = 0, k = 0;
        while (p < dn && k < LVL_S8) {
            s_s8[k++] = uint16_t(p);
            const uint32_t q = s_jmp[p];
            if (q >= dn) break;   // the chain ends (or breaks) within the next 8 runs
            p = q;
        }
        s_ns8 = k;
    }
    __syncthreads();
    const uint32_t ns8 = s_ns8;
    for (uint32_t j = tid; j < ns8; j += LT_NT) {
        uint32_t p = s_s8[j];
        for (uint32_t i = 0; i < LVL_JUMP && p < dn; i++) {
            const uint32_t q = s_nxt[p];
            if (q == 0xffffu) break;   // no run header here: the chain is broken
            atomicOr(&s_mark[p >> 5], 1u << (p & 31u));
            p = q;
        }
    }
    __syncthreads();
    LTS(11);
    // (3) the marked headers in position order: runs decoded at their headers in parallel, their
    // first entries an exclusive scan of the counts, runs with entries at or past the page's dropped
    const uint32_t mw = s_mark[tid >> 1];   // a thread's 16 positions: half a mark word
    const uint32_t mbits = (mw >> (16u * (uint32_t(tid) & 1u))) & 0xffffu;
    const uint32_t p0 = 16u * uint32_t(tid);
    uint32_t hcnt[LVL_PPT], hdat[LVL_PPT], hpk = 0;
    uint64_t csum = 0;
    #pragma unroll
    for (uint32_t k = 0; k < LVL_PPT; k++) {
        hcnt[k] = 0;
        hdat[k] = 0;
        if (!((mbits >> k) & 1u)) continue;
        const uint32_t P = p0 + k;
        uint32_t h = 0, hl = 0;
        for (uint32_t b = 0; b < 3; b++) {
            const uint32_t c = stw[P + b];
            h |= (c & 0x7fu) << (7 * b);
            if (!(c & 0x80u)) { hl = b + 1; break; }
        }
        const uint32_t packed = h & 1u;
        hcnt[k] = packed ? (h >> 1) * 8u : (h >> 1);
        if (packed) hdat[k] = (P + hl) * 8u;
        else for (uint32_t b = 0; b < ((uint32_t(bw) + 7u) >> 3); b++) hdat[k] |= uint32_t(stw[P + hl + b]) << (8 * b);
        hpk |= packed << k;
        csum += hcnt[k];
    }
    __shared__ unsigned long long scan64[LT_NT / 64];
    uint64_t ctot;
    const uint64_t cbase = block_excl_scan64<LT_NT>(csum, scan64, ctot);
    uint32_t emask = 0, bad = 0;
    {
        uint64_t f = cbase;
        #pragma unroll
        for (uint32_t k = 0; k < LVL_PPT; k++) {
            if (hcnt[k] > 0 && f < ne) {
                emask |= 1u << k;
                if (!((hpk >> k) & 1u) && hdat[k] > maxd) bad = 1;
            }
            f += hcnt[k];
        }
    }
    __syncthreads();   // scan_tmp is reused
    uint32_t nr;
    const uint32_t rbase = block_excl_scan<LT_NT>(__popc(emask), scan_tmp, nr);
    {
        uint64_t f = cbase;
        uint32_t rank = rbase;
        #pragma unroll
        for (uint32_t k = 0; k < LVL_PPT; k++) {
            if ((emask >> k) & 1u && nr <= cap) {   // (emitted: f < ne)
                const uint32_t c = uint32_t(min<uint64_t>(hcnt[k], uint64_t(ne) - f));
                const uint32_t cw = c | (((hpk >> k) & 1u) << 31);
                runs[4 * rank + 0] = uint32_t(f);
                runs[4 * rank + 1] = hdat[k];
                runs[4 * rank + 2] = cw;
                if (rank < LVL_RUNS_LDS) {
                    s_runs[4 * rank + 0] = uint32_t(f);
                    s_runs[4 * rank + 1] = hdat[k];
                    s_runs[4 * rank + 2] = cw;
                }
                rank++;
            }
            f += hcnt[k];
        }
    }
    __threadfence_block();   // the run records (HBM and LDS) before the other waves read them
    const bool ok = __syncthreads_or(bad) == 0 && nr <= cap && ctot >= ne;   // (a broken chain covers too few)
    LTS(12);
    if (!ok) {
        if (tid == 0) LT[1] = 0;
        return;
    }
    uint32_t* const R = nr <= LVL_RUNS_LDS ? s_runs : runs;   // the scans below read this copy
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < nr; r0 += LT_NT) {
        const uint32_t r = r0 + uint32_t(tid);
        uint32_t pc = 0;
        if (r < nr) {
            const uint32_t data = R[4 * r + 1], cw = R[4 * r + 2];
            const uint32_t cnt = cw & 0x7fffffffu;
            if (!(cw >> 31)) pc = data == maxd ? cnt : 0u;
            else {
                // packed levels [data, data + cnt * bw) bits (the stage is zero past the section)
                const uint32_t nbits = cnt * uint32_t(bw);
                const uint32_t b0 = woff * 8u + data;
                if (bw == 1) {
                    for (uint32_t i = 0; i < nbits; i += 32) {
                        const uint32_t k = min(32u, nbits - i);
                        if (b0 + i + k <= LVL_STAGE * 8u) pc += __popc(lds_bits(stage, b0 + i, k));
                    }
                } else {
                    for (uint32_t i = 0; i < cnt; i++) {
                        const uint32_t b = b0 + i * uint32_t(bw);
                        if (b + uint32_t(bw) <= LVL_STAGE * 8u) pc += lds_bits(stage, b, uint32_t(bw)) == maxd;
                    }
                }
            }
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<LT_NT>(pc, scan_tmp, tot);
        if (r < nr) {
            runs[4 * r + 3] = carry + ex;
            if (R != runs) R[4 * r + 3] = carry + ex;
        }
        carry += tot;
        __syncthreads();   // scan_tmp is reused
    }
    LTS(13);
    // per FBLK block (k_flat_null): the runs it overlaps [r0, r1), the value indices of its first and
    // end entries, the level bytes its packed runs read and the dictionary-id bytes of its values
    __threadfence_block();
    uint32_t* BT = runs + 4 * cap;
    const uint32_t nblk = (ne + FBLK - 1) / FBLK;
    // dictionary id runs (k_runs, same stream): value index -> bit offset in the id stream
    const uint32_t* TG = pg.runtab;
    const bool dict = is_dict_enc(pg.encoding) && TG != nullptr && TG[2] == 1u && TG[0] <= uint32_t(RUN_CAP) && s.val_n > 0;
    const uint32_t tnr = dict ? TG[0] : 0u, tcov = dict ? TG[1] : 0u;
    if (dict)
        for (uint32_t i = tid; i < 4 + 2 * tnr; i += LT_NT) s_T[i] = TG[i];
    __syncthreads();
    const uint32_t* T = s_T;
    const uint32_t id_bw = dict ? uint32_t(s.val[0]) : 0u;
    uint32_t fit = 1;
    for (uint32_t b = tid; b < nblk; b += LT_NT) {
        const uint32_t eb = b * FBLK, ee = min(ne, eb + FBLK);
        const uint32_t lo = lvl_run_at(R, nr, eb);
        uint32_t a = lo, z = nr;    // first run with first >= ee
        while (a < z) {
            const uint32_t m = (a + z) >> 1;
            if (R[4 * m] < ee) a = m + 1; else z = m;
        }
        const uint32_t vb = lvl_values_before(R, lo, eb, stage, woff, bw, maxd);
        const uint32_t ve = ee == ne ? carry : lvl_values_before(R, lvl_run_at(R, nr, ee), ee, stage, woff, bw, maxd);
        // level bytes: from the first packed run's first bit to the last packed run's end
        uint32_t d0 = 0, d1 = 0;
        for (uint32_t r = lo; r < a; r++) {
            const uint32_t cw = R[4 * r + 2];
            if (!(cw >> 31)) continue;
            const uint32_t f = R[4 * r];
            d0 = (R[4 * r + 1] + (max(eb, f) - f) * uint32_t(bw)) >> 3;
            break;
        }
        for (uint32_t r = a; r > lo; r--) {
            const uint32_t cw = R[4 * (r - 1) + 2];
            if (!(cw >> 31)) continue;
            const uint32_t f = R[4 * (r - 1)], end = min(ee, f + (cw & 0x7fffffffu));
            d1 = (R[4 * (r - 1) + 1] + (end - f) * uint32_t(bw) + 7u) >> 3;
            break;
        }
        // dictionary-id bytes of values [vb, ve)
        uint32_t i0 = 0, i1 = 0;
        if (dict && ve > vb) {
            if (ve > tcov) fit = 0;
            else {
                const uint32_t q0 = id_run_at(T, tnr, vb), q1 = id_run_at(T, tnr, ve - 1);
                for (uint32_t q = q0; q <= q1; q++) {
                    if (!(T[4 + 2 * q] >> 31)) continue;
                    const uint32_t f = T[4 + 2 * q] & 0x7fffffffu;
                    i0 = uint32_t((uint64_t(T[5 + 2 * q]) + uint64_t(max(vb, f) - f) * id_bw) >> 3);
                    break;
                }
                for (uint32_t q = q1 + 1; q > q0; q--) {
                    if (!(T[4 + 2 * (q - 1)] >> 31)) continue;
                    const uint32_t f = T[4 + 2 * (q - 1)] & 0x7fffffffu;
                    const uint32_t nf = q < tnr ? (T[4 + 2 * q] & 0x7fffffffu) : tcov;
                    i1 = uint32_t((uint64_t(T[5 + 2 * (q - 1)]) + uint64_t(min(ve, nf) - f) * id_bw + 7u) >> 3);
                    break;
                }
            }
        }
        if (a - lo > LT_BLOCK_RUNS || d1 - d0 + 16u > dcap || i1 - i0 + 16u > icap || ve < vb) fit = 0;
        uint32_t* bt = BT + LT_BT_WORDS * b;
        bt[0] = lo; bt[1] = a; bt[2] = vb; bt[3] = ve;
        bt[4] = d0; bt[5] = d1; bt[6] = i0; bt[7] = i1;
    }
    fit = __syncthreads_and(fit) ? 1u : 0u;
    if (tid == 0) { LT[0] = nr; LT[2] = carry; LT[1] = fit; }
    LTS(14);
#ifdef PF_STAMPS
    if (tid == 0) PSTAMP(15, __builtin_amdgcn_s_memtime() - lt0_);
    if (tid == 0) PSTAMP(6, nr);
#endif
#undef LTS
}

// k_flat_null<W>: one 256-thread workgroup per 4096-entry block of a nullable W-byte page, 16
// consecutive entries per thread. The block's level runs, the page's id runs and the level / id bytes
// the block reads (k_lvl's block table) are all fetched at once into LDS, so the workgroup waits on one
// round of loads, then on the dictionary gather; no spread step: entry k of a thread takes the value of
// rank popc(fv & (2^k - 1)). The stage is latency-bound (Σ block latency / resident blocks), so what
// sets it is the entries in flight per CU: 16 per lane (round 5; 8 per lane at 512 threads: config 4's
// flat launch 0.97 -> 0.81 ms, gpurun_out/ntn). The runtime gives the kernel only nullable pages of its
// width (its own block lists); a page it does not take goes to the fallback queue (k_flat_all's last workgroups).
#ifndef PF_NTN
#define PF_NTN 256
#endif
constexpr int NTN = PF_NTN;
constexpr int NEPT = FBLK / NTN;   // 8 (512 threads) or 16 (256)
static_assert(NEPT % 4 == 0 && NEPT <= 16, "k_flat_null's stores and present masks");
// Runs in LDS as {first | packed << 31, data}: a run ends where the next begins (k_lvl's level runs
// and k_runs' id runs are contiguous), and one sentinel row after the last holds its end.
struct NullLds {
    uint2 drun[LT_BLOCK_RUNS + 1];
    uint2 vrun[RUN_CAP + 1];
    uint32_t vbits[FBLK / 32 + 2];
    uint32_t scan_tmp[NTN / 64];
};
__device__ __forceinline__ uint32_t rl_first(uint2 r) { return r.x & 0x7fffffffu; }
__device__ __forceinline__ int rl_find(const uint2* runs, int nr, uint32_t i) {   // run holding i (runs[0] first <= i)
    int lo = 0, hi = nr;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (rl_first(runs[mid]) <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// Dynamic LDS, sized by the host per batch (NullCaps): the block's level bytes (dcap + 32), its
// dictionary-id bytes (icap + 32) -- caps from the batch's level and id bit widths, which k_lvl's
// block table was checked against -- and dictionaries of at most dlds bytes (the batch's largest
// fitting one, <= NULL_DICT_LDS; 0 when it has none), gathered from LDS (north_star K3: "dictionary
// staged in LDS when it fits"); larger ones are gathered from L2 / HBM. Config 4 (1-bit levels,
// 17-bit ids): ~16.6 KiB a workgroup, eight resident per CU (the VGPR limit) instead of five.

template <int W> struct WidthType { using type = uint64_t; };
template <> struct WidthType<4> { using type = uint32_t; };

template <int W>
__global__ __launch_bounds__(NTN) void k_flat_null(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                   const int2* __restrict__ blocks, DevChunkResult* res, NullCaps nc,
                                                   int stagger, int* fbq) {
    using VT = typename WidthType<W>::type;
    __shared__ __attribute__((aligned(16))) NullLds S;
    extern __shared__ __attribute__((aligned(16))) uint64_t DYN[];
    uint32_t* const s_dst = reinterpret_cast<uint32_t*>(DYN);
    uint32_t* const s_ist = s_dst + (nc.dcap + 32u) / 4u;
    uint64_t* const DL = reinterpret_cast<uint64_t*>(s_ist + (nc.icap + 32u) / 4u);
    const uint32_t dlds = nc.dlds;
    const int2 pbk = blocks[blockIdx.x];
#ifdef PF_DIAG   // diagnostics build (tests): blocks after a page's first start late, after it has finished
    if (stagger && pbk.y > 0)
        for (int i = 0; i < stagger; i++) __builtin_amdgcn_s_sleep(127);
#else
    (void)stagger;
#endif
    if (pbk.x < 0) return;   // padding of the XCD-grouped block list (runtime)
#ifdef PF_STAMPS   // phase cycles per block: 0 blocks, 1 tables, 2 LDS stage, 3 levels + scan, 4 gather + store
    unsigned long long t_ph = __builtin_amdgcn_s_memtime(), t_beg = t_ph;
#define NSTAMP(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (threadIdx.x == 0) PSTAMP(i, t_ - t_ph); t_ph = t_; }
#else
#define NSTAMP(i) ((void)0)
#endif
    const int pi = pbk.x;
    const uint32_t blk = uint32_t(pbk.y) & 0x0fffffffu;   // (pages with a level table always have FBLK blocks)
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    const uint32_t* LT = pg.lvltab;
    // pages this kernel does not take (whole pages: the conditions are the page's) go to the fallback queue
    // (not DONE_NULL: blocks of this page that finished first set it, and a block starting later must still run)
    if (!LT || res[pg.chunk].status != 0 || ck.max_rep != 0 || ck.width != W ||
        (pg.done & (DONE_FIXED | DONE_PAGE)) || LT[1] != 1u) {   // (k_page_null took it, or no block table)
        null_fallback(fbq, pbk);
        return;
    }
    Sections s;
    const int enc = pg.encoding;
    const bool dict = is_dict_enc(enc);
    const uint32_t* T = pg.runtab;
    if (!page_sections(pg, ck, s) || (!dict && enc != 0) ||
        (dict && !(T != nullptr && T[2] == 1u && T[0] <= uint32_t(RUN_CAP) && s.val_n > 0 && ck.dict_data != nullptr))) {
        null_fallback(fbq, pbk);
        return;
    }
    const uint32_t ne = uint32_t(pg.num_values);
    const uint32_t e_begin = blk * FBLK;
    if (blk > 0 && e_begin >= ne) return;
    const uint32_t e_end = min(ne, e_begin + FBLK);
    constexpr int w = W;
    const int bw = bit_width(uint32_t(ck.max_def));
    const uint32_t maxd = uint32_t(ck.max_def);
    const uint32_t nr = LT[0];
    const uint32_t* runs = LT + 4;
    const uint32_t* bt = runs + 4 * pg.lvl_cap + LT_BT_WORDS * blk;
    const uint32_t r0 = bt[0], r1 = bt[1], vb = bt[2], ve = bt[3], d0 = bt[4], d1 = bt[5], i0 = bt[6], i1 = bt[7];
    const uint32_t id_bw = dict ? uint32_t(s.val[0]) : 0u;
    const uint32_t vnr = dict ? T[0] : 0u;
    const uint32_t idcov = dict ? T[1] : 0u;
    const uint8_t* ids = dict ? s.val + 1 : nullptr;
    const uint64_t ids_n = dict ? s.val_n - 1 : 0;
    if (r1 < r0 || (r1 == r0 && e_end > e_begin) || r1 - r0 > LT_BLOCK_RUNS || r1 > nr || id_bw > 32 || ve < vb || d1 < d0 || d1 - d0 + 16u > nc.dcap ||
        i1 < i0 || i1 - i0 + 16u > nc.icap || (dict && ve > idcov) || (!dict && uint64_t(ve) * uint64_t(w) > s.val_n)) {
        if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi);
        return;
    }
    NSTAMP(1);
    // one round of loads: level runs, id runs, level bytes, id bytes
    const uint32_t nrun = r1 - r0;
    for (uint32_t i = tid; i < nrun; i += NTN) {
        const uint32_t* q = runs + 4 * (r0 + i);
        const uint32_t f = q[0], d = q[1], c = q[2];
        S.drun[i] = make_uint2(f | (c & 0x80000000u), d);
        if (i + 1 == nrun) S.drun[nrun] = make_uint2(f + (c & 0x7fffffffu), 0u);
    }
    for (uint32_t i = tid; i <= vnr; i += NTN)
        S.vrun[i] = i < vnr ? make_uint2(T[4 + 2 * i], T[5 + 2 * i]) : make_uint2(idcov, 0u);
    const uint32_t doff = stage_bytes(s_dst, s.def, s.def_n, d0, d1);
    const uint32_t ioff = dict ? stage_bytes(s_ist, ids, ids_n, i0, i1) : 0u;
    for (uint32_t i = tid; i < FBLK / 32 + 2; i += NTN) S.vbits[i] = 0;
    const bool dl = dict && dlds != 0 && ck.dict_n > 0 && uint64_t(ck.dict_n) * uint64_t(w) <= dlds &&
                    (reinterpret_cast<uintptr_t>(ck.dict_data) & 7u) == 0;
    if (dl) {   // the dictionary into LDS (8-byte loads; the page body is 16-byte aligned scratch)
        const uint64_t* g = reinterpret_cast<const uint64_t*>(ck.dict_data);
        const uint32_t nw = uint32_t((uint64_t(ck.dict_n) * uint64_t(w) + 7u) / 8u);
        for (uint32_t i = tid; i < nw; i += NTN) DL[i] = g[i];
    }
    __syncthreads();
    NSTAMP(2);
    const uint8_t* dst8 = reinterpret_cast<const uint8_t*>(s_dst);
    const uint8_t* ist8 = reinterpret_cast<const uint8_t*>(s_ist);
    const uint32_t dbase = d0 * 8u - doff * 8u;   // stream bit of LDS bit 0
    const uint32_t ibase = i0 * 8u - ioff * 8u;
    const uint32_t dlim = (d1 - d0 + doff + 16u) * 8u;   // readable LDS bits
    const uint32_t ilim = (i1 - i0 + ioff + 16u) * 8u;
    int bad = 0;
    // present bits of this thread's entries
    const uint32_t e = e_begin + uint32_t(tid) * NEPT;
    const uint32_t m = e < e_end ? min(uint32_t(NEPT), e_end - e) : 0u;
    uint32_t fv = 0;
    if (m) {
        int r = rl_find(S.drun, int(nrun), e);
        const uint2 R = S.drun[r];
        const uint32_t Rf = rl_first(R), Rp = R.x >> 31;
        if (e + m <= rl_first(S.drun[r + 1]) && (!Rp || bw == 1)) {   // one run
            if (!Rp) fv = R.y == maxd ? ((1u << m) - 1u) : 0u;
            else {
                const uint32_t b = R.y + (e - Rf) - dbase;
                fv = b + m <= dlim ? lds_bits(dst8, b, m) : 0u;
                bad |= b + m > dlim;
            }
        } else {
            for (uint32_t k = 0; k < m; k++) {
                while (r + 1 < int(nrun) && e + k >= rl_first(S.drun[r + 1])) r++;
                const uint2 Rk = S.drun[r];
                uint32_t dl = Rk.y;
                if (Rk.x >> 31) {
                    const uint32_t b = Rk.y + (e + k - rl_first(Rk)) * uint32_t(bw) - dbase;
                    bad |= b + uint32_t(bw) > dlim;
                    dl = b + uint32_t(bw) <= dlim ? lds_bits(dst8, b, uint32_t(bw)) : 0u;
                }
                bad |= dl > maxd;
                fv |= uint32_t(dl == maxd) << k;
            }
        }
    }
    uint32_t tv;
    const uint32_t vo = block_excl_scan<NTN>(__popc(fv), S.scan_tmp, tv);
    if (tv != ve - vb) bad = 1;   // the block table disagrees with the levels
    NSTAMP(3);
    const uint32_t gv0 = vb + vo;   // value index of this thread's first present entry
    VT v[NEPT];
    #pragma unroll
    for (int k = 0; k < NEPT; k++) v[k] = 0;
    if (fv && !bad) {
        // Two phases: the ids of the present entries (LDS only), then ALL of the thread's gathers
        // issued back to back through global-address-space loads (absent entries load element 0 and
        // are zeroed after), so the wave waits on one round of L2 / HBM latency instead of one per
        // entry (flat loads under per-entry branches each ended in a vmcnt(0) wait).
        if (dict) {
            uint32_t idv[NEPT];
            #pragma unroll
            for (int k = 0; k < NEPT; k++) idv[k] = 0;
            int vr = rl_find(S.vrun, int(vnr), gv0);
            const uint2 V0 = S.vrun[vr];
            // the thread's present values are gv0, gv0 + 1, ...: when one id run holds them all, their
            // ids are consecutive fields of that run (no run search per value)
            const bool one_run = gv0 + uint32_t(__popc(fv)) <= rl_first(S.vrun[vr + 1]);
            const uint32_t b0 = (V0.x >> 31) ? uint32_t(uint64_t(V0.y) + uint64_t(gv0 - rl_first(V0)) * id_bw - ibase) : 0u;
            const int64_t dn = ck.dict_n;
            uint32_t r = 0;
            #pragma unroll
            for (int k = 0; k < NEPT; k++) {
                if (!((fv >> k) & 1u)) continue;
                uint32_t id;
                if (one_run) {
                    id = V0.y;
                    if (V0.x >> 31) {
                        const uint32_t b = b0 + r * id_bw;
                        bad |= b + id_bw > ilim;
                        id = b + id_bw <= ilim ? lds_bits(ist8, b, id_bw) : 0u;
                    }
                } else {
                    const uint32_t gv = gv0 + r;
                    while (vr + 1 < int(vnr) && gv >= rl_first(S.vrun[vr + 1])) vr++;
                    const uint2 V = S.vrun[vr];
                    id = V.y;
                    if (V.x >> 31) {
                        const uint32_t b = uint32_t(uint64_t(V.y) + uint64_t(gv - rl_first(V)) * id_bw - ibase);
                        bad |= b + id_bw > ilim;
                        id = b + id_bw <= ilim ? lds_bits(ist8, b, id_bw) : 0u;
                    }
                }
                r++;
                bad |= int64_t(id) >= dn;
                idv[k] = int64_t(id) < dn ? id : 0u;
            }
            const uintptr_t da = reinterpret_cast<uintptr_t>(ck.dict_data);
            if (dl) {
                #pragma unroll
                for (int k = 0; k < NEPT; k++) v[k] = reinterpret_cast<const VT*>(DL)[idv[k]];
            } else if ((da & uintptr_t(w - 1)) == 0) {   // (dictionary pages start 16-byte aligned in scratch)
                const PF_GLOBAL VT* g = (const PF_GLOBAL VT*)ck.dict_data;
                #pragma unroll
                for (int k = 0; k < NEPT; k++) v[k] = g[idv[k]];
            } else {
                #pragma unroll
                for (int k = 0; k < NEPT; k++) {
                    const uint8_t* src = ck.dict_data + uint64_t(idv[k]) * uint64_t(w);
                    if constexpr (W == 4) v[k] = ld_u32_any(src); else v[k] = ld_u64_any(src);
                }
            }
        } else {
            // value of entry k: gv0 + present entries before k (absent entries load their successor's,
            // clamped to the thread's last present value)
            const uint32_t last = gv0 + uint32_t(__popc(fv)) - 1u;
            uint32_t vi[NEPT];
            #pragma unroll
            for (int k = 0; k < NEPT; k++) vi[k] = min(gv0 + uint32_t(__popc(fv & ((1u << k) - 1u))), last);
            if ((reinterpret_cast<uintptr_t>(s.val) & uintptr_t(w - 1)) == 0) {
                const PF_GLOBAL VT* g = (const PF_GLOBAL VT*)s.val;
                #pragma unroll
                for (int k = 0; k < NEPT; k++) v[k] = g[vi[k]];
            } else {
                #pragma unroll
                for (int k = 0; k < NEPT; k++) {
                    const uint8_t* src = s.val + uint64_t(vi[k]) * uint64_t(w);
                    if constexpr (W == 4) v[k] = ld_u32_any(src); else v[k] = ld_u64_any(src);
                }
            }
        }
        #pragma unroll
        for (int k = 0; k < NEPT; k++)
            if (!((fv >> k) & 1u)) v[k] = 0;
    }
    const uint64_t slot_base = uint64_t(pg.entry_start);
    if (m && !bad) {
        uint8_t* dst0 = ck.values + (slot_base + e) * uint64_t(w);
        if (m == NEPT && (reinterpret_cast<uintptr_t>(dst0) & 15u) == 0) {
            u32x4* d4 = reinterpret_cast<u32x4*>(dst0);
            if constexpr (W == 4) {
                #pragma unroll
                for (int q = 0; q < NEPT / 4; q++) d4[q] = u32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
            } else {
                #pragma unroll
                for (int q = 0; q < NEPT / 2; q++)
                    d4[q] = u32x4{uint32_t(v[2 * q]), uint32_t(v[2 * q] >> 32), uint32_t(v[2 * q + 1]), uint32_t(v[2 * q + 1] >> 32)};
            }
        } else {
            for (uint32_t k = 0; k < m; k++) {
                uint32_t* d = reinterpret_cast<uint32_t*>(dst0 + uint64_t(k) * uint64_t(w));   // 4-byte aligned
                d[0] = uint32_t(v[k]);
                if constexpr (W == 8) d[1] = uint32_t(uint64_t(v[k]) >> 32);
            }
        }
    }
    if (ck.validity && fv) {
        const uint64_t abase = (slot_base + e_begin) & ~uint64_t(31);
        const uint64_t rb = slot_base + e - abase;
        const uint32_t sh = uint32_t(rb & 31);
        atomicOr(&S.vbits[rb >> 5], fv << sh);
        if (sh + NEPT > 32 && sh) atomicOr(&S.vbits[(rb >> 5) + 1], fv >> (32 - sh));
    }
    bad = __syncthreads_or(bad);
    if (bad) {
        if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi);
        return;
    }
    if (ck.validity) flush_bits(S.vbits, slot_base + e_begin, e_end - e_begin, ck.validity);
    if (tid == 0) {
        if (ck.needs_count == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&res[pg.chunk].num_values), (unsigned long long)tv);
        atomicOr(&pg.done, DONE_NULL);
    }
#ifdef PF_STAMPS
    NSTAMP(4);
    if (tid == 0) { PSTAMP(0, 1); PSTAMP(5, t_ph - t_beg); }
#endif
#undef NSTAMP
}

#ifdef PF_DIAG   // diagnostics build only (VERDICT r05 hygiene)
// k_page_null: one 512-thread workgroup per nullable flat page (fixed width 4 / 8, dictionary or
// PLAIN), for pages whose level section (<= LVL_STAGE bytes), level runs (<= PN_RUNS) and
// dictionary-id bytes (<= PN_IST) fit its LDS. It runs before k_lvl in the levels stage and does
// k_lvl's and k_flat_null's work for the page in one launch: the level and id sections are staged
// once, the level run headers are found by the all-positions chain (every byte decoded as a
// header, the chain from 0 followed in LDS), decoded in parallel and prefix-summed, and the page's
// 4096-entry blocks are then decoded in a loop (8 consecutive entries per thread, present bits ->
// block scan -> value index -> id from LDS -> gathers issued together -> 16-byte stores). The
// page's metadata chain, its section staging and the level parse are paid once per page instead of
// once per block, and k_lvl's one-wave block-table pass is gone. Anything it cannot decode
// exactly (a broken chain, an id past the dictionary, too many runs) leaves the page unmarked:
// k_lvl / k_flat_null / k_decode then take it and report it as before.
constexpr int PN_NT = 512;
constexpr uint32_t PN_RUNS = 512;        // level runs held in LDS
constexpr uint32_t PN_IST = 32768;       // dictionary-id bytes staged in LDS
constexpr uint32_t PN_MAX_BLOCKS = 16;   // entries <= 16 * FBLK
constexpr int PN_NEPT = FBLK / PN_NT;    // 8 consecutive entries per thread
struct PageNullLds {
    uint32_t lv[(LVL_STAGE + 64) / 4];
    uint16_t nxt[LVL_STAGE];
    Run drun[PN_RUNS];
    Run vrun[RUN_CAP];
    uint32_t ist[PN_IST / 4 + 8];
    uint32_t vbits[FBLK / 32 + 2];
    uint32_t scan_tmp[PN_NT / 64];
    uint32_t nh, ok, take;
};
__global__ __launch_bounds__(PN_NT) void k_page_null(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                    const int* __restrict__ list, DevChunkResult* res) {
    __shared__ __attribute__((aligned(16))) PageNullLds S;
    const int pi = list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    const uint32_t* T = pg.runtab;
    Sections s;
    const int w = ck.width;
    const bool dict = is_dict_enc(pg.encoding);
    const uint32_t ne = uint32_t(pg.num_values);
    // (uniform: every thread evaluates the same loads)
    bool take = pg.lvltab != nullptr && res[pg.chunk].status == 0 && ck.max_rep == 0 && ck.max_def > 0 &&
                (w == 4 || w == 8) && ck.values != nullptr && !(pg.done & (DONE_FIXED | DONE_NULL)) &&
                (dict || pg.encoding == 0) && ne > 0 && ne <= PN_MAX_BLOCKS * FBLK && page_sections(pg, ck, s) &&
                s.def_rle && s.def_n > 0 && s.def_n <= LVL_STAGE;
    uint32_t id_bw = 0, idn = 0, vnr = 0, idcov = 0;
    if (take && dict) {
        take = T != nullptr && T[2] == 1u && T[0] <= uint32_t(RUN_CAP) && T[0] > 0 && s.val_n > 1 && s.val[0] <= 32 &&
               s.val_n - 1 <= PN_IST && ck.dict_data != nullptr && ck.dict_n > 0;
        if (take) { id_bw = s.val[0]; idn = uint32_t(s.val_n - 1); vnr = T[0]; idcov = T[1]; }
    }
    if (!take) return;
    const int bw = bit_width(uint32_t(ck.max_def));
    const uint32_t maxd = uint32_t(ck.max_def);
    const uint32_t dn = uint32_t(s.def_n);
    // ---- stage: level bytes, id bytes, id runs (one round of loads)
    const uint32_t doff = stage_bytes(S.lv, s.def, dn, 0, dn);
    const uint32_t ioff = dict ? stage_bytes(S.ist, s.val + 1, idn, 0, idn) : 0u;
    for (uint32_t i = tid; i < vnr; i += PN_NT) {
        const uint32_t f = T[4 + 2 * i];
        const uint32_t nf = i + 1 < vnr ? (T[4 + 2 * (i + 1)] & 0x7fffffffu) : idcov;
        Run r;
        r.first = f & 0x7fffffffu;
        r.count = nf - r.first;
        r.data = T[5 + 2 * i];
        r.packed = f >> 31;
        S.vrun[i] = r;
    }
    __syncthreads();
    const uint8_t* lv8 = reinterpret_cast<const uint8_t*>(S.lv);
    const uint8_t* stw = lv8 + doff;   // stw[i] = level section byte i (zero past the section)
    // ---- level run headers: every byte position as a header (position of the next one)
    for (uint32_t p = tid; p < dn; p += PN_NT) {
        uint32_t h = 0, hl = 0, nx = 0xffffu;
        #pragma unroll
        for (uint32_t k = 0; k < 3; k++) {   // (a header of > 3 bytes counts > 2^20 entries: no run here)
            const uint32_t c = p + k < dn ? uint32_t(stw[p + k]) : 0x80u;
            h |= (c & 0x7fu) << (7 * k);
            if (!(c & 0x80u)) { hl = k + 1; break; }
        }
        if (hl) {
            const uint32_t pay = (h & 1u) ? (h >> 1) * uint32_t(bw) : (uint32_t(bw) + 7u) >> 3;
            if (p + hl + pay <= dn) nx = p + hl + pay;
        }
        S.nxt[p] = uint16_t(nx);
    }
    __syncthreads();
    if (tid == 0) {   // the chain from position 0 (one LDS load per run)
        uint32_t p = 0, nh = 0;
        bool ok = true;
        while (p < dn) {
            if (nh == PN_RUNS) { ok = false; break; }
            S.drun[nh++].data = p;   // header position (decoded below)
            const uint32_t q = S.nxt[p];
            if (q == 0xffffu) { ok = false; break; }   // no valid run at p
            p = q;
        }
        S.nh = nh;
        S.ok = ok ? 1u : 0u;
    }
    __syncthreads();
    if (!S.ok) return;   // k_lvl / k_decode take the page (and report what is wrong with it)
    const uint32_t nh = S.nh;
    {   // decode the headers in parallel; first entries by a block scan of the counts
        uint32_t cnt = 0, data = 0, packed = 0;
        bool bad = false;
        const uint32_t k = uint32_t(tid);
        if (k < nh) {
            const uint32_t P = S.drun[k].data;
            uint32_t h = 0, hl = 0;
            for (uint32_t b = 0; b < 3; b++) {
                const uint32_t c = stw[P + b];
                h |= (c & 0x7fu) << (7 * b);
                if (!(c & 0x80u)) { hl = b + 1; break; }
            }
            packed = h & 1u;
            cnt = packed ? (h >> 1) * 8u : (h >> 1);
            if (packed) data = (doff + P + hl) * 8u;   // LDS bit offset of the run's first level
            else {
                for (uint32_t b = 0; b < ((uint32_t(bw) + 7u) >> 3); b++) data |= uint32_t(stw[P + hl + b]) << (8 * b);
                bad = data > maxd;
            }
        }
        uint32_t tot;
        const uint32_t first = block_excl_scan<PN_NT>(cnt, S.scan_tmp, tot);
        if (k < nh) {
            Run r;
            r.first = first;
            r.count = cnt;
            r.data = data;
            r.packed = packed;
            S.drun[k] = r;
        }
        if (__syncthreads_or(bad || (tid == 0 && tot < ne))) return;
    }
    // ---- the page's blocks
    const uint64_t slot_base = uint64_t(pg.entry_start);
    const uint8_t* ist8 = reinterpret_cast<const uint8_t*>(S.ist);
    const uint32_t ilim = (ioff + idn) * 8u;   // staged id bits
    const uint32_t nblk = (ne + FBLK - 1) / FBLK;
    const uintptr_t da = reinterpret_cast<uintptr_t>(dict ? ck.dict_data : s.val);
    const bool galign = (da & uintptr_t(w - 1)) == 0;
    const int64_t dnn = dict ? ck.dict_n : 0;
    uint32_t vbase = 0;   // page-relative index of the block's first present value
    for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t e_begin = b * FBLK, e_end = min(ne, e_begin + FBLK);
        for (uint32_t i = tid; i < FBLK / 32 + 2; i += PN_NT) S.vbits[i] = 0;
        const uint32_t e = e_begin + uint32_t(tid) * PN_NEPT;
        const uint32_t m = e < e_end ? min(uint32_t(PN_NEPT), e_end - e) : 0u;
        uint32_t fv = 0;
        int bad = 0;
        if (m) {
            int r = run_find(S.drun, int(nh), e);
            const Run R = S.drun[r];
            if (e + m <= R.first + R.count && (!R.packed || bw == 1)) {   // one run
                if (!R.packed) fv = R.data == maxd ? ((1u << m) - 1u) : 0u;
                else fv = lds_bits(lv8, R.data + (e - R.first), m);
            } else {
                for (uint32_t k = 0; k < m; k++) {
                    while (r + 1 < int(nh) && e + k >= S.drun[r].first + S.drun[r].count) r++;
                    const Run& Rk = S.drun[r];
                    uint32_t dl = Rk.data;
                    if (Rk.packed) dl = lds_bits(lv8, Rk.data + (e + k - Rk.first) * uint32_t(bw), uint32_t(bw));
                    bad |= dl > maxd;
                    fv |= uint32_t(dl == maxd) << k;
                }
            }
        }
        uint32_t tv;
        const uint32_t vo = block_excl_scan<PN_NT>(__popc(fv), S.scan_tmp, tv);
        const uint32_t gv0 = vbase + vo;
        uint32_t idv[PN_NEPT];
        #pragma unroll
        for (int k = 0; k < PN_NEPT; k++) idv[k] = 0;
        if (fv) {
            if (dict) {
                if (gv0 + uint32_t(__popc(fv)) > idcov) bad = 1;
                int vr = run_find(S.vrun, int(vnr), gv0);
                uint32_t j = 0;
                #pragma unroll
                for (int k = 0; k < PN_NEPT; k++) {
                    if (!((fv >> k) & 1u)) continue;
                    const uint32_t gv = gv0 + j++;
                    while (vr + 1 < int(vnr) && gv >= S.vrun[vr].first + S.vrun[vr].count) vr++;
                    const Run& V = S.vrun[vr];
                    uint32_t id = V.data;
                    if (V.packed) {
                        const uint64_t bb = uint64_t(V.data) + uint64_t(ioff) * 8u + uint64_t(gv - V.first) * id_bw;
                        bad |= bb + id_bw > ilim;
                        id = bb + id_bw <= ilim ? lds_bits(ist8, uint32_t(bb), id_bw) : 0u;
                    }
                    bad |= int64_t(id) >= dnn;
                    idv[k] = int64_t(id) < dnn ? id : 0u;
                }
            } else {
                const uint32_t last = gv0 + uint32_t(__popc(fv)) - 1u;
                if (uint64_t(last + 1) * uint64_t(w) > s.val_n) bad = 1;
                #pragma unroll
                for (int k = 0; k < PN_NEPT; k++) idv[k] = bad ? 0u : min(gv0 + uint32_t(__popc(fv & ((1u << k) - 1u))), last);
            }
        }
        if (__syncthreads_or(bad)) return;   // (nothing counted or marked: the fallback redoes the page)
        uint64_t v[PN_NEPT];
        #pragma unroll
        for (int k = 0; k < PN_NEPT; k++) v[k] = 0;
        if (!fv) {
        } else if (galign) {
            if (w == 4) {
                const PF_GLOBAL uint32_t* g = (const PF_GLOBAL uint32_t*)da;
                #pragma unroll
                for (int k = 0; k < PN_NEPT; k++) v[k] = g[idv[k]];
            } else {
                const PF_GLOBAL uint64_t* g = (const PF_GLOBAL uint64_t*)da;
                #pragma unroll
                for (int k = 0; k < PN_NEPT; k++) v[k] = g[idv[k]];
            }
        } else {
            #pragma unroll
            for (int k = 0; k < PN_NEPT; k++) {
                const uint8_t* src = reinterpret_cast<const uint8_t*>(da) + uint64_t(idv[k]) * uint64_t(w);
                v[k] = w == 4 ? uint64_t(ld_u32_any(src)) : ld_u64_any(src);
            }
        }
        #pragma unroll
        for (int k = 0; k < PN_NEPT; k++)
            if (!((fv >> k) & 1u)) v[k] = 0;
        if (m) {
            uint8_t* dst0 = ck.values + (slot_base + e) * uint64_t(w);
            if (m == PN_NEPT && (reinterpret_cast<uintptr_t>(dst0) & 15u) == 0) {
                u32x4* d4 = reinterpret_cast<u32x4*>(dst0);
                if (w == 4) {
                    d4[0] = u32x4{uint32_t(v[0]), uint32_t(v[1]), uint32_t(v[2]), uint32_t(v[3])};
                    d4[1] = u32x4{uint32_t(v[4]), uint32_t(v[5]), uint32_t(v[6]), uint32_t(v[7])};
                } else {
                    #pragma unroll
                    for (int q = 0; q < 4; q++)
                        d4[q] = u32x4{uint32_t(v[2 * q]), uint32_t(v[2 * q] >> 32), uint32_t(v[2 * q + 1]), uint32_t(v[2 * q + 1] >> 32)};
                }
            } else {
                for (uint32_t k = 0; k < m; k++) {
                    uint32_t* d = reinterpret_cast<uint32_t*>(dst0 + uint64_t(k) * uint64_t(w));   // 4-byte aligned
                    d[0] = uint32_t(v[k]);
                    if (w == 8) d[1] = uint32_t(v[k] >> 32);
                }
            }
        }
        if (ck.validity && fv) {
            const uint64_t abase = (slot_base + e_begin) & ~uint64_t(31);
            const uint64_t rb = slot_base + e - abase;
            const uint32_t sh = uint32_t(rb & 31);
            atomicOr(&S.vbits[rb >> 5], fv << sh);
            if (sh + PN_NEPT > 32 && sh) atomicOr(&S.vbits[(rb >> 5) + 1], fv >> (32 - sh));
        }
        __syncthreads();
        if (ck.validity) flush_bits(S.vbits, slot_base + e_begin, e_end - e_begin, ck.validity);
        vbase += tv;
        __syncthreads();   // (vbits / scan_tmp reused by the next block)
    }
    if (tid == 0) {
        if (ck.needs_count == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&res[pg.chunk].num_values), (unsigned long long)vbase);
        atomicOr(&pg.done, DONE_NULL | DONE_PAGE);
    }
}
#endif  // PF_DIAG

// ---- nested pages in segments (k_nest_*) --------------------------------------------------------
// A nested page's levels are walked run by run from its first entry, so k_count / k_decode take it in
// ONE workgroup tile after tile: a 520K-entry page (one per chunk in config 5) runs ~1000 tiles in
// series on one CU. Here the page is cut into segments of seg_len entries, each decoded by its own
// workgroup from checkpoints of the three hybrid streams (rep, def, dictionary ids):
//   k_nest_lvl   (page x {rep, def} x 8 KiB window): every window position decoded as a run header,
//                pointer jumping to the window exits, a single-pass hand-over between windows, and
//                the state at every segment start;
//   k_count_seg  (page x segment): slots / values / rows of the segment's levels;
//   k_nest_scan  (page, one wave): their prefixes over the page, the page totals (k_scan), and the
//                dictionary-id stream's state at each segment's first value;
//   k_nest_ids   (page x segment, BYTE_ARRAY dictionary): ids kept for k_decode_seg, chars;
//   k_nest_chars (page, one wave): the segments' chars prefix, the page's chars;
//   k_decode_seg (page x segment): decode_page over the segment.
// Checkpoint states are exactly rle_walk's state after the segment's first t values (mid-run when t
// falls inside a run), so each segment's decode is the serial walk's, from t on.
constexpr uint32_t NW_BYTES = 8192;   // nest_walk's LDS window over a stream (k_nest_scan)
static_assert(sizeof(RleState) == NEST_CK_BYTES, "checkpoint size (host plans the segment tables)");

__device__ __forceinline__ RleState* nest_ck(const DevPage& pg, int k) {
    return reinterpret_cast<RleState*>(pg.seg) + size_t(k) * size_t(pg.nseg);
}
__device__ __forceinline__ SegRec* nest_rec(const DevPage& pg) {
    return reinterpret_cast<SegRec*>(pg.seg + 3ull * NEST_CK_BYTES * uint64_t(pg.nseg));
}
__device__ __forceinline__ RleState rle_sentinel() {   // a target the stream never reached: walking from it fails
    RleState s;
    rle_init(s);
    s.pos = ~uint64_t(0);
    s.err = 1;
    return s;
}

// One wave: walk the hybrid stream p[0, n) (bit width bw) from byte pos0 (a run header), and store in
// out[k] the state after target(k) values, k < nt (targets non-decreasing). Targets the stream does
// not reach (it ends, breaks, or holds fewer values) get rle_sentinel(). All lanes walk in step (the
// LDS reads broadcast); lane 0 writes.
template <typename Target>
__device__ void nest_walk(uint32_t* st, const uint8_t* p, uint64_t n, int bw, uint64_t pos0, int nt, Target target,
                          RleState* out) {
    const int lane = threadIdx.x & 63;
    int k = 0;
    uint64_t e = 0, pos = pos0;
    uint64_t wb = ~uint64_t(0);   // stream offset of the window's first byte (st byte woff)
    uint32_t woff = 0;
    const uint8_t* W = reinterpret_cast<const uint8_t*>(st);
    const int nbv = (bw + 7) >> 3;
    uint64_t t = nt > 0 ? target(0) : 0;
    while (k < nt && pos < n) {
        if (wb == ~uint64_t(0) || pos < wb || pos + 16 > wb + NW_BYTES) {
            __syncthreads();
            wb = pos;
            woff = stage_bytes(st, p, n, uint32_t(pos), uint32_t(min<uint64_t>(n, pos + NW_BYTES)));
            __syncthreads();
        }
        // header (uvarint, <= 10 bytes) and an RLE value (<= 4 bytes) lie inside the window
        const uint8_t* q = W + woff + (pos - wb);
        uint64_t h = 0;
        uint32_t hl = 0;
        bool hok = false;
        for (uint32_t sh = 0; sh < 70; sh += 7) {
            if (pos + hl >= n) break;
            const uint32_t c = q[hl++];
            h |= uint64_t(c & 0x7f) << sh;
            if (!(c & 0x80)) { hok = true; break; }
        }
        if (!hok) break;
        const uint64_t a = pos + hl;
        uint64_t cnt, next, bit0 = 0;
        uint32_t val = 0;
        const uint32_t packed = uint32_t(h & 1);
        if (packed) {
            const uint64_t groups = h >> 1;
            cnt = groups * 8;
            bit0 = a * 8;
            const uint64_t nb = groups * uint64_t(bw), avail = n - a;
            next = a + (nb < avail ? nb : avail);
        } else {
            cnt = h >> 1;
            if (a + nbv > n) break;
            for (int b = 0; b < nbv; b++) val |= uint32_t(q[hl + b]) << (8 * b);
            next = a + nbv;
        }
        while (k < nt && t < e + cnt) {
            if (lane == 0) {
                RleState r;
                r.pos = next;
                r.run_left = e + cnt - t;
                r.run_bit = packed ? bit0 + (t - e) * uint64_t(bw) : 0;
                r.run_val = val;
                r.run_packed = int32_t(packed);
                r.err = 0;
                out[k] = r;
            }
            k++;
            if (k < nt) t = target(k);
        }
        e += cnt;
        pos = next;
    }
    for (; k < nt; k++)
        if (lane == 0) out[k] = rle_sentinel();
}

// the page's segment path applies: rep / def sections parse and are RLE hybrid streams
__device__ __forceinline__ bool nest_sections(const DevPage& pg, const DevChunk& ck, Sections& s) {
    return pg.seg != nullptr && ck.max_rep > 0 && page_sections(pg, ck, s) && s.rep_rle && (ck.max_def == 0 || s.def_rle);
}

// One hybrid-stream run header at stream position p (q = its bytes, >= 14 readable): false when p
// holds no run the serial walk (rle_walk) would accept.
struct HybRun {
    uint64_t cnt, next, bit0;
    uint32_t val, packed;
};
__device__ __forceinline__ bool hyb_header(const uint8_t* q, uint64_t p, uint64_t n, int bw, HybRun& r) {
    uint64_t h = 0;
    uint32_t hl = 0;
    bool hok = false;
    for (uint32_t sh = 0; sh < 70; sh += 7) {
        if (p + hl >= n) break;
        const uint32_t c = q[hl++];
        h |= uint64_t(c & 0x7f) << sh;
        if (!(c & 0x80)) { hok = true; break; }
    }
    if (!hok) return false;
    const uint64_t a = p + hl;
    r.packed = uint32_t(h & 1);
    r.val = 0;
    r.bit0 = 0;
    if (r.packed) {
        const uint64_t groups = h >> 1;
        r.cnt = groups * 8;
        r.bit0 = a * 8;
        const uint64_t nb = groups * uint64_t(bw), avail = n - a;
        r.next = a + (nb < avail ? nb : avail);
    } else {
        const int nbv = (bw + 7) >> 3;
        r.cnt = h >> 1;
        if (a + nbv > n) return false;
        for (int b = 0; b < nbv; b++) r.val |= uint32_t(q[hl + b]) << (8 * b);
        r.next = a + nbv;
    }
    return true;
}
__device__ __forceinline__ RleState hyb_state(const HybRun& r, uint64_t e_start, uint64_t t, int bw) {
    RleState x;
    x.pos = r.next;
    x.run_left = e_start + r.cnt - t;
    x.run_bit = r.packed ? r.bit0 + (t - e_start) * uint64_t(bw) : 0;
    x.run_val = r.val;
    x.run_packed = int32_t(r.packed);
    x.err = 0;
    return x;
}

// k_nest_lvl: NL_NT threads per NEST_WIN-byte window of a page's rep or def stream. Run headers can
// only be found by walking from the stream's start, so every byte position of the window is decoded
// as a header at once, and pointer jumping (log2(NEST_WIN) rounds in LDS) gives, for every position,
// where the chain from it leaves the window and the entries it covers on the way (north_star K2: run
// boundaries by parallel scans). The true chain's entry position and count then come from the
// previous window (single-pass hand-over through npub: one lookup per window on the critical path),
// and the window walks its part of the true chain to store the checkpoints inside it (states at
// multiples of seg_len entries) after publishing its exit.
constexpr int NL_NT = 256;
constexpr uint32_t NL_END = 0xFFFFFFu;        // exit field: the chain ends inside the window (no run at its last position)
constexpr uint32_t NL_FAR = 0xFFFFFEu;        // exit field: leaves the window for a position >= w0 + NL_FAR (exact exit by a walk)
constexpr uint64_t NL_CMAX = (1ull << 40) - 1;   // count field saturates (the exact count is then walked)
constexpr uint32_t NL_JNONE = 0xFFFu, NL_JCMAX = 0xFFFFFu;   // J: no exit inside the window; saturated entries
static_assert(NEST_WIN <= 2048, "J packs window-relative exits in 12 bits");
__global__ __launch_bounds__(NL_NT) void k_nest_lvl(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list,
                                                    DevChunkResult* res, uint32_t spin_cap) {
    __shared__ __attribute__((aligned(16))) uint32_t st[(NEST_WIN + 64) / 4];
    __shared__ uint64_t X[NEST_WIN];   // per position: entries to the exit << 24 | exit (window-relative, NL_END, NL_FAR)
    // the same after 5 rounds, packed in 32 bits: jumps over >= 32 runs (or to the exit), for the checkpoint
    // walk; exit in the low 12 bits (NL_JNONE: none inside the window), entries (saturating) above
    __shared__ uint32_t J[NEST_WIN];
    __shared__ uint64_t s_hand[3];
    const int tid = threadIdx.x;
    const int pi = list[blockIdx.z];
    const int which = blockIdx.y;   // 0 = rep, 1 = def
    const uint32_t w = blockIdx.x;
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    Sections s;
    if (res[pg.chunk].status != 0 || !nest_sections(pg, ck, s) || w >= uint32_t(pg.nwin)) return;   // (seg_ok stays 0)
    const int nseg = pg.nseg;
    const uint64_t sl = uint64_t(uint32_t(pg.seg_len));
    RleState* out = nest_ck(pg, which);
    // (max: a window that timed out waiting for its hand-over may already have set 2 = failed)
    if (which == 0 && w == 0 && tid == 0) __hip_atomic_fetch_max(&pg.seg_ok, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (which == 1 && ck.max_def == 0) {
        if (w == 0) for (int k = tid; k < nseg; k += NL_NT) { RleState r; rle_init(r); out[k] = r; }
        return;
    }
    const uint8_t* p = which == 0 ? s.rep : s.def;
    const uint64_t n = which == 0 ? s.rep_n : s.def_n;
    const int bw = bit_width(uint32_t(which == 0 ? ck.max_rep : ck.max_def));
    const uint64_t w0 = uint64_t(w) * NEST_WIN, w1 = w0 + NEST_WIN;
    if (w0 >= n && w > 0) return;                  // past the stream (no one waits on it)
    const bool last = w1 >= n;                     // writes the sentinels of targets the chain never reached
    WinPub* pub = pg.npub + size_t(which) * size_t(pg.nwin);
    // ---- stage the window (+ 16 bytes: a header and an RLE value that start inside it) ----
    const uint32_t woff = stage_bytes(st, p, n, uint32_t(min<uint64_t>(w0, n)), uint32_t(min<uint64_t>(w1 + 16, n)));
    __syncthreads();
    const uint8_t* W = reinterpret_cast<const uint8_t*>(st) + woff;   // W[i] = stream byte w0 + i
    // ---- every position as a header, then pointer jumping to the window's exit ----
    for (uint32_t i = tid; i < NEST_WIN; i += NL_NT) {
        const uint64_t pp = w0 + i;
        HybRun r;
        uint64_t x = NL_END;
        if (pp < n && hyb_header(W + i, pp, n, bw, r)) {
            const uint64_t rel = r.next - w0;
            x = (min<uint64_t>(r.cnt, NL_CMAX) << 24) | (rel < NL_FAR ? rel : uint64_t(NL_FAR));
        }
        X[i] = x;
    }
    __syncthreads();
    for (uint32_t span = 1; span < NEST_WIN; span <<= 1) {
        for (uint32_t i = tid; i < NEST_WIN; i += NL_NT) {
            const uint64_t x = X[i];
            const uint32_t e = uint32_t(x & 0xFFFFFFu);
            if (e < NEST_WIN) {   // (in place: a successor already advanced this round only jumps further)
                const uint64_t y = X[e];
                const uint64_t c = min<uint64_t>((x >> 24) + (y >> 24), NL_CMAX);
                X[i] = (c << 24) | (y & 0xFFFFFFu);
            }
        }
        __syncthreads();
        if (span == 16) {
            for (uint32_t i = tid; i < NEST_WIN; i += NL_NT) {
                const uint64_t x = X[i];
                const uint32_t e = uint32_t(x & 0xFFFFFFu);
                J[i] = (e < NEST_WIN ? e : NL_JNONE) | (uint32_t(min<uint64_t>(x >> 24, NL_JCMAX)) << 12);
            }
        }
    }
    __syncthreads();
    // ---- the true chain's entry from the previous window; exit to the next ----
    if (tid == 0) {
        uint64_t tp = 0, te = 0;
        uint32_t tst = 0;
        bool ok = true;
        // bounded (spin_cap: 2^22; the diagnostics option nest_timeout makes it 0, so every hand-over
        // "times out"): a hand-over that never comes sends the page to the whole-page path (below)
        // instead of hanging
        if (w > 0) ok = winpub_get(pub[w - 1], spin_cap, tp, te, tst);
        s_hand[0] = tp; s_hand[1] = te; s_hand[2] = uint64_t(tst) | (ok ? 0u : 2u);
        uint64_t xp = tp, xe = te;
        uint32_t xst = tst;
        if (ok && tst == 0 && tp < w1) {
            const uint64_t x = X[tp - w0];
            const uint32_t e = uint32_t(x & 0xFFFFFFu);
            const uint64_t c = x >> 24;
            if (e == NL_FAR || c == NL_CMAX) {   // exact exit / count by walking (a run of > 16 MB, or counts near 2^40)
                while (xp < w1) {
                    HybRun r;
                    if (xp >= n || !hyb_header(W + (xp - w0), xp, n, bw, r)) { xst = 1; break; }
                    xe += r.cnt;
                    xp = r.next;
                }
            } else {
                xe = te + c;
                if (e == NL_END) { xst = 1; xp = w1; }   // (where it ended does not matter once it has)
                else xp = w0 + e;
            }
        }
        // a hand-over that never came (a scheduling stall, not the data): the page leaves the segment
        // path and k_count / k_decode decode it whole, as k_dbp_pos does with dbp_ok = 2
        if (!ok) __hip_atomic_fetch_max(&pg.seg_ok, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // a failed hand-over is published as the overflow word, so every later window fails at once
        winpub_put(pub[w], ok ? xp : ~0ull, xe, xst);
    }
    __syncthreads();
    if (s_hand[2] & 2u) return;
    // ---- checkpoints inside the window: one wave walks its part of the true chain ----
    uint64_t tp = s_hand[0], te = s_hand[1];
    uint32_t tst = uint32_t(s_hand[2]);
    if (tid < 64) {   // (all 64 lanes walk in step; lane 0 stores)
        uint64_t k = (te + sl - 1) / sl;   // first target >= te
        if (tst == 0) {
            while (k < uint64_t(nseg) && tp < w1) {
                const uint64_t t = k * sl;
                // jump over runs before the target: >= 32 at a time
                while (true) {
                    const uint32_t x = J[tp - w0];
                    const uint32_t e = x & 0xFFFu, c = x >> 12;
                    if (e >= NEST_WIN || c == NL_JCMAX || te + c > t) break;   // (saturated: the header walk)
                    te += c;
                    tp = w0 + e;
                }
                HybRun r;
                if (tp >= n || !hyb_header(W + (tp - w0), tp, n, bw, r)) { tst = 1; break; }
                if (t < te + r.cnt) {   // the target's run
                    if (tid == 0) out[k] = hyb_state(r, te, t, bw);
                    k++;
                    continue;
                }
                te += r.cnt;
                tp = r.next;
            }
        }
        // targets the chain never reached: the stream's last window, or the window where it ended
        if (last || tst == 1)
            for (uint64_t q = k + tid; q < uint64_t(nseg); q += 64) out[q] = rle_sentinel();
    }
}

__global__ __launch_bounds__(NT) void k_count_seg(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                  const int2* __restrict__ list, DevChunkResult* res) {
    __shared__ LevelLds L;
    __shared__ uint32_t scan_tmp[NT / 64];
    const int pi = list[blockIdx.x].x, sg = list[blockIdx.x].y;
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (pg.seg_ok != 1 || res[pg.chunk].status != 0) return;
    __shared__ uint32_t bufR[SEG_LVL_CAP / 4], bufD[SEG_LVL_CAP / 4];
    Sections s;
    page_sections(pg, ck, s);   // (parsed by k_nest_lvl)
    const uint64_t e_b = uint64_t(sg) * uint32_t(pg.seg_len);
    const uint64_t e_e = min<uint64_t>(uint64_t(pg.num_values), e_b + uint32_t(pg.seg_len));
    {
        const RleState* cr = nest_ck(pg, 0);
        const RleState* cd = nest_ck(pg, 1);
        const bool last = sg + 1 >= pg.nseg;
        const uint64_t lr = stage_seg(bufR, SEG_LVL_CAP, s.rep, s.rep_n, cr[sg], last ? nullptr : &cr[sg + 1]);
        const uint64_t ld = ck.max_def > 0 ? stage_seg(bufD, SEG_LVL_CAP, s.def, s.def_n, cd[sg], last ? nullptr : &cd[sg + 1]) : 0;
        if (threadIdx.x == 0) {
            L.srep = cr[sg]; L.sdef = cd[sg]; L.err = 0;
            rle_rebase(L.srep, lr); rle_rebase(L.sdef, ld);
        }
    }
    __syncthreads();
    uint64_t slots = 0, vals = 0, rows = 0;
    for (uint64_t e0 = e_b; e0 < e_e; e0 += TILE) {
        const uint32_t want = uint32_t(min<uint64_t>(TILE, e_e - e0));
        decode_level_tile(L, s, ck, e0, want);
        if (L.err) break;
        uint32_t ns = 0, nv = 0, nr = 0;
        for (uint32_t i = threadIdx.x; i < want; i += NT) {
            const int d = L.def[i];
            ns += d >= ck.repeated_def;
            nv += d == ck.max_def;
            nr += L.rep[i] == 0;
        }
        uint32_t t;
        block_excl_scan<NT>(ns, scan_tmp, t); slots += t;
        block_excl_scan<NT>(nr, scan_tmp, t); rows += t;
        block_excl_scan<NT>(nv, scan_tmp, t); vals += t;
        __syncthreads();
    }
    if (L.err) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    if (threadIdx.x == 0) {
        SegRec& r = nest_rec(pg)[sg];
        r.ns = uint32_t(slots); r.nv = uint32_t(vals); r.nr = uint32_t(rows); r.chars = 0;
    }
}

__global__ __launch_bounds__(64) void k_nest_scan(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list,
                                                  DevChunkResult* res) {
    __shared__ __attribute__((aligned(16))) uint32_t st[(NW_BYTES + 64) / 4];
    __shared__ uint32_t vb[NEST_MAX_SEGS];
    const int pi = list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (pg.seg_ok != 1 || res[pg.chunk].status != 0) return;
    const int nseg = pg.nseg, lane = threadIdx.x;
    SegRec* R = nest_rec(pg);
    uint64_t cs = 0, cv = 0, cr = 0;
    for (int k0 = 0; k0 < nseg; k0 += 64) {
        const int k = k0 + lane;
        uint64_t ns = 0, nv = 0, nr = 0;
        if (k < nseg) { ns = R[k].ns; nv = R[k].nv; nr = R[k].nr; }
        uint64_t xs = ns, xv = nv, xr = nr;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t ys = __shfl_up(xs, d, 64), yv = __shfl_up(xv, d, 64), yr = __shfl_up(xr, d, 64);
            if (lane >= d) { xs += ys; xv += yv; xr += yr; }
        }
        if (k < nseg) {
            R[k].sb = uint32_t(cs + xs - ns); R[k].vb = uint32_t(cv + xv - nv); R[k].rb = uint32_t(cr + xr - nr);
            vb[k] = uint32_t(cv + xv - nv);
        }
        cs += __shfl(xs, 63, 64); cv += __shfl(xv, 63, 64); cr += __shfl(xr, 63, 64);
    }
    if (lane == 0) { pg.n_slots = int64_t(cs); pg.n_values = int64_t(cv); pg.n_rows = int64_t(cr); pg.n_chars = 0; }
    __syncthreads();
    // dictionary ids: the stream's state at each segment's first value
    if (is_dict_enc(pg.encoding)) {
        Sections s;
        page_sections(pg, ck, s);
        RleState* out = nest_ck(pg, 2);
        const int id_bw = s.val_n > 0 ? int(s.val[0]) : 0;
        if (s.val_n == 0 || id_bw > 32) {
            for (int k = lane; k < nseg; k += 64) out[k] = rle_sentinel();   // (decode reports it)
        } else {
            nest_walk(st, s.val, s.val_n, id_bw, 1, nseg, [](int k) { return uint64_t(vb[k]); }, out);
        }
    }
}

__global__ __launch_bounds__(NT) void k_nest_ids(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                 const int2* __restrict__ list, DevChunkResult* res) {
    __shared__ Piece pval[TILE];
    __shared__ uint32_t ids[TILE];
    __shared__ RleState sval;
    __shared__ int npval, verr;
    __shared__ unsigned long long chars_acc;
    const int pi = list[blockIdx.x].x, sg = list[blockIdx.x].y;
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (pg.seg_ok != 1 || res[pg.chunk].status != 0 || ck.ptype != 6 || !is_dict_enc(pg.encoding)) return;
    Sections s;
    page_sections(pg, ck, s);
    SegRec& rec = nest_rec(pg)[sg];
    const uint64_t v_b = rec.vb, v_e = v_b + rec.nv;
    const int id_bw = s.val_n > 0 ? int(s.val[0]) : 0;
    __shared__ uint32_t bufV[SEG_VAL_CAP / 4];
    const RleState* cv = nest_ck(pg, 2);
    const uint64_t lv = v_e > v_b ? stage_seg(bufV, SEG_VAL_CAP, s.val, s.val_n, cv[sg], sg + 1 < pg.nseg ? &cv[sg + 1] : nullptr) : 0;
    if (threadIdx.x == 0) { sval = cv[sg]; rle_rebase(sval, lv); verr = 0; chars_acc = 0; }
    __syncthreads();
    for (uint64_t v0 = v_b; v0 < v_e; v0 += TILE) {
        const uint32_t t = uint32_t(min<uint64_t>(TILE, v_e - v0));
        if (threadIdx.x == 0) {
            if (id_bw > 32 || !ck.dict_len) verr = 1;
            else {
                const uint32_t got = rle_walk(sval, s.val, s.val_n, id_bw, t, pval, TILE, npval);
                if (got != t || sval.err) verr = 1;
            }
        }
        __syncthreads();
        if (verr) break;
        rle_expand<uint32_t>(pval, npval, s.val, s.val_n, id_bw, ids);
        __syncthreads();
        uint64_t acc = 0;
        int bad = 0;
        for (uint32_t i = threadIdx.x; i < t; i += NT) {
            const uint32_t id = ids[i];
            if (int64_t(id) >= ck.dict_n) { bad = 1; continue; }
            acc += ck.dict_len[id];
            pg.aux[v0 + i] = id;
        }
        if (__syncthreads_or(bad)) { if (threadIdx.x == 0) verr = 1; __syncthreads(); break; }
        atomicAdd(&chars_acc, (unsigned long long)acc);
        __syncthreads();
    }
    if (verr) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    __syncthreads();
    if (threadIdx.x == 0) rec.chars = chars_acc;
}

__global__ __launch_bounds__(64) void k_nest_chars(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list,
                                                   DevChunkResult* res) {
    const int pi = list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (pg.seg_ok != 1 || res[pg.chunk].status != 0 || ck.ptype != 6) return;
    const int nseg = pg.nseg, lane = threadIdx.x;
    SegRec* R = nest_rec(pg);
    uint64_t cc = 0;
    for (int k0 = 0; k0 < nseg; k0 += 64) {
        const int k = k0 + lane;
        const uint64_t c = k < nseg ? R[k].chars : 0;
        uint64_t x = c;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (k < nseg) R[k].cb = cc + x - c;
        cc += __shfl(x, 63, 64);
    }
    if (lane == 0) pg.n_chars = int64_t(cc);
}

#ifndef PF_DSEG_WAVES
#define PF_DSEG_WAVES 4
#endif
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PF_DSEG_WAVES))) void k_decode_seg(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                   const int2* __restrict__ list, DevChunkResult* res) {
    __shared__ DecodeLds S;
    __shared__ uint32_t bufR[SEG_LVL_CAP / 4], bufD[SEG_LVL_CAP / 4], bufV[SEG_VAL_CAP / 4];
    const int pi = list[blockIdx.x].x, sg = list[blockIdx.x].y;
    const DevPage& pg = pages[pi];
    if (pg.seg_ok != 1) return;
    const SegRec& rec = nest_rec(pg)[sg];
    DecodeRange R;
    R.e_b = uint64_t(sg) * uint32_t(pg.seg_len);
    R.e_e = min<uint64_t>(uint64_t(pg.num_values), R.e_b + uint32_t(pg.seg_len));
    R.slot_base = rec.sb; R.row_base = rec.rb; R.vidx = rec.vb;
    R.char_base = chunks[pg.chunk].ptype == 6 ? rec.cb : 0;
    R.st = nest_ck(pg, 0) + sg;
    R.nx = sg + 1 < pg.nseg ? R.st + 1 : nullptr;
    R.nseg = pg.nseg;
    R.buf[0] = bufR; R.buf[1] = bufD; R.buf[2] = bufV;
    decode_page(chunks, pages, pi, res, S, &R);
}

// ---- launchers -------------------------------------------------------------------------------
void launch_nest_lvl(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, int max_nwin, DevChunkResult* d_res,
                     hipStream_t st, bool force_timeout) {
    // windows in blockIdx.x: a window waits on the one before it, which the dispatcher starts first
    if (n > 0 && max_nwin > 0)
        hipLaunchKernelGGL(k_nest_lvl, dim3(max_nwin, 2, n), dim3(NL_NT), 0, st, d_chunks, d_pages, d_list, d_res,
                           force_timeout ? 0u : (1u << 22));
}
void launch_nest_count(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, const int2* d_segs, int n_segs,
                       DevChunkResult* d_res, hipStream_t st) {
    if (n <= 0 || n_segs <= 0) return;
    hipLaunchKernelGGL(k_count_seg, dim3(n_segs), dim3(NT), 0, st, d_chunks, d_pages, d_segs, d_res);
    hipLaunchKernelGGL(k_nest_scan, dim3(n), dim3(64), 0, st, d_chunks, d_pages, d_list, d_res);
    hipLaunchKernelGGL(k_nest_ids, dim3(n_segs), dim3(NT), 0, st, d_chunks, d_pages, d_segs, d_res);
    hipLaunchKernelGGL(k_nest_chars, dim3(n), dim3(64), 0, st, d_chunks, d_pages, d_list, d_res);
}
void launch_nest_decode(const DevChunk* d_chunks, DevPage* d_pages, const int2* d_segs, int n_segs, DevChunkResult* d_res,
                        hipStream_t st) {
    if (n_segs > 0) hipLaunchKernelGGL(k_decode_seg, dim3(n_segs), dim3(NT), 0, st, d_chunks, d_pages, d_segs, d_res);
}
void launch_count(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, int n_flat, const int2* d_dblk, int n_dblk,
                  DevChunkResult* d_res, BaJob* d_bajobs, hipStream_t st, int idle_grid) {
    // d_list: the n_flat flat BYTE_ARRAY pages (k_count_flat's grid; none: no launch) first, then the
    // other pages that need counts. d_dblk: (page, block) pairs of the flat dictionary BYTE_ARRAY
    // pages (k_count_dict, before k_count_flat)
    if (n <= 0) return;
    if (n_dblk > 0) hipLaunchKernelGGL(k_count_dict, dim3(n_dblk), dim3(NT), 0, st, d_chunks, d_pages, d_dblk, d_res);
    if (n_flat > 0) hipLaunchKernelGGL(k_count_flat, dim3(n_flat), dim3(NT), 0, st, d_chunks, d_pages, d_list, d_res, d_bajobs);
    hipLaunchKernelGGL(k_count, dim3(std::min(n, idle_grid)), dim3(NT), 0, st, d_chunks, d_pages, d_list, n, d_res, d_bajobs);
}
// PLAIN BYTE_ARRAY walks of jobs [0, n_jobs) over tiles [0, n_tiles).
void launch_ba(BaJob* d_jobs, int n_jobs, const int2* d_tiles, int n_tiles, DevChunkResult* d_res, hipStream_t st,
               bool short_values) {
    if (n_jobs <= 0 || n_tiles <= 0) return;
    // candidates, both link levels, the count and the chain check in one kernel (k_ba_tile) for batches
    // of short values (short_values; the diagnostics option ba_fused=0 clears it); otherwise the round-3 kernels
    const bool fused = short_values;
    if (!fused) {
        hipLaunchKernelGGL(k_ba_cand, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles);
        hipLaunchKernelGGL(k_ba_link, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles, 1);
        hipLaunchKernelGGL(k_ba_link, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles, 2);
        hipLaunchKernelGGL(k_ba_count, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles);
    } else {
        hipLaunchKernelGGL(k_ba_tile, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles);
    }
    hipLaunchKernelGGL(k_ba_scan, dim3(n_jobs), dim3(NT), 0, st, d_jobs, fused ? int32_t(BA_RELINK) : int32_t(BA_FALLBACK));
    hipLaunchKernelGGL(k_ba_emit, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles);
    if (!fused) hipLaunchKernelGGL(k_ba_verify, dim3(n_tiles), dim3(NT), 0, st, d_jobs, d_tiles);
    hipLaunchKernelGGL(k_ba_fallback, dim3(std::min(n_jobs, 64)), dim3(NT), 0, st, d_jobs, n_jobs, d_res);
}
#ifdef PF_DIAG   // diagnostics build only (VERDICT r05 hygiene)
// Diagnostics (tests/test_gpu_runs.py): walk_runs (one lane) and wave_walk_runs (one wave) over the
// same stream; out = {ret, nruns, covered, pos, first, runs[cap] x 4} for each.
__global__ __launch_bounds__(64) void k_debug_walk(const uint8_t* p, uint64_t n, int bw, uint32_t lo, uint32_t limit, int cap,
                                                    uint32_t pos0, uint32_t first0, uint32_t* out) {
    __shared__ Run R[RUN_CAP];
    __shared__ int s_nr;
    __shared__ uint32_t s_cov;
    __shared__ RunWalk s_st;
    const int tid = threadIdx.x;
    uint32_t* o1 = out;
    uint32_t* o2 = out + 5 + 4 * cap;
    if (tid == 0) {
        RunWalk st{pos0, first0};
        int nr = 0;
        uint32_t cov = 0;
        const int r = walk_runs(p, n, bw, lo, limit, R, cap, nr, cov, st);
        o1[0] = uint32_t(r); o1[1] = uint32_t(nr); o1[2] = cov; o1[3] = uint32_t(st.pos); o1[4] = st.first;
        for (int i = 0; i < nr; i++) { o1[5 + 4 * i] = R[i].first; o1[6 + 4 * i] = R[i].count; o1[7 + 4 * i] = R[i].data; o1[8 + 4 * i] = R[i].packed; }
        s_st = RunWalk{pos0, first0};
    }
    __syncthreads();
    const int r = wave_walk_runs(p, n, bw, lo, limit, R, cap, s_nr, s_cov, s_st, RunWalk{pos0, first0});
    __syncthreads();
    if (tid == 0) {
        o2[0] = uint32_t(r); o2[1] = uint32_t(s_nr); o2[2] = s_cov; o2[3] = uint32_t(s_st.pos); o2[4] = s_st.first;
    }
    for (int i = tid; i < s_nr; i += 64) { o2[5 + 4 * i] = R[i].first; o2[6 + 4 * i] = R[i].count; o2[7 + 4 * i] = R[i].data; o2[8 + 4 * i] = R[i].packed; }
}

extern "C" int pf_debug_walk_runs(const uint8_t* stream, uint64_t n, int bw, uint32_t lo, uint32_t limit, int cap,
                                  uint32_t pos0, uint32_t first0, uint32_t* out) {
    if (cap > int(RUN_CAP) || cap < 0) return -1;
    uint8_t* d = nullptr;
    uint32_t* o = nullptr;
    const size_t ob = 4 * size_t(2 * (5 + 4 * cap));
    if (hipMalloc(&d, n + 64) != hipSuccess) return -1;
    if (hipMalloc(&o, ob) != hipSuccess) { (void)hipFree(d); return -1; }
    int rc = 0;
    if (hipMemset(d, 0, n + 64) != hipSuccess || hipMemcpy(d, stream, n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(o, 0, ob) != hipSuccess)
        rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(k_debug_walk, dim3(1), dim3(64), 0, 0, d, n, bw, lo, limit, cap, pos0, first0, o);
        if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(out, o, ob, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    }
    (void)hipFree(d);
    (void)hipFree(o);
    return rc;
}
#endif  // PF_DIAG

// Dictionary pages that are one Snappy literal (k_snappy_head: FB_LITCOPY): the literal's bytes to
// the page's 16-byte aligned scratch body, 16 bytes per thread per step (aligned dword loads +
// v_alignbyte), LC_SPLIT workgroups per page. The job's literals (k_snappy_head's table in its token
// bitmap: {data offset, output offset} per literal) are found by a binary search per 16-byte chunk;
// a chunk spanning two literals is copied byte by byte.
constexpr int LC_SPLIT = 16;
__global__ __launch_bounds__(NT) void k_snappy_litcopy(const SnappyJob* __restrict__ jobs, const int* __restrict__ list,
                                                       const int* __restrict__ fb) {
    __shared__ uint32_t tab[2 * LC_MAX];
    const int j = list[blockIdx.x];
    if (fb[j] != FB_LITCOPY) return;
    const SnappyJob& J = jobs[j];
    const uint32_t cnt = J.lit;
    if (threadIdx.x < 2 * cnt) tab[threadIdx.x] = J.tokmap[threadIdx.x];
    __syncthreads();
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(J.src);
    const uintptr_t send = s0 + J.src_len;   // aligned dwords below it are readable
    PF_GLOBAL uint8_t* d = gptr(J.dst);
    const uint32_t n = J.dst_len;
    for (uint32_t c = (blockIdx.y * NT + threadIdx.x) * 16u; c < n; c += LC_SPLIT * NT * 16u) {
        uint32_t lo = 0, hi = cnt;   // last literal whose output starts at or before c
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (tab[2 * m + 1] <= c) lo = m; else hi = m;
        }
        const uint32_t oend = lo + 1 < cnt ? tab[2 * lo + 3] : n;
        if (c + 16u <= oend) {
            const uintptr_t sa = s0 + tab[2 * lo] + (c - tab[2 * lo + 1]);
            const uint32_t sh = uint32_t(sa & 3u);
            const PF_GLOBAL uint32_t* q = (const PF_GLOBAL uint32_t*)(sa & ~uintptr_t(3));
            uint32_t w[5];
            #pragma unroll
            for (int k = 0; k < 5; k++) w[k] = (sa & ~uintptr_t(3)) + 4u * uint32_t(k) < send ? q[k] : 0u;
            const u32x4 v = {__builtin_amdgcn_alignbyte(w[1], w[0], sh), __builtin_amdgcn_alignbyte(w[2], w[1], sh),
                             __builtin_amdgcn_alignbyte(w[3], w[2], sh), __builtin_amdgcn_alignbyte(w[4], w[3], sh)};
            *(PF_GLOBAL u32x4*)(d + c) = v;
        } else {   // the chunk ends the page or spans literals
            const PF_GLOBAL uint8_t* g = (const PF_GLOBAL uint8_t*)(J.src);
            uint32_t k = lo;
            for (uint32_t b = c; b < c + 16u && b < n; b++) {
                while (k + 1 < cnt && tab[2 * k + 3] <= b) k++;
                d[b] = g[tab[2 * k] + (b - tab[2 * k + 1])];
            }
        }
    }
}
void launch_snappy_litcopy(const SnappyJob* d_jobs, const int* d_list, int n, const int* d_fb, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_snappy_litcopy, dim3(n, LC_SPLIT), dim3(NT), 0, st, d_jobs, d_list, d_fb);
}
void launch_snappy_head(SnappyJob* d_jobs, int n_jobs, DevPage* d_pages, const DevChunk* d_chunks, int* d_fb,
                        const DevChunkResult* d_res, hipStream_t st) {
    if (n_jobs > 0)
        hipLaunchKernelGGL(k_snappy_head, dim3((n_jobs + 63) / 64), dim3(64), 0, st, d_jobs, n_jobs, d_pages, d_chunks, d_fb,
                           d_res);
}
void launch_scan(DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                 uint8_t* arena, uint64_t cap, unsigned long long* used, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_scan, dim3(n), dim3(64), 0, st, d_chunks, d_pages, d_list, d_res, arena, cap, used);
}
void launch_runs(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                 hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_runs, dim3(n), dim3(128), 0, st, d_chunks, d_pages, d_list, d_res);
}
void launch_lvl(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                hipStream_t st, bool page_null, NullCaps nc) {
    if (n <= 0) return;
    // page_null (diagnostics option): k_page_null first (one 512-thread workgroup and ~57 KiB of LDS per
    // page; under the bench's four streams its workgroups wait for whole CUs: config 4 5.57 ms with it, 4.47 without)
#ifdef PF_DIAG
    if (page_null) hipLaunchKernelGGL(k_page_null, dim3(n), dim3(PN_NT), 0, st, d_chunks, d_pages, d_list, d_res);
#else
    (void)page_null;
#endif
    hipLaunchKernelGGL(k_lvl, dim3(n), dim3(LT_NT), 0, st, d_chunks, d_pages, d_list, d_res, nc.dcap, nc.icap);
}
void launch_flat(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int nfix, int n, int n4, int n8, int* d_fbq,
                 DevChunkResult* d_res, hipStream_t st, NullCaps nc, int stagger) {
    // d_list: nfix (page, block) pairs of flat fixed-width pages (k_flat_fixed), then n of every other
    // flat page (k_flat_all), then n4 / n8 of nullable 4 / 8-byte pages (k_flat_null<4> / <8>; they mark
    // their pages DONE_NULL). Blocks k_flat_null and k_flat_fixed do not take are queued in d_fbq for
    // k_flat_all's last workgroups. nc: k_flat_null's LDS stages (dictionary: nc.dlds bytes); stagger (diagnostics build,
    // tests): k_flat_null's blocks > 0 of a page wait that many sleep rounds (~3 us each) for block 0
    const int2* blocks = reinterpret_cast<const int2*>(d_list);
    const size_t dyn = size_t(nc.dcap) + 32u + nc.icap + 32u + nc.dlds;
    if (n4 > 0)
        hipLaunchKernelGGL(k_flat_null<4>, dim3(n4), dim3(NTN), dyn, st, d_chunks, d_pages, blocks + nfix + n, d_res, nc, stagger, d_fbq);
    if (n8 > 0)
        hipLaunchKernelGGL(k_flat_null<8>, dim3(n8), dim3(NTN), dyn, st, d_chunks, d_pages, blocks + nfix + n + n4, d_res, nc, stagger,
                           d_fbq);
    if (nfix > 0) hipLaunchKernelGGL(k_flat_fixed, dim3(nfix), dim3(NT), 0, st, d_chunks, d_pages, blocks, d_res, d_fbq);
    // k_flat_all last, with min(nq, 32) more workgroups for the fallback queue (nearly always empty; each
    // needs a CU with room for a k_flat_all workgroup: a grid of min(nq, 1024) waited ~0.1 ms under load,
    // and a launch of its own added one more wait per batch)
    const int nq = nfix + n4 + n8;
    const int nqw = nq < 32 ? nq : 32;
    if (n + nqw > 0)
        hipLaunchKernelGGL(k_flat_all, dim3(n + nqw), dim3(NT), 0, st, d_chunks, d_pages, blocks + nfix, n, d_fbq, d_res);
}
void launch_decode(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, int n_first,
                   DevChunkResult* d_res, hipStream_t st, int idle_grid) {
    // n_first: pages at the head of the list that will need k_decode (host-known); the rest are
    // checked by the stride loop, which is nearly always idle: idle_grid blocks (each needs ~23 KiB of
    // LDS, and the launch ends only once every block has found a CU)
    const int g = std::min(n, std::max(idle_grid, n_first));
    if (n > 0) hipLaunchKernelGGL(k_decode, dim3(g), dim3(NT), 0, st, d_chunks, d_pages, d_list, n, d_res);
}

}  // namespace pf
