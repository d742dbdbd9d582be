// pf_delta.hip — K5: DELTA_BINARY_PACKED decode (INT32 / INT64 pages).
//
// Replaces parquet-mr's DeltaBinaryPackingValuesReader / ...ForLong (behind
// ColumnReader.getInteger/getLong, src/main/java/blue/strategic/parquet/ParquetReader.java:158-161).
// Header <block size><miniblocks per block><total count><zigzag first value>; each block:
// <zigzag min delta><one bit-width byte per miniblock><miniblocks of bit-packed deltas>.
// v[i] = v[i-1] + min_delta + d[i], two's-complement wrap (32-bit for INT32: computing in
// 64 bits and truncating gives the same residues). A miniblock is consumed whole while any
// value remains (parquet-mr unpacks all its 8-value groups).
//
// One 256-thread workgroup per page: lane 0 walks block headers into an LDS miniblock table
// (sequential but one step per 32+ values), all threads unpack deltas in parallel, then a
// workgroup prefix sum (carried across tiles) rebuilds the values into the page's aux buffer.
#include <hip/hip_runtime.h>

#include "pf_device.h"

namespace pf {

constexpr int DNT = 256;
constexpr int MB_CAP = 1024;   // miniblocks per round
constexpr int DVPT = 8;        // values per thread per tile

struct MiniBlock {
    uint64_t bitpos;     // absolute bit position of the miniblock's packed data
    int64_t min_delta;
    uint32_t first;      // index (within the page's value stream) of its first delta's value
    int32_t width;
};

struct DbpLds {
    MiniBlock mb[MB_CAP];
    int nmb, err, done;
    uint64_t wpos, vpm_s, total_s, have_s, nmini_s, rend;
    uint64_t carry;
    uint64_t wsum[DNT / 64];
    int64_t cur_min;
    int blk_left;        // miniblocks left in the current block
    uint8_t widths[256];
};

// Values section of a data page (v1: after the rep/def level sections).
__device__ bool values_section(const DevPage& pg, const DevChunk& ck, const uint8_t*& p, uint64_t& n) {
    if (pg.flags & PG_V2) { p = pg.body; n = pg.body_len; return true; }
    uint64_t pos = 0;
    n = pg.body_len; p = pg.body;
    for (int which = 0; which < 2; which++) {
        const int maxl = which == 0 ? ck.max_rep : ck.max_def;
        if (maxl == 0) continue;
        const int enc = which == 0 ? pg.rep_enc : pg.def_enc;
        uint64_t len;
        if (enc == 3) { if (pos + 4 > n) return false; len = ld32le(p, pos, n); pos += 4; }
        else if (enc == 4) len = (uint64_t(pg.num_values) * bit_width(maxl) + 7) / 8;
        else return false;
        if (len > n - pos) return false;
        pos += len;
    }
    p += pos; n -= pos;
    return true;
}

// Workgroup-wide DELTA_BINARY_PACKED decode of [p, p + n) (parquet-mr DeltaBinaryPackingValuesReader
// semantics): values v[0, min(total, cap)) -> out (64-bit; INT32 streams wrap mod 2^32). A
// miniblock is consumed whole while any value remains, so `end` (the byte after the last one read)
// is where a following section (DELTA_LENGTH_BYTE_ARRAY chars, DELTA_BYTE_ARRAY suffixes) starts.
// strict: total > cap is an error (INT pages); otherwise values past cap are parsed, not stored.
// Returns false on a malformed stream. All DNT threads must call.
__device__ bool dbp_decode_wg(DbpLds& S, const uint8_t* p, uint64_t n, bool is64, uint64_t* out, uint64_t cap,
                              bool strict, uint64_t& total_out, uint64_t& end_out) {
    if (threadIdx.x == 0) {
        S.err = 0; S.done = 0;
        uint64_t pos = 0, block, nmini, total, zz;
        if (!uvarint(p, n, pos, block) || !uvarint(p, n, pos, nmini) || !uvarint(p, n, pos, total) ||
            !uvarint(p, n, pos, zz) || nmini == 0 || block == 0 || block % nmini || nmini > 256 || nmini > block ||
            (block / nmini) % 8 || (strict && total > cap)) {   // parquet-mr: miniblock size a multiple of 8
            S.err = 1;
        } else {
            S.vpm_s = block / nmini; S.nmini_s = nmini; S.total_s = total;
            uint64_t first = uint64_t(unzigzag(zz));
            if (!is64) first = uint64_t(uint32_t(first));
            if (total > 0 && cap > 0) out[0] = first;
            S.have_s = total > 0 ? 1 : 0;
            S.wpos = pos; S.blk_left = 0;
            S.carry = first;
        }
    }
    __syncthreads();
    if (S.err) return false;
    const uint64_t vpm = S.vpm_s, total = S.total_s;
    while (true) {
        // ---- thread 0: collect up to MB_CAP miniblock headers ----
        if (threadIdx.x == 0) {
            int k = 0;
            uint64_t have = S.have_s, pos = S.wpos;
            while (have < total && k < MB_CAP) {
                if (S.blk_left == 0) {
                    uint64_t mz;
                    if (!uvarint(p, n, pos, mz) || pos + S.nmini_s > n) { S.err = 1; break; }
                    int64_t md = unzigzag(mz);
                    if (!is64) md = int32_t(md);
                    S.cur_min = md;
                    for (uint64_t m = 0; m < S.nmini_s; m++) S.widths[m] = p[pos + m];
                    pos += S.nmini_s;
                    S.blk_left = int(S.nmini_s);
                }
                const int w = S.widths[S.nmini_s - S.blk_left];
                if (w > (is64 ? 64 : 32)) { S.err = 1; break; }
                const uint64_t nb = vpm * uint64_t(w) / 8;
                if (pos + nb > n) { S.err = 1; break; }
                S.mb[k].bitpos = pos * 8; S.mb[k].width = w; S.mb[k].min_delta = S.cur_min; S.mb[k].first = uint32_t(have);
                k++;
                pos += nb;
                S.blk_left--;
                have += vpm;
                if (have > total) have = total;
            }
            S.nmb = k; S.wpos = pos;
            if (have >= total) S.done = 1;
            S.rend = have;   // values [have_s, have) are covered by these k miniblocks
        }
        __syncthreads();
        if (S.err) break;
        const uint64_t r0 = S.have_s, r1 = S.rend;
        const int nk = S.nmb;
        // ---- all threads: deltas -> values, tile by tile with a carried prefix; DVPT consecutive
        // values per thread (one workgroup scan per DNT * DVPT values) ----
        for (uint64_t t0 = r0; t0 < r1; t0 += uint64_t(DNT) * DVPT) {
            const uint64_t i0 = t0 + uint64_t(threadIdx.x) * DVPT;
            uint64_t d[DVPT];
            uint64_t tsum = 0;
            #pragma unroll
            for (int k = 0; k < DVPT; k++) {
                const uint64_t i = i0 + k;
                uint64_t dk = 0;
                if (i < r1) {
                    const uint64_t j = i - r0;                       // delta index within this round
                    const uint64_t m = j / vpm, q = j % vpm;
                    if (m < uint64_t(nk)) {
                        const MiniBlock& b = S.mb[m];
                        dk = uint64_t(b.min_delta) + bits_le64(p, n, b.bitpos + q * uint64_t(b.width), b.width);
                    }
                }
                tsum += dk;
                d[k] = tsum;                                         // inclusive within the thread
            }
            // exclusive scan of the thread sums across the workgroup
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            uint64_t x = tsum;
            #pragma unroll
            for (int sh = 1; sh < 64; sh <<= 1) {
                const uint64_t y = __shfl_up(x, sh, 64);
                if (lane >= sh) x += y;
            }
            if (lane == 63) S.wsum[wid] = x;
            __syncthreads();
            uint64_t base = S.carry, all = 0;
            for (int w2 = 0; w2 < DNT / 64; w2++) {
                const uint64_t ws = S.wsum[w2];
                if (w2 < wid) base += ws;
                all += ws;
            }
            base += x - tsum;
            #pragma unroll
            for (int k = 0; k < DVPT; k++) {
                const uint64_t i = i0 + k;
                uint64_t v = base + d[k];
                if (!is64) v = uint64_t(uint32_t(v));
                if (i < r1 && i < cap) out[i] = v;
            }
            __syncthreads();   // every thread read carry and wsum
            if (threadIdx.x == 0) S.carry = S.carry + all;
            __syncthreads();
        }
        if (threadIdx.x == 0) S.have_s = r1;
        __syncthreads();
        if (S.done) break;
    }
    total_out = total;
    end_out = S.wpos;
    const bool ok = !S.err;
    __syncthreads();
    return ok;
}

// ---- block-parallel DELTA_BINARY_PACKED (large INT32 / INT64 pages) -----------------------------
// k_delta walks block headers on one lane (one dependent header read per block: ~250 us for a
// 494 K-value page). Blocks hold `block` values each (the last one fewer), so block b's first value
// is 1 + b * block: only the blocks' byte positions form a chain. k_dbp_pos finds them the way
// k_nest_lvl finds level runs (pf_pages.hip): per DBP_WIN-byte window every position is decoded as
// a block header (next = position + header + sum of the miniblocks' bytes), pointer jumping gives
// each position's window exit, windows hand over the true chain's entry in one pass, then walk their
// part of it storing the positions. k_dbp_blk (one wave per block) sums each block's deltas,
// k_dbp_scan turns the sums into block bases, k_dbp_blk (again) writes the values. Any check the
// one-lane walk would fail (header, widths and data of the miniblocks consumed) sets dbp_ok = 2 and
// k_delta, launched last, decodes the page from scratch (and reports it).
constexpr int DP_NT = 256;
constexpr uint32_t DP_END = 0xFFFFFFu;
constexpr uint32_t DP_FAR = 0xFFFFFEu;
constexpr uint32_t DP_MAXMINI = 16;   // pages with more miniblocks per block stay on k_delta

struct DbpHdr {
    uint64_t block, nmini, total, first, pos0, vpm, nblocks;
    bool ok;
};
// The page header, checked as dbp_decode_wg checks it (strict: total <= cap).
__device__ __forceinline__ DbpHdr dbp_header(const uint8_t* p, uint64_t n, bool is64, uint64_t cap) {
    DbpHdr h{};
    uint64_t pos = 0, zz;
    h.ok = uvarint(p, n, pos, h.block) && uvarint(p, n, pos, h.nmini) && uvarint(p, n, pos, h.total) &&
           uvarint(p, n, pos, zz) && h.nmini > 0 && h.block > 0 && h.block % h.nmini == 0 && h.nmini <= DP_MAXMINI &&
           h.nmini <= h.block && (h.block / h.nmini) % 8 == 0 && h.total <= cap;
    if (!h.ok) return h;
    h.first = uint64_t(unzigzag(zz));
    if (!is64) h.first = uint64_t(uint32_t(h.first));
    h.pos0 = pos;
    h.vpm = h.block / h.nmini;
    h.nblocks = h.total > 1 ? (h.total - 1 + h.block - 1) / h.block : 0;
    return h;
}
// block header at stream position q (bytes b = the stream from q, >= 10 + nmini readable): the
// position after its miniblocks (all nmini of them), or false when no header fits there
__device__ __forceinline__ bool dbp_next(const uint8_t* b, uint64_t q, uint64_t n, uint64_t nmini, uint64_t vpm, uint64_t& next) {
    uint32_t hl = 0;
    bool ok = false;
    for (uint32_t sh = 0; sh < 70; sh += 7) {
        if (q + hl >= n) break;
        const uint32_t c = b[hl++];
        if (!(c & 0x80)) { ok = true; break; }
    }
    if (!ok || q + hl + nmini > n) return false;
    uint64_t bits = 0;
    for (uint32_t m = 0; m < nmini; m++) bits += b[hl + m];
    next = q + hl + nmini + bits * vpm / 8;
    return true;
}
__device__ __forceinline__ void dbp_fail(DevPage& pg) {
    __hip_atomic_store(&pg.dbp_ok, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(DP_NT) void k_dbp_pos(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list) {
    __shared__ __attribute__((aligned(16))) uint32_t st[(DBP_WIN + 64 + 32) / 4];
    __shared__ uint64_t X[DBP_WIN];
    __shared__ uint64_t s_hand[3];
    const int tid = threadIdx.x;
    DevPage& pg = pages[list[blockIdx.z]];
    const DevChunk& ck = chunks[pg.chunk];
    const uint32_t w = blockIdx.x;
    if (!pg.dbp || w >= uint32_t(pg.dbp_nwin)) return;
    const uint8_t* p;
    uint64_t n;
    if (!values_section(pg, ck, p, n)) { if (w == 0 && tid == 0) dbp_fail(pg); return; }
    const DbpHdr H = dbp_header(p, n, ck.ptype == 2, uint64_t(pg.aux_cap));
    if (!H.ok || H.nblocks == 0 || H.nblocks > pg.dbp_bcap) { if (w == 0 && tid == 0) dbp_fail(pg); return; }
    if (w == 0 && tid == 0) __hip_atomic_fetch_max(&pg.dbp_ok, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t* bpos = reinterpret_cast<uint32_t*>(pg.dbp);
    const uint64_t w0 = H.pos0 + uint64_t(w) * DBP_WIN, w1 = w0 + DBP_WIN;
    if (w0 >= n && w > 0) return;
    const bool last = w1 >= n;
    WinPub* pub = pg.dbp_pub;
    const uint32_t look = 10 + uint32_t(H.nmini) + 8;
    const uint32_t woff = stage_bytes(st, p, n, uint32_t(min<uint64_t>(w0, n)), uint32_t(min<uint64_t>(w1 + look, n)));
    __syncthreads();
    const uint8_t* W = reinterpret_cast<const uint8_t*>(st) + woff;
    for (uint32_t i = tid; i < DBP_WIN; i += DP_NT) {
        const uint64_t q = w0 + i;
        uint64_t nx, x = DP_END;
        if (q < n && dbp_next(W + i, q, n, H.nmini, H.vpm, nx)) {
            const uint64_t rel = nx - w0;
            x = (1ull << 24) | (rel < DP_FAR ? rel : uint64_t(DP_FAR));
        }
        X[i] = x;
    }
    __syncthreads();
    for (uint32_t span = 1; span < DBP_WIN; span <<= 1) {
        for (uint32_t i = tid; i < DBP_WIN; i += DP_NT) {
            const uint64_t x = X[i];
            const uint32_t e = uint32_t(x & 0xFFFFFFu);
            if (e < DBP_WIN) {
                const uint64_t y = X[e];
                X[i] = (((x >> 24) + (y >> 24)) << 24) | (y & 0xFFFFFFu);
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        uint64_t tp = H.pos0, tb = 0;
        uint32_t tst = 0;
        bool ok = true;
        if (w > 0) ok = winpub_get(pub[w - 1], 1u << 22, tp, tb, tst);   // (bounded: no hang on a stall)
        s_hand[0] = tp; s_hand[1] = tb; s_hand[2] = uint64_t(tst) | (ok ? 0u : 2u);
        uint64_t xp = tp, xb = tb;
        uint32_t xst = tst;
        if (ok && tst == 0 && tb < H.nblocks && tp < w1) {
            const uint64_t x = X[tp - w0];
            const uint32_t e = uint32_t(x & 0xFFFFFFu);
            if (e == DP_FAR) {   // a block of > 16 MB: walk to the exit
                while (xp < w1) {
                    uint64_t nx;
                    if (xp >= n || !dbp_next(W + (xp - w0), xp, n, H.nmini, H.vpm, nx)) { xst = 1; break; }
                    xb++;
                    xp = nx;
                }
            } else {
                xb = tb + (x >> 24);
                if (e == DP_END) { xst = 1; xp = w1; }
                else xp = w0 + e;
            }
        }
        if (!ok) dbp_fail(pg);
        winpub_put(pub[w], ok ? xp : ~0ull, xb, xst);   // (failed: the overflow word, later windows fail at once)
    }
    __syncthreads();
    if (s_hand[2] & 2u) return;
    if (tid < 64) {   // the window's blocks of the true chain (all 64 lanes walk in step)
        uint64_t tp = s_hand[0], tb = s_hand[1];
        uint32_t tst = uint32_t(s_hand[2]);
        if (tst == 0) {
            while (tb < H.nblocks && tp < w1) {
                uint64_t nx;
                if (tp >= n || !dbp_next(W + (tp - w0), tp, n, H.nmini, H.vpm, nx)) { tst = 1; break; }
                if (tid == 0) bpos[tb] = uint32_t(tp);
                tb++;
                tp = nx;
            }
        }
        // the chain ended before the page's last block, or the stream did
        if (tid == 0 && tb < H.nblocks && (tst == 1 || last)) dbp_fail(pg);
    }
}

__device__ bool dbp_block(DevPage& pg, const uint8_t* p, uint64_t n, const DbpHdr& H, bool is64, uint64_t b, int lane, int mode);
// mode 0: each block's delta sum -> sum[b]; mode 1: values from the block bases (k_dbp_scan) -> aux.
// One wave per block (grid-stride), 64 values at a time.
__global__ __launch_bounds__(DP_NT) void k_dbp_blk(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list,
                                                   int mode) {
    DevPage& pg = pages[list[blockIdx.y]];
    const DevChunk& ck = chunks[pg.chunk];
    if (!pg.dbp || __hip_atomic_load(&pg.dbp_ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1) return;
    const uint8_t* p;
    uint64_t n;
    values_section(pg, ck, p, n);
    const bool is64 = ck.ptype == 2;
    const DbpHdr H = dbp_header(p, n, is64, uint64_t(pg.aux_cap));
    const int lane = threadIdx.x & 63;
    for (uint64_t b = uint64_t(blockIdx.x) * (DP_NT / 64) + (threadIdx.x >> 6); b < H.nblocks;
         b += uint64_t(gridDim.x) * (DP_NT / 64))
        if (!dbp_block(pg, p, n, H, is64, b, lane, mode)) return;
}

// one block, one wave (k_dbp_blk); false after a failed check
__device__ bool dbp_block(DevPage& pg, const uint8_t* p, uint64_t n, const DbpHdr& H, bool is64, uint64_t b, int lane, int mode) {
    const uint32_t* bpos = reinterpret_cast<const uint32_t*>(pg.dbp);
    uint64_t* bsum = reinterpret_cast<uint64_t*>(pg.dbp + 4ull * pg.dbp_bcap + 8 - ((4ull * pg.dbp_bcap) & 7));
    uint64_t pos = bpos[b], md;
    if (!uvarint(p, n, pos, md)) { if (lane == 0) dbp_fail(pg); return false; }
    int64_t mind = unzigzag(md);
    if (!is64) mind = int32_t(mind);
    const uint64_t wpos = pos, dpos = pos + H.nmini;   // widths, then miniblock data
    const uint64_t v0 = 1 + b * H.block, v1 = min<uint64_t>(H.total, v0 + H.block);
    const uint32_t maxw = is64 ? 64u : 32u;
    // miniblocks consumed: ceil((v1 - v0) / vpm); their widths and data must be in the stream
    const uint64_t nm = (v1 - v0 + H.vpm - 1) / H.vpm;
    if (wpos + H.nmini > n) { if (lane == 0) dbp_fail(pg); return false; }
    // lane m < nmini: miniblock m's width and bit offset (exclusive prefix over the lanes)
    const uint32_t wl = uint64_t(lane) < H.nmini ? uint32_t(p[wpos + lane]) : 0u;
    uint64_t ol = uint64_t(wl) * H.vpm;
    #pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const uint64_t y = __shfl_up(ol, sh, 64);
        if (lane >= sh) ol += y;
    }
    ol = dpos * 8 + ol - uint64_t(wl) * H.vpm;   // bit offset of miniblock `lane`
    const bool bad = uint64_t(lane) < nm && (wl > maxw || (ol + uint64_t(wl) * H.vpm + 7) / 8 > n);
    if (__any(bad)) { if (lane == 0) dbp_fail(pg); return false; }
    uint64_t carry = mode == 1 ? bsum[b] : 0, acc = 0;
    uint64_t* out = reinterpret_cast<uint64_t*>(pg.aux);
    for (uint64_t c0 = v0; c0 < v1; c0 += 64) {
        const uint64_t i = c0 + lane;
        const uint64_t j = min<uint64_t>(i, v1 - 1) - v0, q = j % H.vpm;
        const int m = int(j / H.vpm);   // (shuffles with every lane active)
        const uint32_t wm = uint32_t(__shfl(int(wl), m, 64));
        const uint64_t om = __shfl(ol, m, 64);
        uint64_t d = 0;
        if (i < v1) d = uint64_t(mind) + bits_le64(p, n, om + q * wm, int(wm));
        uint64_t x = d;
        #pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            const uint64_t y = __shfl_up(x, sh, 64);
            if (lane >= sh) x += y;
        }
        if (mode == 1 && i < v1) {
            uint64_t v = carry + x;
            if (!is64) v = uint64_t(uint32_t(v));
            out[i] = v;
        }
        const uint64_t tot = __shfl(x, 63, 64);
        carry += tot;
        acc += tot;
    }
    if (mode == 0 && lane == 0) bsum[b] = acc;
    return true;
}

// one workgroup per page: exclusive prefix of the block sums from the first value -> block bases
__global__ __launch_bounds__(DP_NT) void k_dbp_scan(const DevChunk* __restrict__ chunks, DevPage* pages, const int* __restrict__ list) {
    __shared__ uint64_t wsum[DP_NT / 64];
    DevPage& pg = pages[list[blockIdx.x]];
    const DevChunk& ck = chunks[pg.chunk];
    if (!pg.dbp || __hip_atomic_load(&pg.dbp_ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1) return;
    const uint8_t* p;
    uint64_t n;
    values_section(pg, ck, p, n);
    const DbpHdr H = dbp_header(p, n, ck.ptype == 2, uint64_t(pg.aux_cap));
    uint64_t* bsum = reinterpret_cast<uint64_t*>(pg.dbp + 4ull * pg.dbp_bcap + 8 - ((4ull * pg.dbp_bcap) & 7));
    if (threadIdx.x == 0 && H.total > 0) reinterpret_cast<uint64_t*>(pg.aux)[0] = H.first;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t carry = H.first;
    for (uint64_t b0 = 0; b0 < H.nblocks; b0 += DP_NT) {
        const uint64_t b = b0 + threadIdx.x;
        const uint64_t s = b < H.nblocks ? bsum[b] : 0;
        uint64_t x = s;
        #pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            const uint64_t y = __shfl_up(x, sh, 64);
            if (lane >= sh) x += y;
        }
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
        uint64_t base = carry, all = 0;
        for (int k = 0; k < DP_NT / 64; k++) { if (k < wid) base += wsum[k]; all += wsum[k]; }
        if (b < H.nblocks) bsum[b] = base + x - s;
        carry += all;
        __syncthreads();
    }
}

__global__ __launch_bounds__(DNT) void k_delta(const DevChunk* __restrict__ chunks, DevPage* pages, const int* page_list,
                                               DevChunkResult* res) {
    __shared__ DbpLds S;
    const int pi = page_list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (res[pg.chunk].status != 0) return;
    if (pg.dbp && pg.dbp_ok == 1) return;   // k_dbp_* decoded it
    const uint8_t* p;
    uint64_t n, total, end;
    if (!values_section(pg, ck, p, n)) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    if (!dbp_decode_wg(S, p, n, ck.ptype == 2, reinterpret_cast<uint64_t*>(pg.aux), uint64_t(pg.aux_cap), true, total,
                       end) && threadIdx.x == 0)
        set_status(res, pg.chunk, ST_CORRUPT, pi);
}

// ---- DELTA_LENGTH_BYTE_ARRAY (6) / DELTA_BYTE_ARRAY (7) BYTE_ARRAY pages -------------------------
// Replaces parquet-mr's DeltaLengthByteArrayValuesReader / DeltaByteArrayReader (behind
// ColumnReader.getBinary, src/main/java/blue/strategic/parquet/ParquetReader.java:151-157).
// k_dlen (before k_count), one workgroup per page: the length stream(s) -> pg.dx:
//   cpos[k] = chars of values [0, k) (u64, k <= T; saturates past 2^62 on a bad length),
//   lenA[k] = DLBA length / DBA prefix length, lenB[k] = DBA suffix length,
// dx_data = where the chars (DLBA) / suffixes (DBA) start in the values section, dx_bad = the
// first value that violates the oracle's checks (length < 0 as int32, prefix longer than the
// previous value, data past the section end). k_count then checks the page's present values
// against T and dx_bad and takes the page's chars from cpos. k_decode writes offsets and, for DLBA,
// the chars; k_dba_chars materialises DELTA_BYTE_ARRAY values (prefix of the previous value +
// suffix) in value order.
constexpr uint64_t CPOS_BAD = 1ull << 62;

__global__ __launch_bounds__(DNT) void k_dlen(const DevChunk* __restrict__ chunks, DevPage* pages, const int* page_list,
                                              DevChunkResult* res) {
    __shared__ DbpLds S;
    __shared__ uint64_t wtot[DNT / 64];
    __shared__ uint64_t s_carry, s_carry_sfx;
    __shared__ uint32_t s_prevlen;
    const int pi = page_list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    if (res[pg.chunk].status != 0) return;
    const bool dba = pg.encoding == 7;
    const uint8_t* p;
    uint64_t n;
    const uint64_t cap = uint64_t(pg.aux_cap);
    uint64_t* cpos = pg.dx;
    uint64_t* la = cpos + cap + 1;
    uint64_t* lb = la + cap;
    uint64_t t1 = 0, e1 = 0, t2 = 0, e2 = 0;
    bool ok = values_section(pg, ck, p, n);
    if (ok) ok = dbp_decode_wg(S, p, n, false, la, cap, false, t1, e1);
    if (ok && dba) ok = dbp_decode_wg(S, p + e1, n - e1, false, lb, cap, false, t2, e2);
    if (!ok) { if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    const uint64_t T = dba ? min(t1, t2) : t1;     // values both streams hold
    const uint64_t data = e1 + e2;                  // chars / suffixes start
    const uint64_t avail = n - data;
    const uint64_t m = min(T, cap);
    if (tid == 0) { s_carry = 0; s_carry_sfx = 0; s_prevlen = 0; pg.dx_bad = int64_t(m); }
    __syncthreads();
    // per-value checks + prefix sums of the value lengths (and of DBA suffix lengths)
    for (uint64_t t0 = 0; t0 < m; t0 += DNT) {
        const uint64_t k = t0 + uint64_t(tid);
        const bool in = k < m;
        const uint32_t a = in ? uint32_t(la[k]) : 0u, b = in && dba ? uint32_t(lb[k]) : 0u;
        bool bad = in && (int32_t(a) < 0 || int32_t(b) < 0);
        const uint64_t len = uint64_t(a) + uint64_t(b);
        const uint64_t sfx = dba ? b : a;           // bytes this value takes from the data section
        // inclusive scans (wave, then across waves)
        const int lane = tid & 63, wid = tid >> 6;
        uint64_t x = len, y = sfx;
        #pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            const uint64_t xu = __shfl_up(x, sh, 64), yu = __shfl_up(y, sh, 64);
            if (lane >= sh) { x += xu; y += yu; }
        }
        if (lane == 63) { wtot[wid] = x; S.wsum[wid] = y; }
        __syncthreads();
        uint64_t bx = s_carry, by = s_carry_sfx;
        for (int w2 = 0; w2 < wid; w2++) { bx += wtot[w2]; by += S.wsum[w2]; }
        const uint64_t cend = bx + x, send = by + y;   // after value k
        if (in) {
            if (send > avail) bad = true;
            if (dba) {   // prefix <= previous value's length
                const uint32_t prev = k == 0 ? 0u : (k == t0 ? s_prevlen : uint32_t(la[k - 1]) + uint32_t(lb[k - 1]));
                if (a > prev) bad = true;
            }
            cpos[k + 1] = min(cend, CPOS_BAD);
            if (k == 0) cpos[0] = 0;
        }
        if (bad) atomicMin(reinterpret_cast<unsigned long long*>(&pg.dx_bad), (unsigned long long)k);
        __syncthreads();
        if (in && (k + 1 == min(m, t0 + DNT))) { s_carry = cend; s_carry_sfx = send; s_prevlen = uint32_t(len); }
        __syncthreads();
    }
    if (tid == 0) {
        if (m == 0) cpos[0] = 0;
        pg.dx_total = int64_t(T);
        pg.dx_data = uint32_t(data);
    }
}

// One wave per DELTA_BYTE_ARRAY page, after k_scan: value k = the first prefix[k] bytes of value
// k-1 + its suffix, written at chars + char_start + cpos[k]. The previous value is kept in LDS
// (values longer than XV_CAP re-read it from the chars just written) and the suffix stream is
// staged through LDS in XS_WIN windows.
constexpr uint32_t XV_CAP = 4096;
constexpr uint32_t XS_WIN = 8192;

__global__ __launch_bounds__(64) void k_dba_chars(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                  const int* page_list, DevChunkResult* res) {
    __shared__ __attribute__((aligned(16))) uint8_t vbuf[2][XV_CAP];
    __shared__ __attribute__((aligned(16))) uint8_t sw[XS_WIN];
    const int pi = page_list[blockIdx.x];
    const DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int lane = threadIdx.x;
    if (res[pg.chunk].status != 0 || !ck.chars || !pg.dx) return;
    const uint8_t* p;
    uint64_t n;
    if (!values_section(pg, ck, p, n)) return;   // k_dlen reported it
    const uint64_t nv = uint64_t(pg.n_values);
    const uint64_t cap = uint64_t(pg.aux_cap);
    const uint64_t* cpos = pg.dx;
    const uint64_t* la = cpos + cap + 1;
    const uint64_t* lb = la + cap;
    const uint8_t* sfx = p + pg.dx_data;
    const uint64_t sfx_n = n - pg.dx_data;
    uint8_t* out = ck.chars + pg.char_start;
    uint64_t sp = 0;            // suffix stream position
    uint64_t ws = 0, we = 0;    // staged window [ws, we)
    int cur = 0;
    uint32_t plen = 0;          // previous value's length
    for (uint64_t k = 0; k < nv; k++) {
        const uint32_t pl = uint32_t(la[k]), sl = uint32_t(lb[k]);
        const uint32_t len = pl + sl;
        uint8_t* o = out + cpos[k];
        const bool fits = len <= XV_CAP && plen <= XV_CAP;
        if (sl > 0 && (sp < ws || sp + sl > we)) {   // restage the suffix window at sp
            if (sl <= XS_WIN) {
                ws = sp;
                we = min<uint64_t>(sp + XS_WIN, sfx_n);
                for (uint64_t i = uint64_t(lane); i < we - ws; i += 64) sw[i] = sfx[ws + i];
                __syncthreads();
            }
        }
        const bool staged = sp >= ws && sp + sl <= we;
        if (!fits) __threadfence_block();            // previous value re-read from the chars just written
        const uint8_t* prev = vbuf[cur ^ 1];
        uint8_t* keep = vbuf[cur];
        for (uint32_t j = uint32_t(lane); j < len; j += 64) {
            uint8_t b;
            if (j < pl) b = fits ? prev[j] : out[cpos[k - 1] + j];
            else b = staged ? sw[sp - ws + (j - pl)] : sfx[sp + (j - pl)];
            o[j] = b;
            if (len <= XV_CAP) keep[j] = b;
        }
        __syncthreads();
        sp += sl;
        plen = len;
        cur ^= 1;
    }
}

void launch_delta(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, int max_dbp_nwin, DevChunkResult* d_res,
                  hipStream_t st) {
    if (n <= 0) return;
    if (max_dbp_nwin > 0) {   // block-parallel pages first (k_delta then skips them, or redoes the ones that failed)
        // block grid: DP_NT / 64 blocks per workgroup, sized for the largest table (pages with fewer exit early)
        constexpr int dbp_grid_blocks = 64;   // workgroups per page (4 waves each, grid-stride over blocks)
        hipLaunchKernelGGL(k_dbp_pos, dim3(max_dbp_nwin, 1, n), dim3(DP_NT), 0, st, d_chunks, d_pages, d_list);
        hipLaunchKernelGGL(k_dbp_blk, dim3(dbp_grid_blocks, n), dim3(DP_NT), 0, st, d_chunks, d_pages, d_list, 0);
        hipLaunchKernelGGL(k_dbp_scan, dim3(n), dim3(DP_NT), 0, st, d_chunks, d_pages, d_list);
        hipLaunchKernelGGL(k_dbp_blk, dim3(dbp_grid_blocks, n), dim3(DP_NT), 0, st, d_chunks, d_pages, d_list, 1);
    }
    hipLaunchKernelGGL(k_delta, dim3(n), dim3(DNT), 0, st, d_chunks, d_pages, d_list, d_res);
}
void launch_dlen(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                 hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_dlen, dim3(n), dim3(DNT), 0, st, d_chunks, d_pages, d_list, d_res);
}
void launch_dba_chars(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                      hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_dba_chars, dim3(n), dim3(64), 0, st, d_chunks, d_pages, d_list, d_res);
}

}  // namespace pf
