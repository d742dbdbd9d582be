// pf_snappy_par.h — wave-parallel Snappy token parsing (device).
//
// A wave parses a window of 64 lanes x SNAP_SEG input bytes that starts at a KNOWN token start.
// Each lane holds its segment (+8 bytes of slack) in registers and computes, four bytes at a
// time, the token input length and output length at every byte position (packed one byte per
// position; literals of 60+ bytes are flagged and resolved exactly when a chain ends on them).
// A chain from any entry is then a static scan over the 32 positions — no dependent memory
// latency. Every lane first assumes its segment starts a token (Snappy token streams
// self-synchronise, so this chain usually coincides with the true one); entries are then taken
// from the previous lane's exit and chains recomputed until a fixed point. A lane whose entry
// equals its predecessor's exit is correct by induction from lane 0, so only that consistent
// prefix is committed (a long literal simply re-bases the next window past its end).
#pragma once
#include "pf_device.h"

namespace pf {

constexpr int SNAP_SEG = 32;                   // bytes per lane
constexpr int SNAP_WIN = 64 * SNAP_SEG;        // 2 KiB per window
constexpr int SNAP_STAGE = SNAP_WIN + 64;      // aligned LDS staging (window + shift + slack)
constexpr int SNAP_ROUNDS = 8;
constexpr uint32_t SNAP_FAR = 0xffffffffu;     // "beyond the window"

// Stage input bytes [base - woff, ...) into LDS with 16-byte loads; returns woff (0..15) so the
// window's byte p is stage[woff + p]. Chunks wholly past `n` are zero; the aligned chunk holding
// the last valid byte is read whole (a 16-B chunk never crosses a page).
__device__ __forceinline__ uint32_t snap_stage_window(uint8_t* stage, const uint8_t* in, uint64_t n, uint64_t base,
                                                      int tid, int nthreads) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(in + base);
    const uint32_t woff = uint32_t(a & 15u);
    const uint4* src = reinterpret_cast<const uint4*>(a - woff);
    const uint64_t first_byte = base - woff;   // stream position of stage[0] (may precede 0 by < 16)
    for (int c = tid; c < SNAP_STAGE / 16; c += nthreads) {
        const uint64_t p = first_byte + uint64_t(c) * 16;   // stream position of this chunk
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p < n) v = src[c];
        reinterpret_cast<uint4*>(stage)[c] = v;
    }
    return woff;
}

// Packed per-byte tables of 4 positions from the dword `w` (bytes are tags).
//   input length: copy1 2, copy2 3, copy4 5, literal (tag>>2)+2; 255 marks a 60+ literal
//   output length: copy1 4+((tag>>2)&7), copy2/4 (tag>>2)+1, literal (tag>>2)+1 (60+: 0)
__device__ __forceinline__ void snap_tables4(uint32_t w, uint32_t& tl, uint32_t& ol) {
    const uint32_t T = w & 0x03030303u;
    const uint32_t L = (w >> 2) & 0x3f3f3f3fu;
    const uint32_t nz = (T | (T >> 1)) & 0x01010101u;          // 1 per byte where type != 0
    const uint32_t copymask = nz * 0xffu;
    const uint32_t t3 = (T >> 1) & T & 0x01010101u;            // type 3
    const uint32_t copy_tl = T + 0x01010101u + t3;             // 2, 3, 5
    // literal: 60..63 -> 255 (long) else L + 2
    const uint32_t big = (((L + 0x04040404u) >> 6) & 0x01010101u) * 0xffu;   // L >= 60
    const uint32_t lit_tl = ((L + 0x02020202u) & ~big) | big;
    tl = (copy_tl & copymask) | (lit_tl & ~copymask);
    const uint32_t t1 = T & ~(T >> 1) & 0x01010101u;           // type 1
    const uint32_t t1m = t1 * 0xffu;
    const uint32_t copy1_ol = ((L & 0x07070707u) + 0x04040404u);
    const uint32_t copyn_ol = L + 0x01010101u;
    const uint32_t c_ol = (copy1_ol & t1m) | (copyn_ol & ~t1m);
    const uint32_t lit_ol = (L + 0x01010101u) & ~big;
    ol = (c_ol & copymask) | (lit_ol & ~copymask);
}

struct SnapSeg {
    uint32_t tl[8], ol[8];   // packed per-byte tables for positions 0..31
    uint32_t w[9];           // the segment's bytes 0..35 (tag + up to 4 operand bytes of token 31)
};

// Registers for one lane's segment: stage bytes [woff + 32*lane, +36).
__device__ __forceinline__ void snap_seg_init(SnapSeg& S, const uint8_t* stage, uint32_t woff, int lane) {
    const uint32_t b0 = woff + uint32_t(lane) * SNAP_SEG;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(stage + (b0 & ~3u));
    const uint32_t sh = (b0 & 3u) * 8u;
    uint32_t raw[10];
    #pragma unroll
    for (int i = 0; i < 10; i++) raw[i] = d[i];
    #pragma unroll
    for (int i = 0; i < 9; i++) S.w[i] = sh ? ((raw[i] >> sh) | (raw[i + 1] << (32u - sh))) : raw[i];
    #pragma unroll
    for (int i = 0; i < 8; i++) snap_tables4(S.w[i], S.tl[i], S.ol[i]);
}

__device__ __forceinline__ uint32_t pk(const uint32_t* t, int b) { return (t[b >> 2] >> (8 * (b & 3))) & 0xffu; }

// Exact length of a literal whose tag is at window byte p (60+ forms).
__device__ __forceinline__ void snap_long_literal(const uint8_t* win, uint32_t p, uint32_t& in_len, uint32_t& out_len) {
    const uint32_t tag = win[p];
    const uint32_t nb = (tag >> 2) - 59;
    uint32_t v = win[p + 1];
    if (nb > 1) v |= uint32_t(win[p + 2]) << 8;
    if (nb > 2) v |= uint32_t(win[p + 3]) << 16;
    if (nb > 3) v |= uint32_t(win[p + 4]) << 24;
    out_len = v + 1u;                                   // wraps only for a 4 GiB literal (rejected later)
    in_len = v > 0xfffffff0u ? SNAP_FAR : v + 2u + nb;
}

// Chain from segment offset `e` (< 32) stopping at offset `lim` (<= 32). Returns the token-start
// mask; `exit` = first chain position >= lim (segment-relative, saturating), `last` = the last
// visited position (or -1).
__device__ __forceinline__ uint32_t snap_chain(const SnapSeg& S, uint32_t e, uint32_t lim, uint32_t& exit, int& last) {
    uint32_t cur = e, mask = 0;
    int lst = -1;
    #pragma unroll
    for (int b = 0; b < 32; b++) {
        if (cur == uint32_t(b) && uint32_t(b) < lim) {
            mask |= 1u << b;
            const uint32_t t = pk(S.tl, b);
            cur = uint32_t(b) + t;
            lst = t == 255u ? b : -1;     // >= 0 only when the chain ends on a 60+ literal
        }
    }
    exit = cur;
    last = lst;
    return mask;
}

struct SnapLane {
    uint32_t valid;      // token starts in this lane's segment (bit i = window byte lane*SEG + i)
    uint32_t exit;       // first true token start at/after the segment end (window-relative, saturating)
    int committed;
};

// Parse the window whose byte 0 (= stage[woff]) is a true token start. `limit` = window-relative
// end (stream or piece end). Must be called by all 64 lanes of one wave. Returns the exit of the
// last committed lane (the next window's entry), SNAP_FAR if it lies beyond 4 GiB.
__device__ inline uint32_t snap_parse_window(const uint8_t* stage, uint32_t woff, uint64_t limit64, SnapLane& L,
                                             SnapSeg& S) {
    const int lane = threadIdx.x & 63;
    const uint8_t* win = stage + woff;
    const uint32_t limit = limit64 > 0xfffffff0ull ? 0xfffffff0u : uint32_t(limit64);
    const uint32_t ss = uint32_t(lane) * SNAP_SEG;
    snap_seg_init(S, stage, woff, lane);
    const uint32_t lim = limit >= ss + 32 ? 32u : (limit <= ss ? 0u : limit - ss);
    // exact exit when a chain ends on a 60+ literal (table value 255)
    auto fix_exit = [&](uint32_t ex_rel, int last) -> uint32_t {
        if (last >= 0) {
            uint32_t il, olen;
            snap_long_literal(win, ss + uint32_t(last), il, olen);
            return il == SNAP_FAR ? SNAP_FAR : (ss + uint32_t(last) + il < ss ? SNAP_FAR : ss + uint32_t(last) + il);
        }
        return ss + ex_rel;
    };
    // chains from entry offsets 0..NSTART-1, computed in one static pass; any true entry
    // inside that range is then a select, not a rescan
    constexpr int NSTART = 8;
    uint32_t cm[NSTART], cx[NSTART];
    int cl[NSTART];
    {
        uint32_t cur[NSTART];
        #pragma unroll
        for (int s = 0; s < NSTART; s++) { cur[s] = uint32_t(s); cm[s] = 0; cl[s] = -1; }
        #pragma unroll
        for (int b = 0; b < 32; b++) {
            const uint32_t t = pk(S.tl, b);
            const bool inlim = uint32_t(b) < lim;
            #pragma unroll
            for (int s = 0; s < NSTART; s++) {
                if (s <= b && cur[s] == uint32_t(b) && inlim) {
                    cm[s] |= 1u << b;
                    cur[s] = uint32_t(b) + t;
                    cl[s] = t == 255u ? b : -1;
                }
            }
        }
        #pragma unroll
        for (int s = 0; s < NSTART; s++) cx[s] = (uint32_t(s) < lim) ? fix_exit(cur[s], cl[s]) : ss + uint32_t(s);
    }
    uint32_t valid = lim ? cm[0] : 0u;
    uint32_t ex = lim ? cx[0] : ss;
    uint32_t entry = ss;
    bool changed = true;
    int rounds_used = 0;
    for (int r = 0; r < 64 && changed; r++) {
        rounds_used = r + 1;
        const uint32_t prev = __shfl_up(ex, 1, 64);
        const uint32_t e = lane == 0 ? 0u : prev;
        const bool ch = e != entry;
        if (ch) {
            entry = e;
            if (e >= ss + 32 || e >= limit) { valid = 0; ex = e; }
            else if (e - ss < uint32_t(NSTART)) {
                const uint32_t o = e - ss;
                uint32_t m = cm[0], x = cx[0];
                #pragma unroll
                for (int s = 1; s < NSTART; s++) if (o == uint32_t(s)) { m = cm[s]; x = cx[s]; }
                valid = m; ex = x;
            } else {
                uint32_t xr;
                int last;
                valid = snap_chain(S, e - ss, lim, xr, last);
                ex = fix_exit(xr, last);
            }
        }
        changed = __any(ch);
    }
    const uint32_t prev = __shfl_up(ex, 1, 64);
    const bool cons = lane == 0 || entry == prev;
    const unsigned long long bad = __ballot(!cons);
    const int f = bad ? __ffsll(bad) - 1 : 64;
#ifdef PF_STAMPS_COUNT
    if (lane == 0) { PF_STAMPS_COUNT[8] += 1; PF_STAMPS_COUNT[9] += f; PF_STAMPS_COUNT[10] += rounds_used; }
#else
    (void)rounds_used;
#endif
    L.committed = lane < f;
    L.valid = L.committed ? valid : 0u;
    L.exit = ex;
    return __shfl(ex, f - 1, 64);
}

// Output bytes of the lane's valid tokens (60+ literals resolved exactly).
__device__ __forceinline__ uint64_t snap_lane_outsum(const SnapSeg& S, const uint8_t* win, uint32_t valid, int lane) {
    uint64_t s = 0;
    #pragma unroll
    for (int b = 0; b < 32; b++) {
        if ((valid >> b) & 1u) {
            uint32_t o = pk(S.ol, b);
            if (pk(S.tl, b) == 255u) { uint32_t il; snap_long_literal(win, uint32_t(lane) * SNAP_SEG + b, il, o); }
            s += o;
        }
    }
    return s;
}

}  // namespace pf
