// pf_snappy_par.h — wave-parallel Snappy token parsing (device).
//
// A wave parses a window of 64 lanes x SEG input bytes that starts at a KNOWN token start.
// Every lane first parses its own segment speculatively from the segment's first byte
// (Snappy token streams self-synchronise: a chain started mid-token almost always lands on
// the true chain within a few tokens). Lanes then take their true entry from the previous
// lane's exit and, where the entry is not on their speculative chain, walk from it until
// they merge with that chain. Entries/exits are iterated to a fixed point; a lane whose
// entry equals its predecessor's exit is correct by induction from lane 0. Windows commit
// only the consistent prefix of lanes, so long literals simply re-base the next window.
#pragma once
#include "pf_device.h"

namespace pf {

constexpr int SNAP_SEG = 32;                   // bytes per lane
constexpr int SNAP_WIN = 64 * SNAP_SEG;        // 2 KiB per window
constexpr int SNAP_SLACK = 8;                  // tag + up to 4 length bytes past a segment
constexpr int SNAP_ROUNDS = 6;

// Input bytes of a token starting at p of the LDS window (relative offsets); literal lengths up
// to 2^32 come back as 64-bit.
__device__ __forceinline__ uint64_t snap_toklen(const uint8_t* w, uint32_t p) {
    uint32_t tag = w[p];
    uint32_t t = tag & 3;
    if (t == 0) {
        uint32_t len = tag >> 2;
        if (len < 60) return uint64_t(len) + 2;
        uint32_t nb = len - 59;
        uint32_t v = w[p + 1];
        if (nb > 1) v |= uint32_t(w[p + 2]) << 8;
        if (nb > 2) v |= uint32_t(w[p + 3]) << 16;
        if (nb > 3) v |= uint32_t(w[p + 4]) << 24;
        return uint64_t(v) + 2 + nb;
    }
    return t == 1 ? 2 : (t == 2 ? 3 : 5);
}

// Output bytes of the token at p.
__device__ __forceinline__ uint64_t snap_outlen(const uint8_t* w, uint32_t p) {
    uint32_t tag = w[p];
    uint32_t t = tag & 3;
    if (t == 0) {
        uint32_t len = tag >> 2;
        if (len < 60) return uint64_t(len) + 1;
        uint32_t nb = len - 59;
        uint32_t v = w[p + 1];
        if (nb > 1) v |= uint32_t(w[p + 2]) << 8;
        if (nb > 2) v |= uint32_t(w[p + 3]) << 16;
        if (nb > 3) v |= uint32_t(w[p + 4]) << 24;
        return uint64_t(v) + 1;
    }
    return t == 1 ? 4 + ((tag >> 2) & 7) : (tag >> 2) + 1;
}

// Load window bytes [base, base + SNAP_WIN + SNAP_SLACK) of `in` (bytes at or past `n` read 0).
__device__ __forceinline__ void snap_load_window(uint8_t* win, const uint8_t* in, uint64_t n, uint64_t base) {
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < (SNAP_WIN + SNAP_SLACK) / 4; i += 64) {
        uint64_t p = base + uint64_t(i) * 4;
        uint32_t v;
        if (p + 4 <= n) v = uint32_t(in[p]) | uint32_t(in[p + 1]) << 8 | uint32_t(in[p + 2]) << 16 | uint32_t(in[p + 3]) << 24;
        else v = ld8(in, p, n) | ld8(in, p + 1, n) << 8 | ld8(in, p + 2, n) << 16 | ld8(in, p + 3, n) << 24;
        reinterpret_cast<uint32_t*>(win)[i] = v;
    }
}

struct SnapLane {
    uint32_t valid;      // token starts in this lane's segment (bit i = window offset lane*SEG + i)
    uint64_t exit;       // first true token start at/after the segment end (window-relative)
    int committed;       // lane is part of the consistent prefix
};

// Parse the window whose byte 0 is a true token start. `limit` = window-relative end of the
// parse (stream end, or the piece's input end). Returns the window-relative exit of the last
// committed lane (the next window's entry).
__device__ inline uint64_t snap_parse_window(const uint8_t* win, uint64_t limit, SnapLane& L) {
    const int lane = threadIdx.x & 63;
    const uint32_t ss = uint32_t(lane) * SNAP_SEG;
    const uint64_t se = min<uint64_t>(uint64_t(ss) + SNAP_SEG, limit);
    // speculative chain from the segment start
    uint32_t mask = 0;
    uint64_t pos = ss;
    while (pos < se) {
        mask |= 1u << uint32_t(pos - ss);
        pos += snap_toklen(win, uint32_t(pos));
    }
    const uint64_t spec_exit = (ss < limit) ? pos : uint64_t(ss);
    uint64_t entry = ss, ex = spec_exit;
    uint32_t valid = mask;
    // fixed-point iteration of entries
    int changed = 1;
    for (int r = 0; r < SNAP_ROUNDS && changed; r++) {
        uint64_t prev_exit = __shfl_up(ex, 1, 64);
        uint64_t e = lane == 0 ? 0 : prev_exit;
        bool ch = (e != entry);
        if (ch) {
            entry = e;
            if (e >= se) {                       // skipped by a long token (or past the limit)
                valid = 0;
                ex = e;
            } else if ((mask >> uint32_t(e - ss)) & 1u) {
                valid = mask & ~((1u << uint32_t(e - ss)) - 1u);
                ex = spec_exit;
            } else {                             // walk from the true entry until the chains merge
                uint32_t fix = 0;
                uint64_t q = e;
                while (q < se && !((mask >> uint32_t(q - ss)) & 1u)) {
                    fix |= 1u << uint32_t(q - ss);
                    q += snap_toklen(win, uint32_t(q));
                }
                if (q < se) { valid = fix | (mask & ~((1u << uint32_t(q - ss)) - 1u)); ex = spec_exit; }
                else { valid = fix; ex = q; }
            }
        }
        changed = __any(ch) ? 1 : 0;
    }
    // consistent prefix: lane 0 always; lane l if its entry equals lane l-1's exit
    uint64_t prev_exit = __shfl_up(ex, 1, 64);
    bool cons = lane == 0 || entry == prev_exit;
    uint64_t bad = __ballot(!cons);
    int f = bad ? __ffsll((unsigned long long)bad) - 1 : 64;
    L.committed = lane < f;
    L.valid = L.committed ? valid : 0;
    L.exit = ex;
    uint64_t last_exit = __shfl(ex, f - 1, 64);
    return last_exit;
}

}  // namespace pf
