// pf_snappy_par.h — Snappy token helpers for the block-parallel decompressor (device).
//
// Raw Snappy tokens (tag byte t, kind = t & 3):
//   0 literal : length-1 in t>>2; 60..63 -> 1..4 little-endian length bytes follow; then data
//   1 copy    : length 4 + ((t>>2)&7), offset ((t>>5)<<8) | next byte
//   2 copy    : length (t>>2)+1, 16-bit LE offset
//   3 copy    : length (t>>2)+1, 32-bit LE offset
#pragma once
#include "pf_device.h"

namespace pf {


constexpr uint32_t SNAP_RB = 128;                 // input bytes per lane region (index pass)
constexpr uint32_t SNAP_WIN = 64 * SNAP_RB;       // 8 KiB of input per index window
constexpr uint32_t SNAP_WSTAGE = SNAP_WIN + 96;   // staged window: + alignment shift (< 16) + 64-lane lookahead
constexpr uint32_t SNAP_WWORDS = SNAP_WIN / 32;   // token-start bitmap words per window
constexpr uint32_t SNAP_INVALID = 0xffffffffu;
constexpr uint32_t SNAP_BLOCK = 65536;            // Google Snappy block = executor piece

// per-job decode path (SnappyJob fallback flags, ordered: atomicMax escalates)
// FB_INPLACE: the page needs no decompression (one literal, k_snappy_head); FB_LITCOPY: a page whose
// stream is at most LC_MAX literals and nothing else, copied to its scratch body by k_snappy_litcopy.
// Every parse / executor kernel skips both.
constexpr uint32_t LC_MAX = 32;   // literals of a FB_LITCOPY job (its table lives in its token bitmap)
enum : int { FB_OK = 0, FB_WHOLE = 1, FB_REDO = 2, FB_SERIAL = 3, FB_INPLACE = 4, FB_LITCOPY = 5 };
// SnapWin.flags
enum : uint32_t { WIN_BROKEN = 1, WIN_PASS = 2, WIN_NOCONV = 4 };
// SnapWin.flags after the chain pass: how the window's bitmap relates to the true chain
enum : uint32_t { WM_KEEP = 16, WM_SKIP = 17, WM_MERGE = 18, WM_FULL = 19, WM_DONE = 20 };

// Result of the index pass for one 8 KiB input window.
struct SnapWin {
    uint32_t entry;   // chain start the window's bitmap was built from
    uint32_t exit;    // first chain position at/after the window end (or the stream end)
    uint32_t out;     // output bytes of the tokens in the window (on that chain)
    uint32_t flags;
};

// Entry-table record (pos carries a 2-bit flag in its top bits).
struct SnapEnt {
    uint32_t pos;
    uint32_t out;
};

struct SnapTok {
    uint64_t tl;      // input bytes (tag + operands + literal data); 64-bit: garbage lengths
    uint32_t ol;      // output bytes
    uint32_t kind;    // 0 literal, 1..3 copy
    uint32_t arg;     // literal: header bytes (1..5); copy: offset
};

// Decode the token whose tag is the low byte of v (v = the 8 stream bytes from the tag on).
// Branch-free (selects), so lanes holding different token kinds do not diverge.
__device__ __forceinline__ SnapTok snap_tok(uint64_t v) {
    SnapTok t;
    const uint32_t tag = uint32_t(v) & 0xffu;
    const uint32_t L = tag >> 2;
    const uint32_t b1 = uint32_t(v >> 8);                             // the 4 bytes after the tag
    const uint32_t kind = tag & 3u;
    // literal: length-1 in L, or in 1..4 little-endian bytes after the tag when L >= 60
    const uint32_t nb = L >= 60 ? L - 59 : 0u;
    const uint32_t lmask = nb >= 4 ? 0xffffffffu : ((1u << (8u * nb)) - 1u);
    const uint32_t lit_ol = (L < 60 ? L : (b1 & lmask)) + 1u;          // 0 only for a 4 GiB literal
    const uint32_t lit_arg = 1u + nb;
    const uint64_t lit_tl = uint64_t(lit_arg) + (lit_ol ? uint64_t(lit_ol) : (1ull << 32));
    t.kind = kind;
    t.ol = kind == 0 ? lit_ol : (kind == 1 ? 4u + (L & 7u) : L + 1u);
    t.arg = kind == 0 ? lit_arg
                      : (kind == 1 ? (((tag >> 5) << 8) | (b1 & 0xffu)) : (kind == 2 ? (b1 & 0xffffu) : b1));
    t.tl = kind == 0 ? lit_tl : uint64_t(kind == 1 ? 2u : (kind == 2 ? 3u : 5u));
    return t;
}

// 32-bit form for the executor's producer (round 6): straight-line selects (the 64-bit form compiles to
// branches on the token kind), tl saturated at 0xffffffff (a 4 GiB literal), from the 8 stream bytes
// lo | hi << 32 starting at the tag.
struct SnapTok32 {
    uint32_t tl, ol, kind, arg;
};
__device__ __forceinline__ SnapTok32 snap_tok32(uint32_t lo, uint32_t hi) {
    const uint32_t tag = lo & 0xffu, kind = tag & 3u, L = tag >> 2;
    const uint32_t b1 = __builtin_amdgcn_alignbyte(hi, lo, 1u);       // the 4 bytes after the tag
    const uint32_t nb = L >= 60u ? L - 59u : 0u;                      // literal length bytes (1..4)
    const uint32_t lmask = nb >= 4u ? 0xffffffffu : ~(0xffffffffu << (8u * nb));
    const uint32_t lit_ol = (L < 60u ? L : (b1 & lmask)) + 1u;        // 0: a 4 GiB literal
    const uint32_t lit_tl = lit_ol == 0u ? 0xffffffffu : __builtin_elementwise_add_sat(1u + nb, lit_ol);
    const uint32_t cp_ol = kind == 1u ? 4u + (L & 7u) : L + 1u;
    const uint32_t sh = (0x00101800u >> (8u * kind)) & 0xffu;         // offset bytes: kind 1 -> 1, 2 -> 2, 3 -> 4
    const uint32_t cp_off = (b1 & (0xffffffffu >> sh)) | (kind == 1u ? ((tag >> 5) << 8) : 0u);
    const uint32_t cp_tl = (0x05030200u >> (8u * kind)) & 0xffu;
    const bool lit = kind == 0u;
    return SnapTok32{lit ? lit_tl : cp_tl, lit ? lit_ol : cp_ol, kind, lit ? 1u + nb : cp_off};
}

// 8 bytes from LDS at byte offset a as two dwords, branch-free (three aligned dword reads; a + 8 + 3 staged).
__device__ __forceinline__ void lds_read8_2(const uint8_t* s, uint32_t a, uint32_t& lo, uint32_t& hi) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], sh = a & 3u;
    lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
    hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
}

// Token lengths from the tag byte alone (literals with a length field, tag_long, need snap_tok).
__device__ __forceinline__ uint32_t tag_tl(uint32_t tag) {   // input bytes (branch-free)
    const uint32_t kind = tag & 3u;
    const uint32_t lit = uint32_t(int32_t(kind - 1u) >> 31);        // all ones for a literal
    return ((0x05030200u >> (kind << 3)) & 0xffu) | (((tag >> 2) + 2u) & lit);
}
__device__ __forceinline__ uint32_t tag_ol(uint32_t tag) {   // output bytes (branch-free)
    const uint32_t L = tag >> 2;
    const uint32_t c1 = uint32_t(-int32_t((tag & 3u) == 1u));     // all ones for a 1-byte-offset copy
    return ((4u + (L & 7u)) & c1) | ((L + 1u) & ~c1);
}
__device__ __forceinline__ bool tag_long(uint32_t tag) { return (tag & 3u) == 0u && tag >= 240u; }

// 8 bytes from LDS at byte offset a (two aligned dword reads; a + 8 + 3 must be staged).
__device__ __forceinline__ uint64_t lds_read8(const uint8_t* s, uint32_t a) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
    const uint64_t v = uint64_t(w[0]) | (uint64_t(w[1]) << 32);
    const uint32_t sh = 8u * (a & 3u);
    return sh ? ((v >> sh) | (uint64_t(w[2]) << (64u - sh))) : v;
}

// 8 bytes from global memory at in[p], zero past n.
__device__ __forceinline__ uint64_t glb_read8(const uint8_t* in, uint64_t n, uint64_t p) {
    const PF_GLOBAL uint8_t* g = gptr(in);
    uint64_t v = 0;
    #pragma unroll
    for (int i = 0; i < 8; i++)
        if (p + i < n) v |= uint64_t(g[p + i]) << (8 * i);
    return v;
}

// Stage input bytes [base - woff, base - woff + bytes) into LDS with 16-byte loads; woff (0..15)
// is base's misalignment, so stream byte base + i is stage[woff + i]. 16-byte chunks wholly at or
// past n are zero; the chunk holding the last valid byte is read whole (it never crosses a page).
__device__ __forceinline__ uint32_t snap_stage(uint8_t* stage, const uint8_t* in, uint64_t n, uint64_t base,
                                               uint32_t bytes, int lane) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(in + base);
    const uint32_t woff = uint32_t(a & 15u);
    const PF_GLOBAL u32x4* src = (const PF_GLOBAL u32x4*)(a - woff);
    const int64_t first = int64_t(base) - int64_t(woff);
    const uint32_t nch = bytes / 16;
    // STAGE_U loads a lane in flight before their stores (round 6: one load -> store round trip per
    // chunk serialised the 9 global latencies of an 8 KiB window)
    constexpr uint32_t STAGE_U = 8;
    for (uint32_t c0 = uint32_t(lane); c0 < nch; c0 += 64u * STAGE_U) {
        u32x4 v[STAGE_U];
        #pragma unroll
        for (uint32_t u = 0; u < STAGE_U; u++) {
            const uint32_t c = c0 + 64u * u;
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (c < nch && first + int64_t(c) * 16 < int64_t(n)) v[u] = src[c];
        }
        #pragma unroll
        for (uint32_t u = 0; u < STAGE_U; u++) {
            const uint32_t c = c0 + 64u * u;
            if (c < nch) reinterpret_cast<u32x4*>(stage)[c] = v[u];
        }
    }
    return woff;
}

}  // namespace pf
