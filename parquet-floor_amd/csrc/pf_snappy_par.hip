// pf_snappy_par.hip — K1: block-parallel Snappy page decompression.
//
// Replaces snappy-java's Snappy.uncompress behind the Hadoop codec shim
// (src/main/java/org/apache/hadoop/io/compress/DecompressorStream.java:61-70,101-173).
//
// Google Snappy (what snappy-java wraps) compresses in independent 64 KiB blocks: no copy reaches
// back across a block boundary and a token starts exactly at every multiple of 65536 of the output.
// A page therefore splits into 64 KiB pieces that decode independently, once the token chain is
// known. Four kernels:
//
//   k_snappy_index  one wave per 8 KiB window of compressed input (all pages). Each lane walks the
//                   token chain of its 128-byte region from the region start (a guess: the true
//                   chain usually enters a little later). A scalar pass then follows the chain
//                   lane to lane from the window entry; a lane whose true entry is not on its
//                   guessed chain re-walks from it, until the chain is consistent (each round
//                   fixes at least the first wrong lane). Output: the token-start bitmap (1 bit per
//                   input byte), per-lane output byte counts, the window exit, and an entry
//                   table: for each entry d < 64 bytes into the window, where the chain from
//                   W0 + d meets the window's chain and the output difference up to there.
//   k_snappy_chain  one wave per page. Window w's true entry is window w-1's exit: one table
//                   lookup per window (a walk in HBM for entries deeper than 64 bytes, a whole-
//                   wave re-parse for unresolved windows). Lanes then repair the bitmap in front
//                   of the merge points, the totals are checked and the input position of the
//                   token at each 64 KiB output boundary is found.
//   k_snappy_exec   one wave per 64 KiB piece: tokens come from the bitmap 1 KiB of input at a
//                   time (parsed 64 at a time, one per lane), then execute in order — each token
//                   is one 64-lane read-then-write step in an 8 KiB LDS ring (copies with larger
//                   offsets read the already-flushed HBM output); full 2 KiB ring slots are
//                   flushed with 16-byte stores.
//   k_snappy_serial (pf_snappy.hip) any page whose stream breaks the block structure or is
//                   corrupt is re-decoded serially — results never depend on the assumption.
#include <hip/hip_runtime.h>


#include "pf_snappy_par.h"

namespace pf {

#ifdef PF_STAMPS
__device__ unsigned long long pf_stamps[16];
#define STAMP_ADD(i, v) atomicAdd(&pf_stamps[i], (unsigned long long)(v))
__device__ unsigned long long pf_cstamps[32];
#define CSTAMP(i, v) atomicAdd(&pf_cstamps[i], (unsigned long long)(v))
extern "C" int pf_debug_cstamps(unsigned long long* out, int n, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_cstamps), sizeof(unsigned long long) * (n < 32 ? n : 32)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pf_cstamps), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#define XT_DECL unsigned long long xt_ = __builtin_amdgcn_s_memtime()
#define XT(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (lane == 0) STAMP_ADD(i, t_ - xt_); xt_ = t_; } while (0)
#else
#define STAMP_ADD(i, v) ((void)0)
#define CSTAMP(i, v) ((void)0)
#define XT_DECL ((void)0)
#define XT(i) ((void)0)
#endif

// ======================================================================== index pass

struct WinLane {
    uint32_t b0, b1, b2, b3;   // token starts in the lane's region (bit i = input byte rs + i)
    uint32_t out;              // output bytes of those tokens
    uint32_t x;                // chain exit (first position >= region end), SNAP_INVALID past the stream
    uint32_t c;                // chain start
};

__device__ __forceinline__ void bit_set(WinLane& L, uint32_t i) {
    const uint32_t m = 1u << (i & 31u), w = i >> 5;
    L.b0 |= w == 0 ? m : 0u;
    L.b1 |= w == 1 ? m : 0u;
    L.b2 |= w == 2 ? m : 0u;
    L.b3 |= w == 3 ? m : 0u;
}
__device__ __forceinline__ void bit_clr(WinLane& L, uint32_t i) {
    const uint32_t m = 1u << (i & 31u), w = i >> 5;
    L.b0 &= w == 0 ? ~m : ~0u;
    L.b1 &= w == 1 ? ~m : ~0u;
    L.b2 &= w == 2 ? ~m : ~0u;
    L.b3 &= w == 3 ? ~m : ~0u;
}
__device__ __forceinline__ bool bit_get(const WinLane& L, uint32_t i) {
    const uint32_t w = i >> 5;
    const uint32_t v = w == 0 ? L.b0 : (w == 1 ? L.b1 : (w == 2 ? L.b2 : L.b3));
    return (v >> (i & 31u)) & 1u;
}

// ---- padded window stage: lane region k (input bytes [W0 + 128k, W0 + 128k + 140)) sits at
// sp + 140k, so 64 lanes reading the same offset of their own regions hit 64 different LDS banks
// (140 B = 35 dwords, odd) and an 8-byte token read at any region offset < 128 stays in the copy.
constexpr uint32_t SNAP_PB = 140;
constexpr uint32_t SNAP_PSTAGE = 64 * SNAP_PB;
constexpr uint32_t XS_SAT = 0x7fffu;       // saturated region exit (a literal longer than ~32 KiB)

// n >= 1. Dwords holding no stream byte are never read (zero instead).
__device__ void stage_pad(uint8_t* sp, const uint8_t* in, uint64_t n, uint32_t W0, int lane) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(in);
    const uintptr_t lastw = (base + n - 1) & ~uintptr_t(3);
    constexpr uint32_t PU = 8;   // dwords a lane in flight before their stores (round 6: 35 serial round trips)
    for (uint32_t i0 = uint32_t(lane); i0 < SNAP_PSTAGE / 4; i0 += 64u * PU) {
        uint32_t lo[PU], hi[PU], sh[PU];
        #pragma unroll
        for (uint32_t u = 0; u < PU; u++) {
            const uint32_t idx = i0 + 64u * u;
            const uint32_t k = idx / (SNAP_PB / 4), jd = idx - k * (SNAP_PB / 4);
            const uintptr_t a = base + W0 + k * SNAP_RB + jd * 4;
            const uintptr_t a0 = a & ~uintptr_t(3);
            const bool in_range = idx < SNAP_PSTAGE / 4;
            lo[u] = in_range && a0 <= lastw ? *(const PF_GLOBAL uint32_t*)a0 : 0u;
            hi[u] = in_range && a0 + 4 <= lastw ? *(const PF_GLOBAL uint32_t*)(a0 + 4) : 0u;
            sh[u] = uint32_t(a & 3u);
        }
        #pragma unroll
        for (uint32_t u = 0; u < PU; u++) {
            const uint32_t idx = i0 + 64u * u;
            if (idx < SNAP_PSTAGE / 4) reinterpret_cast<uint32_t*>(sp)[idx] = __builtin_amdgcn_alignbyte(hi[u], lo[u], sh[u]);
        }
    }
}

// 8 stream bytes from window offset r (< 8 KiB) of a padded stage.
__device__ __forceinline__ uint64_t pad_read8(const uint8_t* sp, uint32_t r) {
    return lds_read8(sp, (r >> 7) * SNAP_PB + (r & 127u));
}

// Input / output bytes of the token at window offset r of a padded stage.
__device__ __forceinline__ uint64_t pad_tok(const uint8_t* sp, uint32_t r, uint32_t& ol) {
    const uint32_t a = (r >> 7) * SNAP_PB + (r & 127u);
    const uint32_t tag = (*reinterpret_cast<const uint32_t*>(sp + (a & ~3u)) >> (8u * (a & 3u))) & 0xffu;
    if (!tag_long(tag)) {
        ol = tag_ol(tag);
        return tag_tl(tag);
    }
    const SnapTok t = snap_tok(lds_read8(sp, a));
    ol = t.ol;
    return t.tl;
}

constexpr int WIN_ROUNDS = 66;       // lane-region fixed-point rounds: each fixes at least the first wrong lane,
                                     // so 64 + 1 always converge (seq_parse stays as a guard)

// Input / output bytes of the token at stage offset a (linear stage; tag decode unless a literal
// carries a length field).
__device__ __forceinline__ uint64_t stage_tok(const uint8_t* stage, uint32_t a, uint32_t& ol) {
    const uint32_t tag = stage[a];
    if (!tag_long(tag)) {
        ol = tag_ol(tag);
        return tag_tl(tag);
    }
    const SnapTok t = snap_tok(lds_read8(stage, a));
    ol = t.ol;
    return t.tl;
}

// The token at stream position p of a linear stage (base = stage offset of position 0): the tag and the 3
// bytes after it from one aligned dword pair; straight-line lengths (a literal length field of 4 bytes,
// >= 16 MiB, cannot be in a page: tl = 0xffffffff breaks the chain).
__device__ __forceinline__ void walk_tok(const uint8_t* stage, uint32_t base, uint32_t p, uint32_t& ol, uint32_t& tl) {
    const uint32_t a = base + p;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(stage + (a & ~3u));
    const uint32_t v = __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
    const uint32_t tag = v & 0xffu, kind = tag & 3u, Lv = tag >> 2;
    const uint32_t nb = Lv >= 60u ? Lv - 59u : 0u;
    const uint32_t lit_ol = (Lv < 60u ? Lv : ((v >> 8) & ((1u << (8u * min(nb, 3u))) - 1u))) + 1u;
    const uint32_t lit_tl = nb >= 4u ? 0xffffffffu : 1u + nb + lit_ol;
    // (selects as bit masks: v_bfi, where the compiler would branch on the kind)
    const uint32_t mlit = 0u - uint32_t(kind == 0u), m1 = 0u - uint32_t(kind == 1u);
    const uint32_t cp_ol = ((4u + (Lv & 7u)) & m1) | ((Lv + 1u) & ~m1);
    tl = (lit_tl & mlit) | (((0x05030200u >> (8u * kind)) & 0xffu) & ~mlit);
    ol = (lit_ol & mlit) | (cp_ol & ~mlit);
}

// Walk the chain from c while positions stay below re (bits relative to rs). The token-start bits are
// OR-ed into the lane's four LDS words lb (one ds_or per token, no register selects; round 6) and read
// back into L at the end.
__device__ void lane_walk(const uint8_t* stage, uint32_t woff, uint32_t W0, uint64_t n, uint32_t rs, uint32_t re,
                          uint32_t c, WinLane& L, uint32_t* lb) {
    *reinterpret_cast<uint4*>(lb) = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t n32 = uint32_t(n);   // (< 2^32 - 1: 0xffffffff marks a broken chain)
    const uint32_t base = woff - W0;    // stage offset of stream position p: base + p
    uint32_t out = 0, p = c;
    L.c = c;
    while (p < re) {
        uint32_t ol, tl;
        walk_tok(stage, base, p, ol, tl);
        const uint32_t i = p - rs;
        atomicOr(lb + (i >> 5), 1u << (i & 31u));
        out = __builtin_elementwise_add_sat(out, ol);
        const uint32_t np = __builtin_elementwise_add_sat(p, tl);
        p = np > n32 ? 0xffffffffu : np;
    }
    const uint4 bv = *reinterpret_cast<const uint4*>(lb);
    L.b0 = bv.x; L.b1 = bv.y; L.b2 = bv.z; L.b3 = bv.w;
    L.out = out;
    L.x = p;   // (SNAP_INVALID when the chain ran past the stream end)
}

// Speculative parse of one window whose chain enters at `entry` (W0 <= entry < min(W0 + SNAP_WIN,
// n)), all 64 lanes, linear stage. Each lane walks the chain of its 128-byte region from the region
// start (a guess: chains started anywhere usually meet the true one within a few tokens); a scalar
// walk then follows the chain lane to lane from the entry, and a lane whose true entry is not on
// its guessed chain re-walks from it, until consistent (each round fixes at least the first wrong
// lane). Returns the window exit; flags = WIN_BROKEN if the chain runs past the stream end,
// WIN_NOCONV if max_rounds did not converge.
__device__ uint32_t win_parse_spec(const uint8_t* stage, uint32_t woff, uint32_t W0, uint64_t n, uint32_t entry,
                                   WinLane& L, uint32_t& flags, uint32_t* lbits, int max_rounds = WIN_ROUNDS) {
    const int lane = threadIdx.x & 63;
    uint32_t* const lb = lbits + 4 * lane;   // the lane's bit words (SNAP_WWORDS words of LDS for the wave)
    const uint32_t rs = W0 + uint32_t(lane) * SNAP_RB;
    const uint32_t re = uint32_t(min(uint64_t(rs) + SNAP_RB, n));
    entry = __builtin_amdgcn_readfirstlane(entry);
    const uint32_t L0 = (entry - W0) / SNAP_RB;
    L.b0 = L.b1 = L.b2 = L.b3 = 0;
    L.out = 0;
    L.c = rs;
    L.x = SNAP_INVALID;
    if (uint32_t(lane) >= L0 && uint64_t(rs) < n) lane_walk(stage, woff, W0, n, rs, re, uint32_t(lane) == L0 ? entry : rs, L, lb);
    uint32_t ent = SNAP_INVALID, X = SNAP_INVALID;
    bool converged = false;
    flags = 0;
    for (int round = 0; round < max_rounds; round++) {
        // follow the chain lane to lane. Fast-forward: while each lane's exit lands in the next lane's
        // region the entries are just the previous lanes' exits (one shuffle); from the first lane
        // where that fails, a uniform scalar walk.
        flags = 0;
        const uint32_t xk = L.x;
        const bool ok = uint32_t(lane) >= L0 && xk != SNAP_INVALID && uint64_t(xk) < n && xk < W0 + SNAP_WIN &&
                        (xk - W0) / SNAP_RB == uint32_t(lane) + 1;
        const uint64_t notok = ~__ballot(ok) & (~0ull << L0);
        const uint32_t la = notok ? uint32_t(__ffsll((unsigned long long)notok) - 1) : 63u;
        const uint32_t xprev = __shfl_up(xk, 1, 64);
        ent = uint32_t(lane) == L0 ? entry : ((uint32_t(lane) > L0 && uint32_t(lane) <= la) ? xprev : SNAP_INVALID);
        uint32_t k = la, e = __builtin_amdgcn_readlane(ent, int(la));
        for (;;) {
            ent = uint32_t(lane) == k ? e : ent;
            const uint32_t x = __builtin_amdgcn_readlane(L.x, int(k));
            if (x == SNAP_INVALID) { flags = WIN_BROKEN; X = SNAP_INVALID; break; }
            if (uint64_t(x) >= n || x >= W0 + SNAP_WIN) { X = x; break; }
            k = (x - W0) / SNAP_RB;
            e = x;
        }
        const bool need = ent != SNAP_INVALID && ent != L.c && !(ent > L.c && bit_get(L, ent - rs));
        if (!__any(need)) { converged = true; break; }
#ifdef PF_STAMPS
        if (lane == 0) { CSTAMP(7, 1); CSTAMP(8, __popcll(__ballot(need))); }
#else
        (void)__ballot(need);
#endif
        if (need) lane_walk(stage, woff, W0, n, rs, re, ent, L, lb);
    }
    if (!converged) flags = WIN_NOCONV;
    // lanes off the chain hold no tokens; drop the guessed prefix before a lane's true entry
    if (ent == SNAP_INVALID) {
        L.b0 = L.b1 = L.b2 = L.b3 = 0;
        L.out = 0;
    } else if (ent > L.c) {
        uint32_t p = L.c;
        while (p < ent) {
            uint32_t ol;
            const uint64_t tl = stage_tok(stage, woff + (p - W0), ol);
            bit_clr(L, p - rs);
            L.out -= ol;
            p += uint32_t(tl);
        }
        L.c = ent;
    }
    return X;
}

// Entry table (index pass -> chain pass): for an entry e = W0 + d, d < 64, where the chain from e
// meets the window's own chain (bitmap) and the output difference up to that point.
constexpr int ENT_STEPS = 384;       // longer walks are left to the chain pass (exact lane-region parse)
constexpr uint32_t ENT_POS = 0x3fffffffu;
enum : uint32_t { ENT_MERGE = 0, ENT_NOMERGE = 1, ENT_SLOW = 2, ENT_BAD = 3 };

__device__ __forceinline__ SnapEnt mk_ent(uint32_t pos, uint32_t flag, uint32_t out) {
    return SnapEnt{pos | (flag << 30), out};
}

// MERGE: pos = meeting point m, out = (true chain output in [e, m)) - (window chain output in
// [W0, m)). NOMERGE: the chain from e leaves the window first: pos = its exit, out = its output.
// SLOW: not resolved within ENT_STEPS tokens. BAD: the chain from e runs past the stream end.
// Linear stage; sb = the window chain's token-start bits, pre[r] = its output before lane region r.
__device__ SnapEnt ent_walk(uint32_t e, uint32_t W0, uint64_t wend, uint64_t n, const uint8_t* stage, uint32_t woff,
                            const uint32_t* sb, const uint32_t* pre) {
    uint64_t q = e;
    uint32_t acc = 0;
    int steps = 0;
    for (;;) {
        if (q >= wend) return mk_ent(uint32_t(q), ENT_NOMERGE, acc);
        const uint32_t r = uint32_t(q) - W0;
        if ((sb[r >> 5] >> (r & 31u)) & 1u) break;
        if (steps == ENT_STEPS) return mk_ent(e, ENT_SLOW, 0);
        uint32_t ol;
        const uint64_t tl = stage_tok(stage, woff + r, ol);
        acc += ol;
        q += tl;
        steps++;
        if (q > n) return mk_ent(e, ENT_BAD, 0);
    }
    const uint32_t rel = uint32_t(q) - W0, rq = rel / SNAP_RB;
    uint32_t g = pre[rq];
    for (uint32_t b = rq * SNAP_RB; b < rel; b += 32) {
        const uint32_t hi = rel - b >= 32 ? 0xffffffffu : ((1u << (rel - b)) - 1u);
        uint32_t mm = sb[b >> 5] & hi;
        while (mm) {
            const uint32_t i = b + uint32_t(__ffs(mm) - 1);
            mm &= mm - 1;
            uint32_t ol;
            stage_tok(stage, woff + i, ol);
            g += ol;
        }
    }
    return mk_ent(uint32_t(q), ENT_MERGE, acc - g);
}

__device__ __forceinline__ uint32_t wave_sum_sat(uint32_t v) {
    uint64_t s = v;
    #pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    return s > 0xffffffffull ? 0xffffffffu : uint32_t(s);
}

// Exact whole-wave parse of the chain from e (a token start, W0 <= e < stop) up to the first chain
// position >= stop, on a staged window. 64 lanes decode the token at cur + lane; the chain through
// those 64 candidates is followed in scalar registers (readlane) and its 64-bit start mask is
// OR-ed into sbits (bit i = W0 + i) by one lane. Afterwards every lane sums the output lengths of
// the tokens in its SNAP_RB region into slo. sbits must be zero on entry. Returns the exit
// (SNAP_INVALID if the chain runs past n) and the output byte total in `out`.
__device__ uint32_t seq_parse(const uint8_t* stage, uint32_t woff, uint32_t W0, uint64_t n, uint32_t e, uint64_t stop,
                              uint32_t* sbits, uint32_t* slo, uint32_t& out) {
    const int lane = threadIdx.x & 63;
    uint64_t cur = e;
    out = 0;
    bool bad = false;
    while (cur < stop) {
        const uint64_t q = cur + uint64_t(lane);
        const SnapTok t = snap_tok(lds_read8(stage, woff + uint32_t(q - W0)));
        const uint32_t tl = t.tl > 0x7fffffffull ? 0x7fffffffu : uint32_t(t.tl);
        const uint32_t lim = uint32_t(min<uint64_t>(64, stop - cur));
        uint32_t k = 0;
        uint64_t mask = 0;
        while (k < lim) {
            mask |= 1ull << k;
            k += __builtin_amdgcn_readlane(tl, k);
        }
        if (lane == 0) {
            const uint32_t r0 = uint32_t(cur - W0), wi = r0 >> 5, sh = r0 & 31u;
            sbits[wi] |= uint32_t(mask << sh);
            const uint32_t m1 = sh ? uint32_t(mask >> (32u - sh)) : uint32_t(mask >> 32);
            const uint32_t m2 = sh ? uint32_t(mask >> (64u - sh)) : 0u;
            if (m1 && wi + 1 < SNAP_WWORDS) sbits[wi + 1] |= m1;
            if (m2 && wi + 2 < SNAP_WWORDS) sbits[wi + 2] |= m2;
        }
        cur += k;
        if (cur > n) { bad = true; break; }
    }
    __syncthreads();
    // output bytes per lane region, from the marked tokens
    uint32_t acc = 0;
    #pragma unroll
    for (int kw = 0; kw < 4; kw++) {
        uint32_t m = sbits[lane * 4 + kw];
        while (m) {
            const uint32_t i = uint32_t(lane) * SNAP_RB + uint32_t(kw) * 32u + uint32_t(__ffs(m) - 1);
            m &= m - 1;
            const uint32_t o = snap_tok(lds_read8(stage, woff + i)).ol;
            acc = acc + o < acc ? 0xffffffffu : acc + o;
        }
    }
    slo[lane] = acc;
    if (bad) return SNAP_INVALID;
    out = wave_sum_sat(acc);
    return uint32_t(cur);
}

// Exact parse of the 8 KiB window at W0 whose chain enters at `entry` (W0 <= entry < min(W0 + 8 KiB,
// n)), all 64 lanes, lane k owning input region k. (1) Every offset i of the region is decoded as
// if a token started there: xs[i][k] = i + token length when that is inside the region, else the
// tagged offset the token ends at. (2) A backward pass turns this into the region exit of the
// chain from every offset (tokens are >= 2 bytes, so offsets i and i-1 never depend on each other:
// two per LDS round trip). Offsets at or past the stream end stop every chain (a chain stepping
// over n is broken). (3) The true chain crosses the regions with one lookup per region (offsets
// < 8 from registers). (4) Each lane walks the true chain through its region: token-start bits and
// output bytes. Returns the window exit (SNAP_INVALID: broken); a saturated exit falls back to the
// exact whole-wave parse on a linear stage (xs reused). sp must be staged (stage_pad) and synced.
__device__ uint32_t win_parse(const uint8_t* in, uint64_t n, uint32_t W0, uint32_t entry, const uint8_t* sp,
                              uint16_t* xs, uint32_t* sbits, uint32_t* slo, WinLane& L) {
    const int lane = threadIdx.x & 63;
    const uint32_t rs = W0 + uint32_t(lane) * SNAP_RB;
    const int64_t nrel = int64_t(n) - int64_t(rs);
    const uint8_t* mine = sp + uint32_t(lane) * SNAP_PB;
#ifdef PF_STAMPS
    unsigned long long pt0 = __builtin_amdgcn_s_memtime();
#define PT(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (lane == 0) CSTAMP(i, t_ - pt0); pt0 = t_; } while (0)
#else
#define PT(i) ((void)0)
#endif
    // (1) + (2), 8 offsets at a time from the region end: their tags (and literal length fields)
    // come from 4 LDS dwords; an exit inside the group is resolved in registers, one beyond it is
    // read from xs (final already)
    uint32_t c[8];
    for (int g = SNAP_RB / 8 - 1; g >= 0; g--) {
        const uint32_t* mw = reinterpret_cast<const uint32_t*>(mine) + 2 * g;
        const uint32_t d[4] = {mw[0], mw[1], mw[2], mw[3]};
        uint32_t tl[8];
        bool any_long = false;
        #pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const uint32_t tag = (d[jj >> 2] >> (8 * (jj & 3))) & 0xffu;
            tl[jj] = tag_tl(tag);
            any_long |= tag_long(tag);
        }
        if (__any(any_long)) {
            #pragma unroll
            for (int jj = 0; jj < 8; jj++) {
                const uint32_t tag = (d[jj >> 2] >> (8 * (jj & 3))) & 0xffu;
                const int q = (jj + 1) >> 2, sh = (jj + 1) & 3;
                const uint32_t b1 = __builtin_amdgcn_alignbyte(d[q + 1], d[q], uint32_t(sh));
                const uint32_t nb = (tag >> 2) - 59u;
                const uint32_t len = b1 & (nb >= 4u ? 0xffffffffu : (1u << (8u * nb)) - 1u);
                if (tag_long(tag)) tl[jj] = len >= XS_SAT ? XS_SAT : 2u + nb + len;
            }
        }
        uint32_t res[8];   // 0x8000 | exit offset, or an offset beyond the group to take the exit of
        #pragma unroll
        for (int jj = 7; jj >= 0; jj--) {
            const uint32_t i = uint32_t(8 * g + jj);
            const uint32_t nx = i + tl[jj];
            uint32_t r = nx >= SNAP_RB ? (0x8000u | min(nx, XS_SAT)) : nx;
            #pragma unroll
            for (int m = jj + 2; m < 8; m++) r = nx == uint32_t(8 * g + m) ? res[m] : r;
            if (int64_t(i) >= nrel) r = 0x8000u | i;
            res[jj] = r;
        }
        uint32_t rd[8];
        #pragma unroll
        for (int jj = 0; jj < 8; jj++) rd[jj] = xs[((res[jj] & 0x8000u) ? uint32_t(8 * g + jj) : res[jj]) * 64 + lane];
        #pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            c[jj] = (res[jj] & 0x8000u) ? (res[jj] & 0x7fffu) : rd[jj];
            xs[(8 * g + jj) * 64 + lane] = uint16_t(c[jj]);
        }
    }
    PT(21);
    PT(22);
    // (3) region entries by a prefix over the lanes of entry maps: lane k's map sends an entry
    // offset d < 8 to the offset its chain enters region k+1 at (8: not below 8 there, or it
    // leaves otherwise). The chain is exact up to the first lane the maps lose it at; from there a
    // scalar walk follows it region by region.
    uint32_t e = __builtin_amdgcn_readfirstlane(entry);
    const uint32_t L0 = (e - W0) >> 7, d0 = e - W0 - (L0 << 7);
    uint32_t ent = SNAP_INVALID;
    if (d0 < 8) {
        uint32_t P = 0;
        #pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t o = c[q] - SNAP_RB;
            P |= (o < 8u ? o : 8u) << (4 * q);
        }
        if (uint32_t(lane) < L0) P = 0x76543210u;   // identity
        #pragma unroll
        for (int h = 1; h < 64; h <<= 1) {
            uint32_t A = __shfl_up(P, h, 64);
            if (lane < h) A = 0x76543210u;
            uint32_t np = 0;
            #pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t a = (A >> (4 * q)) & 15u;
                np |= (a >= 8u ? 8u : (P >> (4u * a)) & 15u) << (4 * q);
            }
            P = np;
        }
        const uint32_t Pp = __shfl_up(P, 1, 64);
        const uint32_t off = uint32_t(lane) == L0 ? d0 : (uint32_t(lane) > L0 ? (Pp >> (4u * d0)) & 15u : 8u);
        const uint64_t lost = __ballot(uint32_t(lane) > L0 && off == 8u);
        const uint32_t j = lost ? uint32_t(__ffsll((unsigned long long)lost) - 1) : 64u;
        if (uint32_t(lane) >= L0 && uint32_t(lane) < j) ent = rs + off;
        e = __builtin_amdgcn_readlane(ent, int(j - 1));   // the last lane the maps resolved
    }
    uint64_t X;
    bool sat = false;
    for (;;) {   // uniform (scalar) walk
        const uint32_t k = (e - W0) >> 7, d = e - W0 - (k << 7);
        uint32_t x;
        if (d < 8) {
            uint32_t r[8];
            #pragma unroll
            for (int q = 0; q < 8; q++) r[q] = __builtin_amdgcn_readlane(c[q], int(k));
            x = r[0];
            #pragma unroll
            for (int q = 1; q < 8; q++) x = d == uint32_t(q) ? r[q] : x;
        } else {
            x = __builtin_amdgcn_readfirstlane(uint32_t(xs[d * 64 + k]));
        }
        ent = uint32_t(lane) == k ? e : ent;
        if (x == XS_SAT) { sat = true; X = 0; break; }
        const uint64_t ex = uint64_t(W0) + (k << 7) + x;
        if (ex >= n || ex >= uint64_t(W0) + SNAP_WIN) { X = ex; break; }
        e = uint32_t(ex);
    }
    PT(23);
    L.b0 = L.b1 = L.b2 = L.b3 = 0;
    L.out = 0;
    if (sat) {   // exact whole-wave parse on a linear stage
        __syncthreads();
        const uint32_t woff = snap_stage(reinterpret_cast<uint8_t*>(xs), in, n, W0, SNAP_WSTAGE, lane);
        reinterpret_cast<uint4*>(sbits)[lane] = make_uint4(0, 0, 0, 0);
        slo[lane] = 0;
        __syncthreads();
        uint32_t sum;
        const uint64_t wend = min(uint64_t(W0) + SNAP_WIN, n);
        const uint32_t Xs = seq_parse(reinterpret_cast<const uint8_t*>(xs), woff, W0, n, entry, wend, sbits, slo, sum);
        __syncthreads();
        const uint4 v = reinterpret_cast<const uint4*>(sbits)[lane];
        L.b0 = v.x; L.b1 = v.y; L.b2 = v.z; L.b3 = v.w;
        L.out = slo[lane];
        return Xs;
    }
    if (X > n) return SNAP_INVALID;
    // (4)
    if (ent != SNAP_INVALID) {
        const uint32_t re = uint32_t(min<uint64_t>(uint64_t(rs) + SNAP_RB, n));
        uint32_t p = ent;
        while (p < re) {
            const uint32_t o = p - rs;
            const uint32_t tag = (*reinterpret_cast<const uint32_t*>(mine + (o & ~3u)) >> (8u * (o & 3u))) & 0xffu;
            uint32_t tl = tag_tl(tag), ol = tag_ol(tag);
            if (tag_long(tag)) {   // < 2^15 past the region (the exits are not saturated)
                const SnapTok t = snap_tok(lds_read8(mine, o));
                tl = uint32_t(t.tl);
                ol = t.ol;
            }
            bit_set(L, o);
            const uint32_t s2 = L.out + ol;
            L.out = s2 < L.out ? 0xffffffffu : s2;
            p += tl;
        }
    }
    PT(24);
    return uint32_t(X);
#undef PT
}

__device__ __forceinline__ void store_window(uint32_t* tm, uint32_t* lo, const WinLane& L, int lane) {
    reinterpret_cast<uint4*>(tm)[lane] = make_uint4(L.b0, L.b1, L.b2, L.b3);
    lo[lane] = L.out;
}

__global__ __launch_bounds__(64) void k_snappy_index(const SnappyJob* __restrict__ jobs, const int2* __restrict__ wins,
                                                     SnapWin* __restrict__ win, SnapEnt* __restrict__ ent,
                                                     uint32_t* __restrict__ lane_out, int* __restrict__ fb) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SNAP_WSTAGE];
    __shared__ __attribute__((aligned(16))) uint32_t sbits[SNAP_WWORDS];
    __shared__ uint32_t slo[64];
    const int2 jw = wins[blockIdx.x];
    if (fb[jw.x] >= FB_INPLACE) return;   // one literal: in place, or copied by k_snappy_litcopy
    const SnappyJob job = jobs[jw.x];
    const int lane = threadIdx.x;
    const uint64_t n = job.src_len;
    const uint32_t W0 = uint32_t(jw.y) * SNAP_WIN;
    const uint32_t wi = job.win_base + uint32_t(jw.y);
    uint32_t* tm = job.tokmap + size_t(jw.y) * SNAP_WWORDS;
    uint32_t* lo = lane_out + size_t(wi) * 64;
    uint32_t entry = W0;
    WinLane L{};
    if (jw.y == 0) {
        uint64_t pos = 0, ulen = 0;
        if (!uvarint(job.src, n, pos, ulen) || ulen != job.dst_len) {   // the serial kernel reports it
            store_window(tm, lo, L, lane);
            if (lane == 0) { win[wi] = SnapWin{0, SNAP_INVALID, 0, WIN_BROKEN}; fb[jw.x] = FB_SERIAL; }
            return;
        }
        entry = uint32_t(pos);
    }
    if (entry >= n) {   // empty body
        store_window(tm, lo, L, lane);
        if (lane == 0) win[wi] = SnapWin{entry, entry, 0, 0};
        return;
    }
    const uint64_t wend = min(uint64_t(W0) + SNAP_WIN, n);
#ifdef PF_STAMPS
    unsigned long long it0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t woff = snap_stage(stage, job.src, n, W0, SNAP_WSTAGE, lane);
    __syncthreads();
    uint32_t flags;
    uint32_t X = win_parse_spec(stage, woff, W0, n, entry, L, flags, sbits);
#ifdef PF_STAMPS
    { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (lane == 0) { CSTAMP(0, 1); CSTAMP(1, t_ - it0); if (flags & WIN_NOCONV) CSTAMP(2, 1); } it0 = t_; }
#endif
    uint32_t sum;
    if (flags & WIN_NOCONV) {   // chains that do not synchronise: exact whole-wave parse instead
        reinterpret_cast<uint4*>(sbits)[lane] = make_uint4(0, 0, 0, 0);
        slo[lane] = 0;
        __syncthreads();
        X = seq_parse(stage, woff, W0, n, entry, wend, sbits, slo, sum);
        flags = X == SNAP_INVALID ? WIN_BROKEN : 0u;
        __syncthreads();
        const uint4 v = reinterpret_cast<const uint4*>(sbits)[lane];
        L.b0 = v.x; L.b1 = v.y; L.b2 = v.z; L.b3 = v.w;
        L.out = slo[lane];
    } else {
        sum = wave_sum_sat(L.out);
    }
    store_window(tm, lo, L, lane);
    if (lane == 0) win[wi] = SnapWin{entry, X, sum, flags};
#ifdef PF_STAMPS
    { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (lane == 0) CSTAMP(3, t_ - it0); it0 = t_; }
#endif
    if (jw.y == 0) return;   // window 0's entry is exact: no table
    // entry table: lane d follows the chain from W0 + d until it meets this window's chain
    __syncthreads();
    reinterpret_cast<uint4*>(sbits)[lane] = make_uint4(L.b0, L.b1, L.b2, L.b3);
    {   // exclusive prefix of the lane-region outputs (wrapping: only differences are used)
        uint32_t x = L.out;
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t y = __shfl_up(x, dd, 64);
            if (lane >= dd) x += y;
        }
        slo[lane] = x - L.out;
    }
    __syncthreads();
    SnapEnt T = mk_ent(0, ENT_SLOW, 0);
    if (!(flags & WIN_BROKEN) && uint64_t(W0) + lane < wend)
        T = ent_walk(W0 + uint32_t(lane), W0, wend, n, stage, woff, sbits, slo);
    ent[size_t(wi) * 64 + lane] = T;
#ifdef PF_STAMPS
    {
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();
        if (lane == 0) CSTAMP(4, t_ - it0);
        const unsigned long long sl = __ballot((T.pos >> 30) == ENT_SLOW);
        if (lane == 0 && sl) CSTAMP(5, 1);
        if (lane == 0) CSTAMP(6, __popcll(sl));
    }
#endif
}

#ifdef PF_SNAP_TRACE
__device__ uint32_t pf_trace[8192];
__device__ uint32_t pf_trace_n;
#define TRACE(...)                                                                             \
    do {                                                                                       \
        if (tr && lane == 0) {                                                                 \
            const uint32_t v_[] = {__VA_ARGS__};                                               \
            const uint32_t at_ = atomicAdd(&pf_trace_n, uint32_t(sizeof v_ / 4));              \
            for (uint32_t q_ = 0; q_ < sizeof v_ / 4 && at_ + q_ < 8192; q_++) pf_trace[at_ + q_] = v_[q_]; \
        }                                                                                      \
    } while (0)
extern "C" int pf_debug_trace(uint32_t* out, int n, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_trace), 4 * size_t(n < 8192 ? n : 8192)) != hipSuccess) return -1;
    if (reset) {
        uint32_t z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(pf_trace_n), &z, 4) != hipSuccess) return -1;
    }
    return 0;
}
#define TRACEF(...)                                                                            \
    do {                                                                                       \
        const uint32_t v_[] = {__VA_ARGS__};                                                   \
        const uint32_t at_ = atomicAdd(&pf_trace_n, uint32_t(sizeof v_ / 4));                  \
        for (uint32_t q_ = 0; q_ < sizeof v_ / 4 && at_ + q_ < 8192; q_++) pf_trace[at_ + q_] = v_[q_]; \
    } while (0)
#else
#define TRACE(...) ((void)0)
#define TRACEF(...) ((void)0)
#endif

// ======================================================================== chain pass

constexpr int FIX_MAXW = 1024;       // pages up to 8 MiB compressed (larger: serial fallback)

__device__ __forceinline__ bool tm_get(const uint32_t* tm, uint32_t i) { return (tm[i >> 5] >> (i & 31u)) & 1u; }

constexpr int DEEP_STEPS = 24;       // HBM token walks of the chain pass; longer: exact parse of the window

// Entry deeper than 64 bytes into window w (after a long literal): follow the chain from e in HBM
// until it meets the window's own chain (bitmap) or leaves the window. The window chain's output in
// [W0, m) is the lane-region counts before m's region plus the tokens of m's region below m.
__device__ SnapEnt deep_walk(const SnappyJob& job, uint32_t w, uint32_t e, uint64_t wend, const uint32_t* LOw) {
    const uint64_t n = job.src_len;
    const uint32_t W0 = w * SNAP_WIN;
    const uint32_t* tm = job.tokmap + size_t(w) * SNAP_WWORDS;
    uint64_t q = e;
    uint32_t acc = 0;
    int steps = 0;
    for (;;) {
        if (q >= wend) return mk_ent(uint32_t(q), ENT_NOMERGE, acc);
        if (tm_get(tm, uint32_t(q) - W0)) break;
        if (steps == DEEP_STEPS) return mk_ent(e, ENT_SLOW, 0);
        const SnapTok t = snap_tok(glb_read8(job.src, n, q));
        acc += t.ol;
        q += t.tl;
        steps++;
        if (q > n) return mk_ent(e, ENT_BAD, 0);
    }
    const uint32_t rel = uint32_t(q) - W0, rq = rel / SNAP_RB;
    uint32_t g = 0;
    for (uint32_t r = 0; r < rq; r++) g += LOw[r];
    for (uint32_t b = rq * SNAP_RB; b < rel; b += 32) {
        const uint32_t hi = rel - b >= 32 ? 0xffffffffu : ((1u << (rel - b)) - 1u);
        uint32_t mm = tm[b >> 5] & hi;
        while (mm) {
            const uint32_t i = b + uint32_t(__ffs(mm) - 1);
            mm &= mm - 1;
            g += snap_tok(glb_read8(job.src, n, W0 + i)).ol;
        }
    }
    return mk_ent(uint32_t(q), ENT_MERGE, acc - g);
}

// One wave per page, lanes over windows. Window 0's entry is exact (after the varint); window w's
// true entry is window w-1's true exit. Every window's exit as a function of its entry is known
// from the index pass for entries that merge with the window's own chain (exit = the window's own
// exit) or that leave it first (the entry table); so all windows are evaluated at once from a
// guessed entry (the previous window's own exit) and re-evaluated where the previous exit
// changed, until the entries are consistent: the fixed point of e_w = exit_{w-1}(e_{w-1}) with
// e_1 exact is unique, so a consistent assignment is the true chain. Usually two rounds, each one
// table load per window. A window the table cannot resolve (entry not within ENT_STEPS tokens of
// the chain) stops the propagation; the first such window is parsed exactly by the whole wave
// once its entry is final, and the rounds continue behind it. The result replaces each window's
// SnapWin: {true entry, merge point / exit, true output bytes, WM_* mode}.
// LDS: the DP stage of the exact window parse (25 KiB) plus five per-window words sized by the host
// to the batch's largest page (dynamic LDS, cap windows; round 3 sized them for FIX_MAXW = 20 KiB).
// (r04: a whole-wave sequential exact parse instead of win_parse needs 9.5 KiB in all, but took the
// isolated chain launch 93 -> 433 us on SF1: dense windows are parsed exactly often.)
__global__ __launch_bounds__(64) void k_snappy_chain(const SnappyJob* __restrict__ jobs, SnapWin* __restrict__ win,
                                                     const SnapEnt* __restrict__ ent, uint32_t* __restrict__ lane_out,
                                                     int* __restrict__ fb, uint32_t cap) {
    __shared__ __attribute__((aligned(16))) uint8_t sp[SNAP_PSTAGE];
    __shared__ __attribute__((aligned(16))) uint16_t xs[SNAP_RB * 64];
    __shared__ __attribute__((aligned(16))) uint32_t sbits[SNAP_WWORDS];
    __shared__ uint32_t slo[64];
    extern __shared__ uint32_t dyn_chain[];
    uint32_t* const s_e = dyn_chain;              // current entry of window w
    uint32_t* const s_x = dyn_chain + cap;        // exit given that entry (unresolved: the window's own exit)
    uint32_t* const s_pos = dyn_chain + 2 * cap;  // merge point / exit (SnapWin.exit)
    uint32_t* const s_out = dyn_chain + 3 * cap;  // true output bytes
    uint32_t* const s_mode = dyn_chain + 4 * cap; // 0 entry changed, 1 unresolved, else WM_* (WM_DONE: final)
    const int j = blockIdx.x;
    const int lane = threadIdx.x;
    const SnappyJob job = jobs[j];
    if (fb[j] >= FB_SERIAL) return;
    const uint32_t nw = job.n_win;
    const uint64_t n = job.src_len;
    SnapWin* Wn = win + job.win_base;
    const SnapEnt* E = ent + size_t(job.win_base) * 64;
    uint32_t* LO = lane_out + size_t(job.win_base) * 64;
    if (nw > cap || nw > uint32_t(FIX_MAXW) || (Wn[0].flags & WIN_BROKEN)) {
        if (lane == 0) fb[j] = FB_SERIAL;
        return;
    }
    const SnapWin w0 = Wn[0];
    if (lane == 0) {
        Wn[0] = SnapWin{w0.entry, w0.exit, w0.out, WM_KEEP};
        s_x[0] = w0.exit;
        s_mode[0] = WM_KEEP;
    }
    for (uint32_t w = 1 + lane; w < nw; w += 64) {   // first guess: the previous window's own exit
        s_e[w] = w == 1 ? w0.exit : Wn[w - 1].exit;
        s_mode[w] = 0;
    }
    __syncthreads();
#ifdef PF_STAMPS
    const unsigned long long cstart = __builtin_amdgcn_s_memtime();
    if (lane == 0) { CSTAMP(17, 1); CSTAMP(18, nw); }
#endif
    bool bad = false;
    uint32_t base = 1;       // windows before base are final
    bool dirty_all = true;   // first round: evaluate every window
    while (base < nw) {
        // fixed-point rounds over [base, nw): re-evaluate windows whose entry changed (mode 0).
        // An unresolved window (mode 1) passes its own exit on as the guess for the next entry.
        for (;;) {
            for (uint32_t w = base + lane; w < nw; w += 64) {
                if (s_mode[w] == WM_DONE || (!dirty_all && s_mode[w] != 0)) continue;
                const uint32_t e = s_e[w];
                const uint32_t W0 = w * SNAP_WIN;
                const uint64_t wend = min(uint64_t(W0) + SNAP_WIN, n);
                uint32_t x, pos = 0, out = 0, mode;
                if (uint64_t(e) >= wend) {   // inside a literal that started earlier: no token here
                    x = e; pos = e; mode = WM_SKIP;
                } else {
                    const SnapWin sw = Wn[w];
                    SnapEnt T = mk_ent(e, ENT_SLOW, 0);
                    const uint32_t d = e - W0;
                    if (!(sw.flags & WIN_BROKEN)) {
#ifdef PF_STAMPS
                        const unsigned long long dt0 = __builtin_amdgcn_s_memtime();
#endif
                        T = d < 64 ? E[size_t(w) * 64 + d] : deep_walk(job, w, e, wend, LO + size_t(w) * 64);
#ifdef PF_STAMPS
                        if (d >= 64) { CSTAMP(11, 1); CSTAMP(12, __builtin_amdgcn_s_memtime() - dt0); }
#endif
                    }
                    const uint32_t fl = T.pos >> 30, tp = T.pos & ENT_POS;
                    x = sw.exit; mode = 1u;
                    if (fl == ENT_MERGE) { pos = tp; out = sw.out + T.out; mode = WM_MERGE; }
                    else if (fl == ENT_NOMERGE) { x = tp; pos = tp; out = T.out; mode = WM_FULL; }
                }
                s_x[w] = x; s_pos[w] = pos; s_out[w] = out; s_mode[w] = mode;
            }
            dirty_all = false;
            if (lane == 0) CSTAMP(13, 1);
            __syncthreads();
            bool changed = false;
            for (uint32_t w = base + lane; w < nw; w += 64) {   // window base - 1 is final
                const uint32_t ne = s_x[w - 1];
                if (ne != s_e[w]) { s_e[w] = ne; s_mode[w] = 0; changed = true; }
            }
            __syncthreads();
            if (!__any(changed)) break;
        }
        // the first unresolved window: its entry is final now, parse it exactly
        uint32_t u = nw;
        for (uint32_t w = base + lane; w < nw; w += 64)
            if (s_mode[w] == 1u) { u = w; break; }
        #pragma unroll
        for (int dd = 32; dd >= 1; dd >>= 1) u = min(u, uint32_t(__shfl_xor(u, dd, 64)));
        if (u >= nw) break;
#ifdef PF_STAMPS
        const unsigned long long xt0 = __builtin_amdgcn_s_memtime();
#endif
        const uint32_t e = s_e[u];
        const uint32_t W0 = u * SNAP_WIN;
        stage_pad(sp, job.src, n, W0, lane);
        __syncthreads();
        WinLane WL{};
        const uint32_t X = win_parse(job.src, n, W0, e, sp, xs, sbits, slo, WL);
        if (X == SNAP_INVALID) { bad = true; break; }
        const uint32_t sum = wave_sum_sat(WL.out);
        store_window(job.tokmap + size_t(u) * SNAP_WWORDS, LO + size_t(u) * 64, WL, lane);
        __syncthreads();
        if (lane == 0) {
            s_x[u] = X; s_pos[u] = X; s_out[u] = sum; s_mode[u] = WM_DONE;
        }
        __syncthreads();
        base = u + 1;
#ifdef PF_STAMPS
        if (lane == 0) { CSTAMP(14, 1); CSTAMP(16, __builtin_amdgcn_s_memtime() - xt0); }
#endif
    }
    if (!bad) {
        bad = uint64_t(s_x[nw - 1]) != n;
        for (uint32_t w = 1 + lane; w < nw && !bad; w += 64) Wn[w] = SnapWin{s_e[w], s_pos[w], s_out[w], s_mode[w]};
    }
    if (bad && lane == 0) fb[j] = FB_SERIAL;
#ifdef PF_STAMPS
    if (lane == 0) { const unsigned long long dt_ = __builtin_amdgcn_s_memtime() - cstart; CSTAMP(19, dt_); atomicMax(&pf_cstamps[20], dt_); }
#endif
}

// One wave per window: make the bitmap and lane output counts of windows whose true entry is not
// their own chain's start exact — tokens in [W0, merge point) for WM_MERGE, the whole window for
// WM_FULL — by parsing from the true entry on the staged window; clear the bitmap of windows the
// chain jumps over (WM_SKIP).
__device__ void repair_window(const SnappyJob* __restrict__ jobs, const int2 jw, const SnapWin* __restrict__ win,
                              uint32_t* __restrict__ lane_out, int* __restrict__ fb, uint8_t* stage, uint32_t* sbits,
                              uint32_t* slo) {
    const SnappyJob job = jobs[jw.x];
    const int lane = threadIdx.x;
    if (fb[jw.x] >= FB_SERIAL) return;
    const uint32_t w = uint32_t(jw.y);
    const SnapWin sw = win[job.win_base + w];
    const uint32_t W0 = w * SNAP_WIN;
    if (sw.flags == WM_SKIP) {   // inside a literal: no token starts here (the index pass's guesses are cleared,
                                 // so the bitmap is exact over the whole stream)
        reinterpret_cast<uint4*>(job.tokmap + size_t(w) * SNAP_WWORDS)[lane] = make_uint4(0, 0, 0, 0);
        return;
    }
    if (!((sw.flags == WM_MERGE && sw.entry != W0) || sw.flags == WM_FULL)) return;
    const uint64_t n = job.src_len;
    const uint64_t wend = min(uint64_t(W0) + SNAP_WIN, n);
    const uint64_t stop = sw.flags == WM_FULL ? wend : uint64_t(sw.exit);
    // WM_MERGE reads the window only up to its merge point's lane region (+ a token's bytes and the
    // parse's 64-position lookahead): usually the first 256 bytes, not the whole 8 KiB (round 5)
    const uint32_t need = sw.flags == WM_FULL ? SNAP_WSTAGE
                                              : min(SNAP_WSTAGE, ((sw.exit - W0) / SNAP_RB + 1) * SNAP_RB + 128u);
    const uint32_t woff = snap_stage(stage, job.src, n, W0, need, lane);
    reinterpret_cast<uint4*>(sbits)[lane] = make_uint4(0, 0, 0, 0);
    slo[lane] = 0;
    __syncthreads();
    uint32_t sum;
    const uint32_t X = seq_parse(stage, woff, W0, n, sw.entry, stop, sbits, slo, sum);
    __syncthreads();
    uint32_t* tm = job.tokmap + size_t(w) * SNAP_WWORDS;
    uint32_t* lo = lane_out + size_t(job.win_base + w) * 64;
    if (sw.flags == WM_FULL) {
        if (X == SNAP_INVALID || uint64_t(X) < wend) { if (lane == 0) atomicMax(&fb[jw.x], FB_SERIAL); return; }
        reinterpret_cast<uint4*>(tm)[lane] = reinterpret_cast<const uint4*>(sbits)[lane];
        lo[lane] = slo[lane];
        return;
    }
    if (X != sw.exit) { if (lane == 0) atomicMax(&fb[jw.x], FB_SERIAL); return; }
    // WM_MERGE: bits below the merge point m come from the parse, bits from m on stay
    const uint32_t rel = sw.exit - W0, rm = rel / SNAP_RB;
    if (uint32_t(lane) > rm) return;
    uint32_t nb[4];
    #pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t wi = uint32_t(lane) * 4 + k, b0 = wi * 32;
        const uint32_t low = b0 + 32 <= rel ? 0xffffffffu : (b0 >= rel ? 0u : (1u << (rel - b0)) - 1u);
        nb[k] = low == 0xffffffffu ? sbits[wi] : ((sbits[wi] & low) | (tm[wi] & ~low));
        tm[wi] = nb[k];
    }
    if (uint32_t(lane) < rm) { lo[lane] = slo[lane]; return; }
    // the merge point's region: parsed tokens below m plus the window's own tokens from m on
    uint32_t acc = slo[lane];
    #pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t b0 = (uint32_t(lane) * 4 + k) * 32;
        uint32_t mm = nb[k] & ~(b0 + 32 <= rel ? 0xffffffffu : (b0 >= rel ? 0u : (1u << (rel - b0)) - 1u));
        while (mm) {
            const uint32_t i = b0 + uint32_t(__ffs(mm) - 1);
            mm &= mm - 1;
            acc += snap_tok(lds_read8(stage, woff + i)).ol;
        }
    }
    lo[lane] = acc;
}

// Grid-stride over the windows (PF_REPAIR_GRID bounds the grid; by default one block per window):
// only windows the chain pass could not resolve (WM_MERGE / WM_FULL) and windows inside a literal
// (WM_SKIP: bitmap cleared) do work.
__global__ __launch_bounds__(64) void k_snappy_repair(const SnappyJob* __restrict__ jobs, const int2* __restrict__ wins,
                                                      int n_wins, const SnapWin* __restrict__ win,
                                                      uint32_t* __restrict__ lane_out, int* __restrict__ fb) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SNAP_WSTAGE];
    __shared__ __attribute__((aligned(16))) uint32_t sbits[SNAP_WWORDS];
    __shared__ uint32_t slo[64];
    for (int b = blockIdx.x; b < n_wins; b += gridDim.x) {
        repair_window(jobs, wins[b], win, lane_out, fb, stage, sbits, slo);
        __syncthreads();
    }
}

// One workgroup per page: wave 0 checks the output total (window prefix sums into LDS); then each
// wave takes pieces in turn and finds the input position of the token that starts at the piece's
// 64 KiB output boundary with all of its loads issued together: the window's 64 lane-region output
// counts (one per lane; a ballot picks the region), then the region's 128 bytes (+ 8 for the last
// token's length bytes) and its 4 token-start bitmap words, then one token per lane position and a
// wave scan of their output lengths. (Round 3 walked the region counts and the tokens one dependent
// load at a time per piece: ~50 us per launch.)
constexpr int SP_NT = 256;
__global__ __launch_bounds__(SP_NT) void k_snappy_splits(const SnappyJob* __restrict__ jobs, const SnapWin* __restrict__ win,
                                                         const uint32_t* __restrict__ lane_out, uint32_t* __restrict__ splits,
                                                         int* __restrict__ fb) {
    __shared__ uint32_t s_pre[FIX_MAXW + 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_reg[SP_NT / 64][SNAP_RB + 16];
    __shared__ uint32_t s_tm[SP_NT / 64][4];
    __shared__ int s_ok;
    const int j = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const SnappyJob job = jobs[j];
    if (fb[j] >= FB_SERIAL) return;   // (block-uniform)
    const uint32_t nw = job.n_win;
    const uint64_t n = job.src_len;
    const SnapWin* Wn = win + job.win_base;
    const uint32_t* LO = lane_out + size_t(job.win_base) * 64;
    if (wv == 0) {
        uint32_t run = 0;
        bool ovf = false;
        for (uint32_t w0i = 0; w0i < nw; w0i += 64) {
            const uint32_t w = w0i + lane;
            const uint32_t o = w < nw ? Wn[w].out : 0u;
            uint64_t x = o;
            #pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint64_t y = __shfl_up(x, dd, 64);
                if (lane >= dd) x += y;
            }
            if (w < nw) s_pre[w] = uint32_t(run + x - o);
            const uint64_t t = uint64_t(run) + __shfl(x, 63, 64);
            ovf |= t > 0xffffffffull;
            run = uint32_t(t);
        }
        const bool ok = !ovf && run == job.dst_len;
        if (lane == 0) { s_ok = ok; if (!ok) fb[j] = FB_SERIAL; }
    }
    __syncthreads();
    if (!s_ok) return;
    uint32_t* sp = splits + job.split_base;
    uint8_t* R = s_reg[wv];
    const PF_GLOBAL uint8_t* src = gptr(job.src);
    for (uint32_t k = 1 + uint32_t(wv); k < job.n_pieces; k += SP_NT / 64) {
        const uint32_t B = k * SNAP_BLOCK;
        uint32_t a = 0, b = nw;   // last window with s_pre <= B
        while (b - a > 1) {
            const uint32_t m = (a + b) / 2;
            if (s_pre[m] <= B) a = m; else b = m;
        }
        const uint32_t w = a;
        // the lane region holding output byte B: the first of regions 0..62 whose end passes B (else 63)
        const uint32_t v = LO[size_t(w) * 64 + lane];
        uint64_t x = v;
        #pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint64_t y = __shfl_up(x, dd, 64);
            if (lane >= dd) x += y;
        }
        const uint64_t base = s_pre[w];
        const uint64_t past = __ballot(lane < 63 && uint64_t(B) < base + x);
        const int l = past ? __ffsll((unsigned long long)past) - 1 : 63;
        const uint64_t cum0 = base + __shfl(x - v, l, 64);   // output before region l
        // the region's bytes (zero past the stream) and its token-start bitmap
        const uint32_t rs = w * SNAP_WIN + uint32_t(l) * SNAP_RB;
        const uint64_t q0 = uint64_t(rs) + uint32_t(lane), q1 = q0 + 64, q2 = q0 + 128;
        const uint8_t c0 = q0 < n ? src[q0] : uint8_t(0), c1 = q1 < n ? src[q1] : uint8_t(0);
        const uint8_t c2 = (lane < 16 && q2 < n) ? src[q2] : uint8_t(0);
        const uint32_t tw = lane < 4 ? job.tokmap[size_t(w) * SNAP_WWORDS + uint32_t(l) * 4 + uint32_t(lane)] : 0u;
        R[lane] = c0; R[64 + lane] = c1;
        if (lane < 16) R[128 + lane] = c2;
        if (lane < 4) s_tm[wv][lane] = tw;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // one position per lane and half: output length of the token starting there (0: none)
        uint32_t ol[2];
        bool st[2];
        for (int h = 0; h < 2; h++) {
            const uint32_t i = uint32_t(h) * 64 + uint32_t(lane);
            st[h] = (s_tm[wv][i >> 5] >> (i & 31)) & 1u;
            uint64_t t8 = 0;
            #pragma unroll
            for (int u = 0; u < 8; u++) t8 |= uint64_t(R[i + u]) << (8 * u);
            ol[h] = st[h] ? snap_tok(t8).ol : 0u;
        }
        // the first token whose preceding output reaches B: found when it equals B
        uint32_t found = SNAP_INVALID;
        uint64_t cum = cum0;
        for (int h = 0; h < 2; h++) {
            uint64_t y = ol[h];
            #pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint64_t z = __shfl_up(y, dd, 64);
                if (lane >= dd) y += z;
            }
            const uint64_t before = cum + y - ol[h];
            const uint64_t hit = __ballot(st[h] && before >= uint64_t(B));
            if (hit) {
                const int f = __ffsll((unsigned long long)hit) - 1;
                if (__shfl(before, f, 64) == uint64_t(B)) found = rs + uint32_t(h) * 64 + uint32_t(f);
                break;
            }
            cum += __shfl(y, 63, 64);
        }
        if (lane == 0) sp[k] = found;
        __builtin_amdgcn_wave_barrier();   // (the region buffer is rewritten by the next piece)
    }
}

// ======================================================================== executor


#ifndef PF_XRING
#define PF_XRING 4096
#endif
constexpr uint32_t XRING = PF_XRING; // output ring (LDS); copies reaching further back read HBM (far copies)
constexpr uint32_t XRMASK = XRING - 1;
constexpr uint32_t XSLOT = 1024;     // flush granule
constexpr uint32_t XCHUNK = 1024;    // input bytes whose tokens are enumerated at once
constexpr uint32_t XSTAGE = XCHUNK + 64 + 16;
#ifndef PF_XBATCH
#define PF_XBATCH 1024
#endif
[[maybe_unused]] constexpr uint32_t XBATCH = PF_XBATCH;   // output bytes of one parallel step (ring: XBATCH + XSLOT <= XRING)
constexpr uint32_t XLIT = 1024;      // long literals are copied in pieces of this many bytes
constexpr uint32_t FBUF_W = 17;      // dwords per far copy's source slot (64 bytes + misalignment)
#ifndef PF_XFAR
#define PF_XFAR 24
#endif
constexpr uint32_t XFAR = PF_XFAR;   // far copies per step (the step is cut before the next one)

__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// x mod d for 0 <= x < 64, 1 <= d <= 64 ((x + 0.5) / d is never within 1/128 of an integer).
__device__ __forceinline__ uint32_t mod_small(uint32_t x, uint32_t d) {
    const uint32_t q = uint32_t((float(x) + 0.5f) * __builtin_amdgcn_rcpf(float(d)));
    return x - q * d;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    #pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, uint32_t(__shfl_xor(v, d, 64)));
    return v;
}

// Number of lanes whose key is < x; keys ascend over the lanes (all 64 lanes must call).
__device__ __forceinline__ uint32_t lanes_below(uint32_t key, uint32_t x) {
    uint32_t idx = 0;
    #pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint32_t kv = __shfl(key, int(idx) + s - 1, 64);
        if (kv < x) idx += uint32_t(s);
    }
    const uint32_t k63 = __shfl(key, 63, 64);
    return (idx == 63 && k63 < x) ? 64u : idx;
}

__device__ __forceinline__ uint64_t lane_mask_lt(uint32_t k) { return k >= 64 ? ~0ull : ((1ull << k) - 1ull); }

// Store ring bytes [F, upto) in whole XSLOT slots (16-byte stores, XSLOT / 64 bytes per lane).
// Returns the number of store instructions issued.
constexpr uint32_t XST = XSLOT / 64 / 16;   // 16-byte stores per lane per slot

// Where a job's output goes: dst + a, or for a direct job (k_snappy_head) ddst + a from output
// offset dlo on (the column's values; dgran-wide stores, ddst's alignment).
struct OutDst {
    PF_GLOBAL uint8_t* dst;
    PF_GLOBAL uint8_t* dd;   // null: not direct
    uint32_t dlo, gran;
};

// Rare: a 16-byte chunk holding the end of the level section (kept out of put16's registers).
__device__ __attribute__((noinline)) void put16_split(PF_GLOBAL uint8_t* dst, PF_GLOBAL uint8_t* dd, uint32_t dlo, uint32_t a,
                                                     u32x4 v) {
    for (uint32_t k = 0; k < 16; k++) {
        const uint8_t b = uint8_t(v[k >> 2] >> (8 * (k & 3)));
        (a + k < dlo ? dst : dd)[a + k] = b;
    }
}

// 16 output bytes at the 16-aligned output offset a.
__device__ __forceinline__ void put16(const OutDst& o, uint32_t a, u32x4 v) {
    if (o.dd == nullptr || a + 16u <= o.dlo) {
        *(PF_GLOBAL u32x4*)(o.dst + a) = v;
    } else if (a >= o.dlo) {
        PF_GLOBAL uint8_t* p = o.dd + a;
        if (o.gran == 16u) {
            *(PF_GLOBAL u32x4*)p = v;
        } else if (o.gran == 8u) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            reinterpret_cast<PF_GLOBAL u32x2*>(p)[0] = u32x2{v.x, v.y};
            reinterpret_cast<PF_GLOBAL u32x2*>(p)[1] = u32x2{v.z, v.w};
        } else {
            PF_GLOBAL uint32_t* q = reinterpret_cast<PF_GLOBAL uint32_t*>(p);
            q[0] = v.x; q[1] = v.y; q[2] = v.z; q[3] = v.w;
        }
    } else {   // straddles dlo (the end of the level section)
        put16_split(o.dst, o.dd, o.dlo, a, v);
    }
}
__device__ __forceinline__ void put1(const OutDst& o, uint32_t a, uint8_t b) {
    (o.dd == nullptr || a < o.dlo ? o.dst : o.dd)[a] = b;
}

__device__ __forceinline__ uint32_t flush_slots(const uint8_t* ring, const OutDst& o, uint32_t& F, uint32_t upto, int lane) {
    uint32_t nsl = 0;
    while (upto - F >= XSLOT) {
        const uint32_t a0 = F + uint32_t(lane) * (XSLOT / 64);
        #pragma unroll
        for (uint32_t u = 0; u < XST; u++)
            put16(o, a0 + 16 * u, *reinterpret_cast<const u32x4*>(ring + ((a0 + 16 * u) & XRMASK)));
        F += XSLOT;
        nsl += XST;
    }
    return nsl;
}

// ---- wave64 DPP helpers (VALU-speed; __shfl goes through LDS) ----
__device__ __forceinline__ uint32_t dpp_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}
__device__ __forceinline__ uint32_t dpp_prev(uint32_t v) {               // lane i <- lane i-1
    return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

__device__ __forceinline__ void wait_vmem_last_slot() {   // all but the last flush slot's XST stores
    if constexpr (XST == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
}

// ======================================================================== executor v2
//
// Same token supply, chain checks, step cuts and far-copy prefetch as k_snappy_exec, but every
// output byte of a step is produced by one byte-lane pass: the step's output is walked in
// sub-steps of 64 bytes, lane x owning byte x0 + x. Its token comes from the step's token-start
// bitmap (word prefix counts + popcount), the token's packed descriptor from the token's lane
// (ds_bpermute, no LDS table), and its source is
//   a literal byte (staged input) or a far-copy byte (prefetched source slot): one LDS read;
//   a copy byte whose source precedes the sub-step: one ring read (earlier sub-steps of the same
//     step are already in the ring: single wave, LDS operations execute in order);
//   a copy byte whose source lies in the same sub-step (dependent copies, self-overlapping runs):
//     resolved across the 64 lanes by pointer jumping on a packed {value, pending, source lane}
//     word (ds_bpermute per round; a source lane always precedes its reader, so <= 6 rounds).
// Self-overlapping copies read source byte (j mod offset), so a run never chains through itself.
// Dependent copies therefore cost a few register rounds per 64 bytes instead of one serial
// read-then-write per token.
[[maybe_unused]] constexpr uint32_t X2_STAGE_OFF = XRING;                            // [ring | stage | far slots] in one LDS array,
constexpr uint32_t X2_FBUF_OFF = XRING + ((XSTAGE + 15u) & ~15u);   // so one byte address selects any source
[[maybe_unused]] constexpr uint32_t X2_LDS = X2_FBUF_OFF + XFAR * FBUF_W * 4;
enum : uint32_t { X2_LDSADDR = 0, X2_COPY = 1 };

#ifdef PF_DIAG   // diagnostics build only (VERDICT r05 hygiene)
__global__ __launch_bounds__(64) void k_snappy_exec2(const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                                     const uint32_t* __restrict__ splits, int* __restrict__ fb, int mode) {
    __shared__ __attribute__((aligned(16))) uint8_t L[X2_LDS];
    __shared__ uint16_t tokpos[XCHUNK / 2];
    __shared__ uint32_t sbits[XBATCH / 32];                               // token starts of the step's output
    __shared__ uint32_t wpre[XBATCH / 32];                                // tokens starting in earlier words
    __shared__ uint16_t jv[256];                                          // pointer-jumping words of a window
    uint8_t* const ring = L;
    uint8_t* const stage = L + X2_STAGE_OFF;
    uint32_t* const fbuf = reinterpret_cast<uint32_t*>(L + X2_FBUF_OFF);
    const int lane = threadIdx.x;
    int j, k;
    if (mode == 0) {
        const int2 pc = pieces[blockIdx.x];
        j = pc.x;
        k = pc.y;
    } else {
        j = blockIdx.x;
        k = 0;
    }
    const int f = fb[j];
    bool whole;
    if (mode == 0) {
        if (f >= FB_REDO || (f == FB_WHOLE && k > 0)) return;
        whole = f == FB_WHOLE;
    } else {
        if (f != FB_REDO) return;
        whole = true;
    }
    const SnappyJob job = jobs[j];
    const uint8_t* in = job.src;
    uint8_t* dst = job.dst;
    const uint64_t n = job.src_len;
    const uint32_t* sp = splits + job.split_base;
    uint64_t pos0 = 0, ulen = 0;
    if (!uvarint(in, n, pos0, ulen) || ulen != job.dst_len) {
        if (lane == 0) atomicMax(&fb[j], FB_SERIAL);
        return;
    }
    if (mode == 0 && (job.dflags & 1u)) {   // diagnostics: forced redo
        if (lane == 0) atomicMax(&fb[j], FB_REDO);
        return;
    }
    uint32_t ip, out_start, out_end = job.dst_len;
    if (whole) {
        ip = uint32_t(pos0);
        out_start = 0;
    } else {
        if (k > 0 && sp[k] == SNAP_INVALID) return;   // no token at this boundary: an earlier piece covers it
        ip = k == 0 ? uint32_t(pos0) : sp[k];
        out_start = uint32_t(k) * SNAP_BLOCK;
        for (uint32_t k2 = k + 1; k2 < job.n_pieces; k2++)
            if (sp[k2] != SNAP_INVALID) { out_end = k2 * SNAP_BLOCK; break; }
    }
    const PF_GLOBAL uint16_t* tm16 = (const PF_GLOBAL uint16_t*)(job.tokmap);
    const PF_GLOBAL uint8_t* gin = gptr(in);
    PF_GLOBAL uint8_t* gdst = gptr(dst);
    const OutDst od{gdst, mode == 0 ? gptr(job.ddst) : nullptr, job.dlo, job.dgran};
    uint32_t op = out_start, F = out_start;
    uint32_t nst = 0;   // store instructions issued by the last flush (still possibly in flight)
    bool bad = false;
    XT_DECL;
#ifdef PF_STAMPS
    const unsigned long long xt0 = xt_;
    if (lane == 0) STAMP_ADD(13, 1);
#endif
    while (op < out_end && !bad) {
        if (ip >= n) { bad = true; break; }
        const uint32_t I = ip & ~15u;
        __syncthreads();
        const uint32_t woff = snap_stage(stage, in, n, I, XSTAGE, lane);
        // token starts in [ip, I + XCHUNK): 16 input bytes per lane
        const uint32_t p16 = I + 16u * uint32_t(lane);
        uint32_t bits = uint64_t(p16) < n ? uint32_t(tm16[p16 >> 4]) : 0u;
        if (p16 + 16u <= ip) bits = 0;
        else if (p16 < ip) bits &= ~((1u << (ip - p16)) - 1u);
        const uint32_t cnt = __popc(bits);
        const uint32_t ex = dpp_incl_scan(cnt);
        const uint32_t T = __builtin_amdgcn_readlane(ex, 63);
        uint32_t q = ex - cnt;
        while (bits) {
            const uint32_t b = uint32_t(__ffs(bits) - 1);
            bits &= bits - 1;
            tokpos[q++] = uint16_t(16u * uint32_t(lane) + b);
        }
        nst = 0;   // the bitmap loads above waited for every earlier store
        __syncthreads();
        XT(7);
        if (T == 0) { bad = true; break; }
        uint32_t sb = 0;
        while (sb < T && op < out_end) {
            const uint32_t t = sb + uint32_t(lane);
            const bool v = t < T;
            const uint32_t pos = v ? uint32_t(tokpos[t]) : 0u;
            const SnapTok tk = snap_tok(lds_read8(stage, woff + pos));
            const uint32_t ol = v ? tk.ol : 0u;
            const uint32_t start = I + pos;
            const uint32_t endp = tk.tl > uint64_t(0xffffffffu - start) ? 0xffffffffu : start + uint32_t(tk.tl);
            const uint32_t prev = dpp_prev(endp);
            const uint32_t inc = dpp_incl_scan(ol);
            const uint32_t otok = op + inc - ol;
            const bool take = v && otok < out_end;
            const int nt = __popcll(__ballot(take));
            const bool wrong = take && ((lane == 0 ? start != ip : start != prev) || endp > n || op + inc > out_end ||
                                        inc < ol);
            if (__any(wrong)) { bad = true; break; }
            if (nt == 0) break;   // the previous step ended exactly at out_end
            const uint32_t kd = tk.kind;
            const uint32_t off = tk.arg;
            const uint32_t srcv = start + tk.arg;   // literal data position
            const bool lstaged = srcv + ol <= I + XCHUNK + 64;
            const uint32_t a = otok - off;                       // copy source start
            const bool farc = take && kd != 0 && a + min(ol, off) <= op && int32_t(a - (op + XBATCH - XRING)) < 0;
            const unsigned long long farm = __ballot(farc);
            const uint32_t frank = uint32_t(__popcll(farm & lane_mask_lt(uint32_t(lane))));
            const unsigned long long cutm = __ballot(take && (ol > 64u || inc > XBATCH || (kd == 0 && !lstaged) ||
                                                              (farc && frank >= XFAR)));
            const uint32_t cut = cutm ? uint32_t(__ffsll(cutm) - 1) : uint32_t(nt);
            uint32_t used, btot;
            XT(1);
            if (lane == 0) STAMP_ADD(0, 1);
            if (cut == 0) {
                // one literal, from HBM (copies are <= 64 bytes, so only a literal gets here)
                const uint32_t L0 = __builtin_amdgcn_readfirstlane(ol);
                const uint32_t s0 = __builtin_amdgcn_readfirstlane(srcv);
                if (__builtin_amdgcn_readfirstlane(kd) != 0) { bad = true; break; }
                uint32_t fl_slots = 0;
                for (uint32_t d0 = 0; d0 < L0; d0 += XLIT) {
                    const uint32_t c = min(L0 - d0, XLIT);
                    const uint32_t b0 = uint32_t(lane) * 16u;
                    if (b0 < c) {
                        uint8_t by[16];
                        #pragma unroll
                        for (int u = 0; u < 16; u++) by[u] = b0 + u < c ? gin[s0 + d0 + b0 + u] : uint8_t(0);
                        #pragma unroll
                        for (int u = 0; u < 16; u++)
                            if (b0 + u < c) ring[(op + d0 + b0 + u) & XRMASK] = by[u];
                    }
                    fl_slots += flush_slots(ring, od, F, op + d0 + c, lane);
                }
                nst = fl_slots;
                used = 1;
                btot = L0;
                XT(11);
            } else {
                used = cut;
                btot = __builtin_amdgcn_readlane(inc, cut - 1);
                const bool inb = take && uint32_t(lane) < cut;
                const bool lit = inb && kd == 0;
                const bool cp = inb && kd != 0;
                if (__any(cp && (off == 0 || off > otok - out_start))) { bad = true; break; }
                const bool far = cp && farc;
                // a far source straddling the direct split (level bytes | values) is not one window
                if (od.dd != nullptr && __any(far && a < od.dlo && a + ol > od.dlo)) { bad = true; break; }
                // far copies: their source (flushed output) into this token's LDS slot
                if (__any(far)) {
                    if (nst == XST) wait_vmem_last_slot();   // all but the last slot's stores have landed
                    else wait_vmem();
                    if (far) {
                        const PF_GLOBAL uint8_t* fb0 = od.dd != nullptr && a >= od.dlo ? od.dd + a : gdst + a;
                        const uintptr_t fa = reinterpret_cast<uintptr_t>(fb0);
                        const PF_GLOBAL uint32_t* fsrc = (const PF_GLOBAL uint32_t*)(fa & ~uintptr_t(3));
                        const uint32_t nwd = (uint32_t(fa & 3u) + ol + 3u) >> 2;
                        uint32_t fw[FBUF_W];
                        #pragma unroll
                        for (int u = 0; u < int(FBUF_W); u++) fw[u] = uint32_t(u) < nwd ? fsrc[u] : 0u;
                        uint32_t* fl = fbuf + frank * FBUF_W;
                        #pragma unroll
                        for (int u = 0; u < int(FBUF_W); u++)
                            if (uint32_t(u) < nwd) fl[u] = fw[u];
                    }
                }
                if (lane == 0 && __any(far)) STAMP_ADD(9, 1);
                XT(3);
                // packed token descriptor, read by the byte lanes with ds_bpermute:
                //   d0 = rel (11 bits) | kind (1 bit, 11) | self-overlap (bit 12) | offset << 16
                //   d1 = LDS byte address of the token's first source byte (literal / far copy) or the
                //        absolute output position of its source (near copy)
                const uint32_t rel = otok - op;
                uint32_t d0 = 0, d1 = 0;
                if (inb) {
                    const bool near = cp && !far;
                    d0 = rel | ((near ? X2_COPY : X2_LDSADDR) << 11) | ((near && off < ol) ? (1u << 12) : 0u) |
                         (min(off, 0xffffu) << 16);
                    const uint32_t fsh = od.dd != nullptr && a >= od.dlo
                                             ? uint32_t((reinterpret_cast<uintptr_t>(od.dd) + a) & 3u) : (a & 3u);
                    d1 = lit ? X2_STAGE_OFF + woff + (srcv - I)
                             : (far ? X2_FBUF_OFF + frank * (FBUF_W * 4) + fsh : a);
                }
                if (lane < int(XBATCH / 32)) sbits[lane] = 0;
                __syncthreads();
                if (inb) atomicOr(&sbits[rel >> 5], 1u << (rel & 31u));
                __syncthreads();
                {
                    const uint32_t c = lane < int(XBATCH / 32) ? __popc(sbits[lane]) : 0u;
                    const uint32_t e2 = dpp_incl_scan(c) - c;
                    if (lane < int(XBATCH / 32)) wpre[lane] = e2;
                }
                __syncthreads();
                XT(4);
                // 256-byte windows: lane L owns bytes w0 + 64u + L (u < 4). A byte's word is its value
                // (< 0x100) or 0x100 | p: "same as window byte p" (p < its own position).
                for (uint32_t w0 = 0; w0 < btot; w0 += 256) {
                    if (lane == 0) STAMP_ADD(8, 1);
                    const uint32_t s0 = op + w0;
                    // straight-line phases over the four slots (no branches: the compiler keeps the four
                    // chains of LDS operations in flight together)
                    uint32_t W[4], xw[4], ti[4], i0[4], i1[4], addr[4];
                    bool act[4], pend[4];
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t x = w0 + 64u * uint32_t(u) + uint32_t(lane);
                        act[u] = x < btot;
                        xw[u] = act[u] ? x : btot - 1u;
                    }
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t wd = xw[u] >> 5;
                        ti[u] = wpre[wd] + __popc(sbits[wd] & ((2u << (xw[u] & 31u)) - 1u)) - 1u;
                    }
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        i0[u] = uint32_t(__builtin_amdgcn_ds_bpermute(int(ti[u] << 2), int(d0)));
                        i1[u] = uint32_t(__builtin_amdgcn_ds_bpermute(int(ti[u] << 2), int(d1)));
                    }
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t jj = xw[u] - (i0[u] & 0x7ffu);
                        const bool copy = ((i0[u] >> 11) & 1u) == X2_COPY;
                        const uint32_t offv = max(i0[u] >> 16, 1u);
                        const uint32_t r = (i0[u] & (1u << 12)) ? mod_small(jj & 63u, offv) : jj;
                        const uint32_t y = i1[u] + r;                 // copy: absolute output position of the source byte
                        pend[u] = act[u] && copy && y >= s0;          // produced in this window
                        addr[u] = copy ? (y & XRMASK) : (i1[u] + jj);
                        W[u] = 0x100u | ((y - s0) & 0xffu);
                    }
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t v = uint32_t(L[addr[u]]);
                        W[u] = pend[u] ? W[u] : (act[u] ? v : 0u);
                    }
                    // pointer jumping over the window's 256 bytes (a source always precedes its reader):
                    // every round publishes the window's words to LDS (byte x of the window at jv[x]) and
                    // each pending byte takes the word it points at. A single wave's LDS operations run in
                    // order, so the reads see this round's writes; one LDS read per byte and round instead
                    // of two permutes plus the half-word selects (~20 instead of ~60 VALU per round).
                    while (__any(((W[0] | W[1] | W[2] | W[3]) & 0x100u) != 0u)) {
                        if (lane == 0) STAMP_ADD(5, 1);
                        #pragma unroll
                        for (int u = 0; u < 4; u++) jv[64u * uint32_t(u) + uint32_t(lane)] = uint16_t(W[u]);
                        uint32_t G[4];
                        #pragma unroll
                        for (int u = 0; u < 4; u++) G[u] = jv[W[u] & 0xffu];
                        #pragma unroll
                        for (int u = 0; u < 4; u++) W[u] = (W[u] & 0x100u) ? G[u] : W[u];
                    }
                    #pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (act[u]) ring[(s0 + 64u * uint32_t(u) + uint32_t(lane)) & XRMASK] = uint8_t(W[u]);
                }
                XT(2);
                const uint32_t sl = flush_slots(ring, od, F, op + btot, lane);
                if (sl) nst = sl;
                XT(6);
            }
            op += btot;
            ip = __builtin_amdgcn_readlane(endp, int(used) - 1);
            sb += used;
        }
    }
    if (bad) {
        if (lane == 0) atomicMax(&fb[j], whole ? FB_SERIAL : FB_REDO);
        return;
    }
#ifdef PF_STAMPS
    if (lane == 0) STAMP_ADD(12, __builtin_amdgcn_s_memtime() - xt0);
#endif
    // tail: bytes [F, op)
    for (uint32_t a = F + uint32_t(lane) * 16u; a + 16u <= op; a += 1024u)
        put16(od, a, *reinterpret_cast<const u32x4*>(ring + (a & XRMASK)));
    for (uint32_t a = F + ((op - F) & ~15u) + uint32_t(lane); a < op; a += 64) put1(od, a, ring[a & XRMASK]);
}
#endif  // PF_DIAG

// ======================================================================== executor v5
//
// k_snappy_exec2 runs each 64-token batch as one serial instruction stream, and a dense piece
// (16 K tokens per 64 KiB: l_partkey, l_extendedprice; sorted l_orderkey) is issue-bound at one
// wave's rate — a wave alone on its SIMD issues a VALU instruction every 4 cycles — at ~600-700 K
// cycles; the slowest piece sets the executor launch. k_snappy_exec5 splits that stream over the
// two waves of one workgroup (two SIMDs), pipelined by one batch:
//   wave 0 (producer): stages input, enumerates token starts, decodes batch i's tokens (output
//     offsets, chain checks, cuts), loads its far-copy sources from HBM into LDS and writes the
//     packed descriptors and token-start words into LDS buffer i & 1;
//   wave 1 (consumer): meanwhile resolves batch i-1's bytes (exec2's windows, descriptors read from
//     LDS instead of permuted from the token lanes) into the ring and flushes whole ring slots.
// One workgroup barrier per batch. A far copy's source was flushed by the consumer: before every
// barrier the consumer waits until all but its newest store have landed (all of them after a long
// literal or an empty batch), the producer derives from the batch history the frontier below which
// that guarantees the bytes (and their cache line) are in HBM, and a far copy above it cuts the batch
// (one empty batch when it is the first token, which only follows a long literal).
#ifndef PF_X5_BATCH
#define PF_X5_BATCH 764
#endif
constexpr uint32_t X5_BATCH = PF_X5_BATCH;                     // output bytes of one batch (ring: + XSLOT + far margin)
constexpr uint32_t X5_STG = (XSTAGE + 15u) & ~15u;     // one staged input chunk
constexpr uint32_t X5_FSLOT = 80u;                     // a far copy's source: 5 aligned 16-byte chunks (<= 64 B + shift < 16)
constexpr uint32_t X5_FSL = XFAR * X5_FSLOT;           // far-copy source slots of one batch
constexpr uint32_t X5_STAGE0 = XRING;                  // [ring | stage x2 | far slots x2]: one byte address
constexpr uint32_t X5_LDS = XRING + 2u * X5_STG;       // selects any byte source (the far slots: their own array)
constexpr uint32_t X5_W = 768u / 32u;                  // token-start words of a batch (+ its alignment bytes)
constexpr uint32_t X5_LINE = 128u;                     // a far source's cache line must be wholly landed
constexpr uint32_t X5_FREAD = 5u * 16u;                // bytes a far load reads from its 16-byte aligned base
#ifndef PF_X5_TPL
#define PF_X5_TPL 2
#endif
constexpr int X5_TPL = PF_X5_TPL;                      // tokens a producer lane decodes per batch
constexpr uint32_t X5_DS = 64u * X5_TPL + 1u;          // descriptor table: entry t at [t], its second word at [t + X5_DS]
static_assert(X5_BATCH + 3u <= 768u, "a batch and its alignment bytes are at most three 256-byte windows");
static_assert((X5_FSLOT & 15u) == 0u, "far slots are 16-byte aligned");
static_assert(5u * XFAR <= 128u, "a batch's far-copy chunks are loaded by two LDS-DMA wave instructions");
enum : uint32_t { R5_NORMAL = 0, R5_LONG = 1, R5_NOP = 2, R5_END = 3, R5_BAD = 4 };
// Descriptor word 0: the token's first output byte relative to the batch's 4-byte aligned base S
// (bits 0-15); a copy whose source is read through the ring / the window: its offset (< 4 KiB) in bits
// 16-30 and bit 31 set. Word 1: a literal or far copy: the LDS address of its byte at base position x is
// word1 + x; a ring copy: m = floor(65536 / offset) + 1 (or one more), so that (j * m) >> 16 =
// floor(j / offset) for the byte's index j < 64 in the token: byte x's source is
// x - offset * (1 + floor(j / offset)), the byte an overlapping copy reads as j mod offset. Entry 0 is a
// dummy literal for the batch's alignment bytes (token t of the batch is entry t + 1).
constexpr uint32_t X5_CP = 0x80000000u;

// Workgroup barrier for LDS hand-over only (no wait on outstanding global stores).
__device__ __forceinline__ void x5_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// Compiler ordering point for one wave's LDS accesses (the hardware runs them in order).
__device__ __forceinline__ void x5_order() { asm volatile("" ::: "memory"); }

// Two 16-bit jump words at once: each half of w still pending (bit 15) takes the half of g
// (v_pk_ashrrev_i16 makes the per-half mask, v_bfi_b32 merges; the compiler otherwise splits the halves).
__device__ __forceinline__ uint32_t x5_pick(uint32_t w, uint32_t g) {
    uint32_t m, r;
    asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(m) : "v"(w));   // (the shift in both halves)
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(g), "v"(w));
    return r;
}

struct X5Lds {
    __attribute__((aligned(16))) uint8_t L[X5_LDS];
    uint16_t tokpos[XCHUNK / 2];
    uint32_t D[2][2 * X5_DS];            // token descriptors (entry 0: the dummy literal)
    uint32_t SB[2][X5_W], WP[2][X5_W];   // token starts from the batch's aligned base, tokens in earlier words
    uint32_t REC[2][4];                  // kind, output start, output bytes, long literal input position
    __attribute__((aligned(8))) uint16_t jv[256];
#if defined(PF_X5_PAD) && PF_X5_PAD > 0
    uint8_t pad[PF_X5_PAD];   // diagnostics: fewer executor workgroups per CU (room for other streams' kernels)
#endif
};

// 16 input bytes from gin[src] (src + 15 < the stream's end) as four dwords: 16-byte aligned loads only
// (the second chunk only when src is not aligned), so no load passes the chunk holding the last byte.
__device__ __forceinline__ u32x4 x5_load16(const PF_GLOBAL uint8_t* gin, uint32_t src) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(gin) + src;
    const PF_GLOBAL u32x4* p = (const PF_GLOBAL u32x4*)(a & ~uintptr_t(15));
    const uint32_t sh = uint32_t(a & 15u);
    const u32x4 A = p[0];
    u32x4 B = A;
    if (sh) B = p[1];
    const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    const uint32_t k = sh >> 2, s = sh & 3u;
    u32x4 r;
    #pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = k == 0 ? w[i] : (k == 1 ? w[i + 1] : (k == 2 ? w[i + 2] : w[i + 3]));
        const uint32_t hi = k == 0 ? w[i + 1] : (k == 1 ? w[i + 2] : (k == 2 ? w[i + 3] : w[i + 4]));
        r[i] = __builtin_amdgcn_alignbyte(hi, lo, s);
    }
    return r;
}

// 16 bytes a lane from global address g into LDS at m0 + 16 * lane (LDS-DMA). Issued from inline asm: the
// compiler, which cannot tell the destination from the producer's other LDS accesses, would otherwise wait
// for the load before the next of them; the producer waits for it itself before the batch's barrier.
// (m0 is a reserved register the compiler does not take as a clobber; no code it generates for this file's
// kernels reads m0 -- checked in the assembly, round 6 -- so every m0 value is this function's.)
__device__ __forceinline__ void x5_dma16(uint64_t g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g), "s"(lds) : "memory");
}

// One input chunk [I - woff, I - woff + XSTAGE) as lane l's 16-byte chunks l and 64 + l (lanes < 5), and its
// token-start bits (16 input bytes a lane): every load issued before any is used. Chunks wholly at or past n
// read as zero (the chunk holding the last byte is read whole, as snap_stage does).
static_assert(XSTAGE == 64u * 16u + 5u * 16u, "a staged chunk is 64 + 5 lane loads");
__device__ __forceinline__ void x5_chunk_load(const PF_GLOBAL uint8_t* gin, const PF_GLOBAL uint16_t* tm16, uint64_t n, uint32_t I,
                                              int lane, u32x4& va, u32x4& vb, uint32_t& bits) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(gin + I);
    const uint32_t woff = uint32_t(a & 15u);
    const PF_GLOBAL u32x4* src = (const PF_GLOBAL u32x4*)(a - woff);
    const int64_t first = int64_t(I) - int64_t(woff);
    va = u32x4{0u, 0u, 0u, 0u};
    vb = u32x4{0u, 0u, 0u, 0u};
    bits = 0u;
    if (first + 16 * int64_t(lane) < int64_t(n)) va = src[lane];
    if (lane < 5 && first + 16 * int64_t(64 + lane) < int64_t(n)) vb = src[64 + lane];
    const uint32_t p16 = I + 16u * uint32_t(lane);
    if (uint64_t(p16) < n) bits = uint32_t(tm16[p16 >> 4]);
}

// One piece (mode 0: pieces[item]) or one whole-page redo (mode 1: job item) by the workgroup's two waves.
__device__ __forceinline__ void exec5_piece(X5Lds& S, uint8_t* FS, const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                            const uint32_t* __restrict__ splits, int* __restrict__ fb, int mode, int item) {
    uint8_t* const L = S.L;
    uint16_t* const tokpos = S.tokpos;
    auto& D = S.D;
    auto& SB = S.SB;
    auto& WP = S.WP;
    auto& REC = S.REC;
    uint8_t* const jvb = reinterpret_cast<uint8_t*>(S.jv);
    uint8_t* const ring = L;
    // The far-copy slots are a separate LDS array, so the compiler can tell the producer's LDS-DMA from its
    // other LDS accesses (one array: it waits for the loads before the first descriptor write); the
    // consumer reaches them through the same byte address as the ring and stage, relative to L.
    const uint32_t Lb = uint32_t(reinterpret_cast<uintptr_t>(L));   // (a flat LDS address's low half: the LDS offset)
    const uint32_t FSB = uint32_t(reinterpret_cast<uintptr_t>(FS)) - Lb;
    const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
    const int lane = int(threadIdx.x) & 63;
    int j, k;
    if (mode == 0) {
        const int2 pc = pieces[item];
        j = pc.x;
        k = pc.y;
    } else {
        j = item;
        k = 0;
    }
    const int f = fb[j];
    bool whole;
    if (mode == 0) {
        if (f >= FB_REDO || (f == FB_WHOLE && k > 0)) return;
        whole = f == FB_WHOLE;
    } else {
        if (f != FB_REDO) return;
        whole = true;
    }
    const SnappyJob job = jobs[j];
    const uint8_t* in = job.src;
    const uint64_t n = job.src_len;
    const uint32_t* sp = splits + job.split_base;
    uint64_t pos0 = 0, ulen = 0;
    if (!uvarint(in, n, pos0, ulen) || ulen != job.dst_len) {
        if (threadIdx.x == 0) atomicMax(&fb[j], FB_SERIAL);
        return;
    }
    if (mode == 0 && (job.dflags & 1u)) {   // diagnostics: forced redo
        if (threadIdx.x == 0) atomicMax(&fb[j], FB_REDO);
        return;
    }
    uint32_t ip, out_start, out_end = job.dst_len;
    if (whole) {
        ip = uint32_t(pos0);
        out_start = 0;
    } else {
        if (k > 0 && sp[k] == SNAP_INVALID) return;   // no token at this boundary: an earlier piece covers it
        ip = k == 0 ? uint32_t(pos0) : sp[k];
        out_start = uint32_t(k) * SNAP_BLOCK;
        for (uint32_t k2 = k + 1; k2 < job.n_pieces; k2++)
            if (sp[k2] != SNAP_INVALID) { out_end = k2 * SNAP_BLOCK; break; }
    }
    const PF_GLOBAL uint16_t* tm16 = (const PF_GLOBAL uint16_t*)(job.tokmap);
    const PF_GLOBAL uint8_t* gin = gptr(in);
    PF_GLOBAL uint8_t* gdst = gptr(job.dst);
    const OutDst od{gdst, mode == 0 ? gptr(job.ddst) : nullptr, job.dlo, job.dgran};
    if (threadIdx.x < 2) {   // the dummy entry of both descriptor buffers (a literal reading ring bytes)
        D[threadIdx.x][0] = 0u;
        D[threadIdx.x][X5_DS] = 0u;
    }
    // producer state
    uint32_t op = out_start, sb = 0, T = 0, I = 0, woff = 0, cb = 1;
    uint32_t ops_m1 = out_start, k_m1 = R5_NOP, k_m2 = R5_NOP, nops = 0;
    uint32_t pfI = ~0u, pfbits = 0;   // prefetched input chunk (base, token-start bits, data)
    u32x4 pfa = {0u, 0u, 0u, 0u}, pfb = {0u, 0u, 0u, 0u};
    // consumer state
    uint32_t F = out_start, cop = out_start;
    uint32_t last = R5_END;
#ifdef PF_STAMPS   // per phase cycles: producer slots 0-4 (wave 0), consumer 6-9 (wave 1), 12 batches, 13 pieces
    unsigned long long x5t = __builtin_amdgcn_s_memtime();
#define X5T(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (lane == 0) STAMP_ADD(i, t_ - x5t); x5t = t_; } while (0)
    if (threadIdx.x == 0) STAMP_ADD(13, 1);
#else
#define X5T(i) ((void)0)
#endif
    for (uint32_t it = 0;; it++) {
        const uint32_t b = it & 1u;
        if (wv == 0) {
            if (lane == 0) STAMP_ADD(12, 1);
            // ---------------- producer: batch it into buffer b
            uint32_t kind = R5_BAD, b_op = op, b_tot = 0, b_s0 = 0;
            // landed frontier: the consumer finished batch it-2 before the last barrier
            const uint32_t sf = out_start + ((ops_m1 - out_start) & ~(XSLOT - 1u));
            const uint32_t LF = k_m2 == R5_NORMAL ? (sf >= out_start + XSLOT ? sf - XSLOT : out_start) : sf;
            bool ok = true;
            if (op >= out_end) {
                kind = R5_END;
                ok = false;
            } else if (sb >= T) {   // next input chunk (the other stage buffer: the consumer may read this one)
                if (ip >= n) {
                    ok = false;
                } else {
                    I = ip & ~15u;
                    cb ^= 1u;
                    // the chunk from the registers when the last staging prefetched it (the next chunk starts
                    // where the last token of this one ends: past I + XCHUNK, in the same 16 bytes unless that
                    // token is a literal)
                    u32x4 va, vb;
                    uint32_t bits;
                    if (I == pfI) {
                        va = pfa;
                        vb = pfb;
                        bits = pfbits;
                    } else {
                        x5_chunk_load(gin, tm16, n, I, lane, va, vb, bits);
                    }
                    u32x4* stq = reinterpret_cast<u32x4*>(L + X5_STAGE0 + cb * X5_STG);
                    stq[lane] = va;
                    if (lane < 5) stq[64 + lane] = vb;
                    woff = uint32_t(reinterpret_cast<uintptr_t>(gin + I) & 15u);
                    // prefetch the next chunk: its loads land while this chunk's batches are decoded
                    pfI = I + XCHUNK;
                    if (uint64_t(pfI) < n) x5_chunk_load(gin, tm16, n, pfI, lane, pfa, pfb, pfbits);
                    else pfI = ~0u;
                    const uint32_t p16 = I + 16u * uint32_t(lane);
                    if (p16 + 16u <= ip) bits = 0;
                    else if (p16 < ip) bits &= ~((1u << (ip - p16)) - 1u);
                    const uint32_t cnt = __popc(bits);
                    const uint32_t ex = dpp_incl_scan(cnt);
                    T = __builtin_amdgcn_readlane(ex, 63);
                    uint32_t q = ex - cnt;
                    while (bits) {
                        const uint32_t bb = uint32_t(__ffs(bits) - 1);
                        bits &= bits - 1;
                        tokpos[q++] = uint16_t(16u * uint32_t(lane) + bb);
                    }
                    sb = 0;
                    x5_order();
                    if (T == 0) ok = false;
                }
            }
            X5T(0);   // chunk staging + token enumeration
            if (ok) {
                // X5_TPL tokens a lane: token sb + 64 h + lane in half h (batches of up to 64 X5_TPL tokens)
                const uint32_t stg_off = __builtin_amdgcn_readfirstlane(cb) ? X5_STAGE0 + X5_STG : X5_STAGE0;
                const uint8_t* stg = L + stg_off;
                uint32_t pos[X5_TPL], ol[X5_TPL], start[X5_TPL], endp[X5_TPL], inc[X5_TPL], otok[X5_TPL];
                bool v[X5_TPL], take[X5_TPL];
                SnapTok32 tk[X5_TPL];
                #pragma unroll
                for (int h = 0; h < X5_TPL; h++) {
                    const uint32_t t = sb + 64u * uint32_t(h) + uint32_t(lane);
                    v[h] = t < T;
                    pos[h] = uint32_t(tokpos[min(t, XCHUNK / 2u - 1u)]);   // (read unconditionally; v gates the use)
                    if (!v[h]) pos[h] = 0u;
                }
                uint32_t tlo[X5_TPL], thi[X5_TPL];
                #pragma unroll
                for (int h = 0; h < X5_TPL; h++) lds_read8_2(stg, woff + pos[h], tlo[h], thi[h]);
                #pragma unroll
                for (int h = 0; h < X5_TPL; h++) tk[h] = snap_tok32(tlo[h], thi[h]);
                int nt = 0;
                bool wrong = false;
                uint32_t prevlast = ip, incbase = 0;
                #pragma unroll
                for (int h = 0; h < X5_TPL; h++) {
                    ol[h] = v[h] ? tk[h].ol : 0u;
                    start[h] = I + pos[h];
                    endp[h] = __builtin_elementwise_add_sat(start[h], tk[h].tl);
                    const uint32_t pdpp = dpp_prev(endp[h]);   // (every lane runs the DPP move)
                    const uint32_t prev = lane == 0 ? prevlast : pdpp;
                    inc[h] = incbase + dpp_incl_scan(ol[h]);
                    otok[h] = op + inc[h] - ol[h];
                    take[h] = v[h] && otok[h] < out_end;
                    nt += __popcll(__ballot(take[h]));
                    wrong = wrong || (take[h] && (start[h] != prev || endp[h] > n || op + inc[h] > out_end || inc[h] < ol[h] ||
                                                  inc[h] < incbase));
                    prevlast = __builtin_amdgcn_readlane(endp[h], 63);
                    incbase = __builtin_amdgcn_readlane(inc[h], 63);
                }
                if (__any(wrong) || nt == 0) {
                    ok = false;
                } else {
                    uint32_t kd[X5_TPL], off[X5_TPL], srcv[X5_TPL], a[X5_TPL], frank[X5_TPL];
                    bool farc[X5_TPL], fnr[X5_TPL], lstaged[X5_TPL];
                    unsigned long long farm[X5_TPL], cutm[X5_TPL];
                    uint32_t fbase = 0;
                    #pragma unroll
                    for (int h = 0; h < X5_TPL; h++) {
                        kd[h] = tk[h].kind;
                        off[h] = tk[h].arg;
                        srcv[h] = start[h] + tk[h].arg;   // literal data position
                        lstaged[h] = srcv[h] + ol[h] <= I + XCHUNK + 64;
                        a[h] = otok[h] - off[h];          // copy source start
                        farc[h] = take[h] && kd[h] != 0 && a[h] + min(ol[h], off[h]) <= op &&
                                  int32_t(a[h] - (op + X5_BATCH - XRING)) < 0;
                        // source not yet landed in HBM: every cache line its 80-byte aligned read touches must be
                        fnr[h] = farc[h] && a[h] + X5_FREAD + X5_LINE > LF;
                        farm[h] = __ballot(farc[h]);
                        frank[h] = fbase + uint32_t(__popcll(farm[h] & lane_mask_lt(uint32_t(lane))));
                        fbase += uint32_t(__popcll(farm[h]));
                        cutm[h] = __ballot(take[h] && (ol[h] > 64u || inc[h] > X5_BATCH || (kd[h] == 0 && !lstaged[h]) ||
                                                       (farc[h] && frank[h] >= XFAR) || fnr[h]));
                    }
                    uint32_t cut = uint32_t(nt);
                    #pragma unroll
                    for (int h = X5_TPL - 1; h >= 0; h--)
                        if (cutm[h]) cut = 64u * uint32_t(h) + uint32_t(__ffsll(cutm[h]) - 1);
                    uint32_t used = 0;
                    if (cut == 0) {
                        if (__builtin_amdgcn_readfirstlane(kd[0]) == 0) {   // one long literal: the consumer copies it
                            kind = R5_LONG;
                            b_tot = __builtin_amdgcn_readfirstlane(ol[0]);
                            b_s0 = __builtin_amdgcn_readfirstlane(srcv[0]);
                            used = 1;
                            nops = 0;
                        } else if (__builtin_amdgcn_readfirstlane(uint32_t(fnr[0])) && nops < 3) {
                            kind = R5_NOP;   // wait one batch for the source's stores to land
                            nops++;
                        } else {
                            ok = false;
                        }
                    } else {
                        used = cut;
                        const uint32_t ch = (cut - 1u) >> 6;   // the half holding the batch's last token
                        uint32_t btot = 0;
                        #pragma unroll
                        for (int h = 0; h < X5_TPL; h++)
                            if (ch == uint32_t(h)) btot = __builtin_amdgcn_readlane(inc[h], (cut - 1u) & 63u);
                        bool inb[X5_TPL], lit[X5_TPL], cp[X5_TPL], far[X5_TPL];
                        bool bad = false;
                        #pragma unroll
                        for (int h = 0; h < X5_TPL; h++) {
                            inb[h] = take[h] && 64u * uint32_t(h) + uint32_t(lane) < cut;
                            lit[h] = inb[h] && kd[h] == 0;
                            cp[h] = inb[h] && kd[h] != 0;
                            far[h] = cp[h] && farc[h];
                            bad = bad || (cp[h] && (off[h] == 0 || off[h] > otok[h] - out_start));
                            // a far source straddling the direct split (level bytes | values) is not one window
                            bad = bad || (od.dd != nullptr && far[h] && a[h] < od.dlo && a[h] + ol[h] > od.dlo);
                        }
                        if (__any(bad)) ok = false;
                        X5T(1);   // token decode, chain checks, cuts
                        if (ok) {
                            uint32_t fsh[X5_TPL];
                            uint32_t nfar = 0;
                            uint64_t* fa = reinterpret_cast<uint64_t*>(FS + b * X5_FSL);   // (overwritten by the loads)
                            #pragma unroll
                            for (int h = 0; h < X5_TPL; h++) {
                                const PF_GLOBAL uint8_t* fb0 = od.dd != nullptr && a[h] >= od.dlo ? od.dd + a[h] : gdst + a[h];
                                fsh[h] = uint32_t(reinterpret_cast<uintptr_t>(fb0) & 15u);
                                if (far[h]) fa[frank[h]] = reinterpret_cast<uintptr_t>(fb0) & ~uintptr_t(15);
                                nfar += uint32_t(__popcll(farm[h] & lane_mask_lt(cut > 64u * uint32_t(h) ? cut - 64u * uint32_t(h) : 0u)));
                            }
                            // far-copy sources: five aligned 16-byte chunks each (the arenas keep >= 80 bytes of
                            // slack), loaded straight into the slots by LDS-DMA -- lane l loads chunk l % 5 of far
                            // copy l / 5, so the lane-linear destination is the slot layout -- and waited for only
                            // before the barrier, after the descriptors (no data registers, latency behind them)
                            if (nfar) {
                                x5_order();
                                const uint32_t l0 = uint32_t(lane), f0 = (l0 * 205u) >> 10;   // l / 5 for l < 128
                                const uint64_t s0a = fa[f0] + 16u * (l0 - 5u * f0);
                                uint64_t s1a = 0;
                                if (nfar > 12u) {
                                    const uint32_t l1 = l0 + 64u, f1 = (l1 * 205u) >> 10;
                                    s1a = fa[min(f1, XFAR - 1u)] + 16u * (l1 - 5u * f1);
                                }
                                uint8_t* slots = FS + b * X5_FSL;
                                const uint32_t sl0 = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(slots)));
                                if (l0 < 5u * nfar) x5_dma16(s0a, sl0);
                                if (nfar > 12u && l0 + 64u < 5u * nfar) x5_dma16(s1a, sl0 + 1024u);
                            }
                            X5T(2);   // far-copy source loads (issued)
                            if (lane < int(X5_W)) SB[b][lane] = 0;
                            #pragma unroll
                            for (int h = 0; h < X5_TPL; h++) {
                                const uint32_t relS = otok[h] - (op & ~3u);   // from the batch's aligned base
                                uint32_t d0 = 0, d1 = 0;
                                if (inb[h]) {
                                    const bool near = cp[h] && !far[h];
                                    d0 = relS | (near ? (X5_CP | (off[h] << 16)) : 0u);
                                    d1 = near ? uint32_t(65536.0f * __builtin_amdgcn_rcpf(float(off[h]))) + 1u
                                              : (lit[h] ? stg_off + woff + (srcv[h] - I) - relS
                                                        : FSB + b * X5_FSL + frank[h] * X5_FSLOT + fsh[h] - relS);
                                }
                                D[b][1 + 64 * h + lane] = d0;
                                D[b][1 + X5_DS + 64 * h + lane] = d1;
                                x5_order();
                                if (inb[h]) atomicOr(&SB[b][relS >> 5], 1u << (relS & 31u));
                            }
                            x5_order();
                            const uint32_t c = lane < int(X5_W) ? __popc(SB[b][lane]) : 0u;
                            const uint32_t e2 = dpp_incl_scan(c) - c;
                            if (lane < int(X5_W)) WP[b][lane] = e2;
                            kind = R5_NORMAL;
                            b_tot = btot;
                            nops = 0;
                        }
                    }
                    if (ok && used) {
                        op += b_tot;
                        const uint32_t uh = (used - 1u) >> 6;
                        #pragma unroll
                        for (int h = 0; h < X5_TPL; h++)
                            if (uh == uint32_t(h)) ip = __builtin_amdgcn_readlane(endp[h], (used - 1u) & 63u);
                        sb += used;
                    }
                }
            }
            if (!ok && kind != R5_END) kind = R5_BAD;
            if (lane == 0) {
                REC[b][0] = kind;
                REC[b][1] = b_op;
                REC[b][2] = b_tot;
                REC[b][3] = b_s0;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // far-copy slots landed in LDS
            X5T(3);   // descriptors, token-start words, far-copy loads landed
            k_m2 = k_m1;
            k_m1 = kind;
            ops_m1 = b_op;
        } else if (it > 0) {
            // ---------------- consumer: batch it-1 from buffer b ^ 1
            const uint32_t pb = b ^ 1u;
            const uint32_t kind = __builtin_amdgcn_readfirstlane(REC[pb][0]);
            const uint32_t s0 = __builtin_amdgcn_readfirstlane(REC[pb][1]);
            const uint32_t btot = __builtin_amdgcn_readfirstlane(REC[pb][2]);
            if (kind == R5_NORMAL) {
                // 256-byte windows from the aligned base Sb = s0 & ~3, four consecutive bytes a lane; the
                // al = s0 & 3 bytes before s0 belong to the previous batch (read, never written)
                const uint32_t al = s0 & 3u;
                const uint32_t Sb = s0 - al;
                const uint32_t btS = btot + al;
                const uint32_t* sbw = SB[pb];
                const uint32_t* wpw = WP[pb];
                const uint32_t* Dp = D[pb];
                for (uint32_t w0 = 0; w0 < btS; w0 += 256) {
                    const uint32_t x0 = w0 + 4u * uint32_t(lane);
                    const uint32_t ws = w0 == 0 ? al : w0;   // sources at or past ws are resolved in the window
                    const uint32_t wd = x0 >> 5, sh = x0 & 31u;
                    const uint32_t sbv = sbw[wd];
                    const uint32_t t0 = wpw[wd] + __popc(sbv & ((2u << sh) - 1u));   // entry of byte x0
                    const uint32_t nb = sbv >> sh;
                    uint32_t tk[4];
                    tk[0] = t0;
                    tk[1] = t0 + ((nb >> 1) & 1u);
                    tk[2] = tk[1] + ((nb >> 2) & 1u);
                    tk[3] = tk[2] + ((nb >> 3) & 1u);
                    uint32_t d0[4], d1[4];
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        d0[u] = Dp[tk[u]];
                        d1[u] = Dp[tk[u] + X5_DS];
                    }
                    uint32_t addr[4], pw[4];
                    bool pend[4];
                    #pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t x = x0 + uint32_t(u);
                        const uint32_t jj = x - (d0[u] & 0xffffu);
                        const bool cp = int32_t(d0[u]) < 0;
                        const uint32_t q = __umul24(jj, d1[u]) >> 16;        // floor(jj / offset) (copies)
                        const uint32_t of = (d0[u] >> 16) & 0x7fffu;
                        uint32_t t;   // of * q + of, kept a 24-bit multiply (the compiler folds it into v_mad_u64_u32)
                        asm("v_mad_u32_u24 %0, %1, %2, %1" : "=v"(t) : "v"(of), "v"(q));
                        const uint32_t y = x - t;                            // a copy's source (from Sb; may wrap)
                        pend[u] = cp && int32_t(y) >= int32_t(ws);
                        addr[u] = cp ? ((Sb + y) & XRMASK) : (d1[u] + x);
                        // (bits above the window's 8 stay in the word: the rounds mask the address with 0x1fe)
                        pw[u] = 0x8000u | (y << 1);
                    }
                    // the four source reads issued together (every addr is inside the workgroup's LDS)
                    uint32_t vv[4];
                    #pragma unroll
                    for (int u = 0; u < 4; u++) vv[u] = uint32_t(*reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(size_t(Lb + addr[u])));
                    asm volatile("" : "+v"(vv[0]), "+v"(vv[1]), "+v"(vv[2]), "+v"(vv[3]));
                    // jump words, two per dword: (value << 1), or 0x8000 | (window position << 1) while pending
                    uint32_t Wa = (pend[0] ? pw[0] : (vv[0] << 1)) | ((pend[1] ? pw[1] : (vv[1] << 1)) << 16);
                    uint32_t Wb = (pend[2] ? pw[2] : (vv[2] << 1)) | ((pend[3] ? pw[3] : (vv[3] << 1)) << 16);
                    while (__any(((Wa | Wb) & 0x80008000u) != 0u)) {
                        *reinterpret_cast<uint2*>(jvb + 8u * uint32_t(lane)) = make_uint2(Wa, Wb);
                        const uint32_t g0 = *reinterpret_cast<const uint16_t*>(jvb + (Wa & 0x1feu));
                        const uint32_t g1 = *reinterpret_cast<const uint16_t*>(jvb + ((Wa >> 16) & 0x1feu));
                        const uint32_t g2 = *reinterpret_cast<const uint16_t*>(jvb + (Wb & 0x1feu));
                        const uint32_t g3 = *reinterpret_cast<const uint16_t*>(jvb + ((Wb >> 16) & 0x1feu));
                        const uint32_t ga = __builtin_amdgcn_perm(g1, g0, 0x05040100u), gb = __builtin_amdgcn_perm(g3, g2, 0x05040100u);
                        Wa = x5_pick(Wa, ga);
                        Wb = x5_pick(Wb, gb);
                    }
                    const uint32_t o4 = __builtin_amdgcn_perm(Wb >> 1, Wa >> 1, 0x06040200u);
                    if (x0 < btS) {
                        const uint32_t ra = (Sb + x0) & XRMASK;
                        if (x0 >= al) {   // (a dword past the batch end writes <= 3 bytes the next batch rewrites)
                            *reinterpret_cast<uint32_t*>(ring + ra) = o4;
                        } else {          // the batch's first dword: only bytes from s0 on
                            #pragma unroll
                            for (uint32_t u = 1; u < 4; u++)
                                if (u >= al) ring[ra + u] = uint8_t(o4 >> (8u * u));
                        }
                    }
                }
                X5T(6);   // windows
                flush_slots(ring, od, F, s0 + btot, lane);
                cop = s0 + btot;
                X5T(7);   // flush
                asm volatile("s_waitcnt vmcnt(1)" ::: "memory");   // all but the newest store have landed
                X5T(8);   // store drain
            } else if (kind == R5_LONG) {
                // bytes [s0, s0 + btot) = input [sl, sl + btot): whole 16-byte ring blocks from 16-byte loads,
                // the partial first / last block byte by byte
                const uint32_t sl = __builtin_amdgcn_readfirstlane(REC[pb][3]);
                const uint32_t e = s0 + btot;
                for (uint32_t base = s0 & ~15u; base < e; base += XLIT) {
                    const uint32_t p = base + 16u * uint32_t(lane);   // this lane's block
                    if (p < e) {
                        if (p >= s0 && p + 16u <= e) {
                            *reinterpret_cast<u32x4*>(ring + (p & XRMASK)) = x5_load16(gin, sl + (p - s0));
                        } else {
                            for (uint32_t q = max(p, s0); q < min(p + 16u, e); q++) ring[q & XRMASK] = gin[sl + (q - s0)];
                        }
                    }
                    flush_slots(ring, od, F, min(base + XLIT, e), lane);
                }
                cop = e;
                wait_vmem();
            } else {
                wait_vmem();
            }
        }
        X5T(9);   // (long literal / empty batch)
        x5_barrier();
        if (wv == 0) X5T(4); else X5T(10);   // barrier wait
        last = __builtin_amdgcn_readfirstlane(REC[b][0]);
        if (last >= R5_END) break;
    }
    if (last == R5_BAD) {
        if (threadIdx.x == 0) atomicMax(&fb[j], whole ? FB_SERIAL : FB_REDO);
        return;
    }
    if (wv == 1) {   // tail: bytes [F, cop)
        for (uint32_t a = F + uint32_t(lane) * 16u; a + 16u <= cop; a += 1024u)
            put16(od, a, *reinterpret_cast<const u32x4*>(ring + (a & XRMASK)));
        for (uint32_t a = F + ((cop - F) & ~15u) + uint32_t(lane); a < cop; a += 64) put1(od, a, ring[a & XRMASK]);
    }
#undef X5T
}

// One workgroup per item: mode 0 = a 64 KiB piece (pieces[blockIdx.x]), mode 1 = a whole-page redo.
__global__ __launch_bounds__(128) void k_snappy_exec5(const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                                      const uint32_t* __restrict__ splits, int* __restrict__ fb, int mode) {
    __shared__ X5Lds S;
    __shared__ __attribute__((aligned(16))) uint8_t FS[2 * X5_FSL];   // far-copy source slots of two batches
    exec5_piece(S, FS, jobs, pieces, splits, fb, mode, int(blockIdx.x));
}

#ifdef PF_STAMPS
extern "C" int pf_debug_stamps(unsigned long long* out, int n, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_stamps), sizeof(unsigned long long) * (n < 16 ? n : 16)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pf_stamps), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif

void launch_snappy_serial(const SnappyJob*, int, const int*, DevChunkResult*, hipStream_t);

// Parse stage (token-start bitmaps, chain, 64 KiB split points) and execute stage, separately so
// the runtime can time them apart.
void launch_snappy_parse(const SnappyJob* d_jobs, int n_jobs, const int2* d_wins, int n_wins, SnapWin* d_win,
                         SnapEnt* d_ent, uint32_t* d_lane_out, uint32_t* d_splits, int* d_fb, int max_nwin, hipStream_t s) {
    if (n_jobs <= 0) return;
    hipLaunchKernelGGL(k_snappy_index, dim3(n_wins), dim3(64), 0, s, d_jobs, d_wins, d_win, d_ent, d_lane_out, d_fb);
    // per-window tables of the largest page (multiple of 16 windows; pages above FIX_MAXW go serial)
    const uint32_t cap = uint32_t(std::min(FIX_MAXW, (std::max(max_nwin, 1) + 15) & ~15));
    hipLaunchKernelGGL(k_snappy_chain, dim3(n_jobs), dim3(64), 5 * 4 * cap, s, d_jobs, d_win, (const SnapEnt*)d_ent,
                       d_lane_out, d_fb, cap);
#ifndef PF_REPAIR_GRID   // (1024: SF1 3.30 ms mean of 6 interleaved runs; 4096: 3.28; one per window: 3.26 of 3)
#define PF_REPAIR_GRID (1 << 24)
#endif
    hipLaunchKernelGGL(k_snappy_repair, dim3(std::min(n_wins, PF_REPAIR_GRID)), dim3(64), 0, s, d_jobs, d_wins, n_wins,
                       (const SnapWin*)d_win, d_lane_out, d_fb);
    hipLaunchKernelGGL(k_snappy_splits, dim3(n_jobs), dim3(SP_NT), 0, s, d_jobs, (const SnapWin*)d_win,
                       (const uint32_t*)d_lane_out, d_splits, d_fb);
}

void launch_snappy_exec(const SnappyJob* d_jobs, int n_jobs, const int2* d_pieces, int n_pieces, uint32_t* d_splits,
                        int* d_fb, DevChunkResult* d_res, int exec, hipStream_t s) {
    if (n_jobs <= 0) return;
    // exec (PfOpts; the diagnostics build's PF_EXEC): 5 = producer / consumer waves (default), 2 = one wave
    // per piece. The whole-page redo is always the same kernel's mode 1.
#ifdef PF_DIAG
    if (exec == 2) {
        hipLaunchKernelGGL(k_snappy_exec2, dim3(n_pieces), dim3(64), 0, s, d_jobs, d_pieces, (const uint32_t*)d_splits, d_fb, 0);
        // whole-page redo of pages whose pieces were not independent
        hipLaunchKernelGGL(k_snappy_exec2, dim3(n_jobs), dim3(64), 0, s, d_jobs, d_pieces, (const uint32_t*)d_splits, d_fb, 1);
    } else
#else
    (void)exec;
#endif
    {
        hipLaunchKernelGGL(k_snappy_exec5, dim3(n_pieces), dim3(128), 0, s, d_jobs, d_pieces, (const uint32_t*)d_splits, d_fb, 0);
        hipLaunchKernelGGL(k_snappy_exec5, dim3(n_jobs), dim3(128), 0, s, d_jobs, d_pieces, (const uint32_t*)d_splits, d_fb, 1);
    }
    launch_snappy_serial(d_jobs, n_jobs, d_fb, d_res, s);
}

// All Snappy work of one batch, in stream order. fb must be zero on entry.
void launch_snappy(const SnappyJob* d_jobs, int n_jobs, const int2* d_wins, int n_wins, SnapWin* d_win,
                   SnapEnt* d_ent, uint32_t* d_lane_out, const int2* d_pieces, int n_pieces, uint32_t* d_splits,
                   int* d_fb, DevChunkResult* d_res, int max_nwin, int exec, hipStream_t s) {
    launch_snappy_parse(d_jobs, n_jobs, d_wins, n_wins, d_win, d_ent, d_lane_out, d_splits, d_fb, max_nwin, s);
    launch_snappy_exec(d_jobs, n_jobs, d_pieces, n_pieces, d_splits, d_fb, d_res, exec, s);
}

}  // namespace pf
