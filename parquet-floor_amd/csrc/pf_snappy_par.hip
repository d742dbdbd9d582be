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
//                   input byte), per-lane output byte counts, the window exit.
//   k_snappy_fix    one wave per page. Window w's true entry is window w-1's exit; every window
//                   walks the true chain from there until it meets its own (guessed) chain —
//                   usually within a few tokens — and patches the bitmap; windows where they never
//                   meet are re-parsed. Iterates until no exit changes, checks the totals, then
//                   finds the input position of the token at each 64 KiB output boundary.
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
#else
#define STAMP_ADD(i, v) ((void)0)
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

// Walk the chain from c while positions stay below re (bits relative to rs).
__device__ void lane_walk(const uint8_t* stage, uint32_t woff, uint32_t W0, uint64_t n, uint32_t rs, uint32_t re,
                          uint32_t c, WinLane& L) {
    L.b0 = L.b1 = L.b2 = L.b3 = 0;
    L.out = 0;
    L.c = c;
    uint64_t p = c;
    bool bad = false;
    while (p < re) {
        const SnapTok t = snap_tok(lds_read8(stage, woff + uint32_t(p - W0)));
        bit_set(L, uint32_t(p) - rs);
        const uint32_t o = L.out + t.ol;
        L.out = o < L.out ? 0xffffffffu : o;
        p += t.tl;
        if (p > n) { bad = true; break; }
    }
    L.x = bad ? SNAP_INVALID : uint32_t(p);
}

// Parse one window whose chain enters at `entry` (W0 <= entry < min(W0 + SNAP_WIN, n)). All 64
// lanes. Returns the window exit; flags = WIN_BROKEN if the chain runs past the stream end.
__device__ uint32_t win_parse(const uint8_t* stage, uint32_t woff, uint32_t W0, uint64_t n, uint32_t entry, WinLane& L,
                              uint32_t& flags) {
    const int lane = threadIdx.x & 63;
    const uint32_t rs = W0 + uint32_t(lane) * SNAP_RB;
    const uint32_t re = uint32_t(min(uint64_t(rs) + SNAP_RB, n));
    const int L0 = int((entry - W0) / SNAP_RB);
    L.b0 = L.b1 = L.b2 = L.b3 = 0;
    L.out = 0;
    L.c = rs;
    L.x = SNAP_INVALID;
    if (lane >= L0 && uint64_t(rs) < n) lane_walk(stage, woff, W0, n, rs, re, lane == L0 ? entry : rs, L);
    uint32_t ent = SNAP_INVALID, X = SNAP_INVALID;
    bool converged = false;
    flags = 0;
    for (int round = 0; round <= 64; round++) {
        // follow the chain lane to lane (uniform scalar loop)
        ent = SNAP_INVALID;
        flags = 0;
        int k = L0;
        uint32_t e = entry;
        for (;;) {
            if (lane == k) ent = e;
            const uint32_t x = __builtin_amdgcn_readlane(L.x, k);
            if (x == SNAP_INVALID) { flags = WIN_BROKEN; X = SNAP_INVALID; break; }
            if (uint64_t(x) >= n || x >= W0 + SNAP_WIN) { X = x; break; }
            k = int((x - W0) / SNAP_RB);
            e = x;
        }
        const bool need = ent != SNAP_INVALID && ent != L.c && !(ent > L.c && bit_get(L, ent - rs));
        if (!__any(need)) { converged = true; break; }
        if (need) lane_walk(stage, woff, W0, n, rs, re, ent, L);
    }
    if (!converged) flags = WIN_BROKEN;
    // lanes off the chain hold no tokens; drop the guessed prefix before a lane's true entry
    if (ent == SNAP_INVALID) {
        L.b0 = L.b1 = L.b2 = L.b3 = 0;
        L.out = 0;
    } else if (ent > L.c) {
        uint32_t p = L.c;
        while (p < ent) {
            const SnapTok t = snap_tok(lds_read8(stage, woff + (p - W0)));
            bit_clr(L, p - rs);
            L.out -= t.ol;
            p += uint32_t(t.tl);
        }
        L.c = ent;
    }
    return X;
}

__device__ __forceinline__ uint32_t wave_sum_sat(uint32_t v) {
    uint64_t s = v;
    #pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    return s > 0xffffffffull ? 0xffffffffu : uint32_t(s);
}

__device__ __forceinline__ void store_window(uint32_t* tm, uint32_t* lo, const WinLane& L, int lane) {
    reinterpret_cast<uint4*>(tm)[lane] = make_uint4(L.b0, L.b1, L.b2, L.b3);
    lo[lane] = L.out;
}

__global__ __launch_bounds__(64) void k_snappy_index(const SnappyJob* __restrict__ jobs, const int2* __restrict__ wins,
                                                     SnapWin* __restrict__ win, uint32_t* __restrict__ lane_out,
                                                     int* __restrict__ fb) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SNAP_WSTAGE];
    const int2 jw = wins[blockIdx.x];
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
    const uint32_t woff = snap_stage(stage, job.src, n, W0, SNAP_WSTAGE, lane);
    __syncthreads();
    uint32_t flags;
    const uint32_t X = win_parse(stage, woff, W0, n, entry, L, flags);
    store_window(tm, lo, L, lane);
    const uint32_t sum = wave_sum_sat(L.out);
    if (lane == 0) win[wi] = SnapWin{entry, X, sum, flags};
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

// ======================================================================== fix pass

constexpr int FIX_MAXW = 1024;       // pages up to 8 MiB compressed (larger: serial fallback)
constexpr int MERGE_STEPS = 64;      // true-chain steps before a window is re-parsed instead
constexpr int FIX_ROUNDS = 256;

__device__ __forceinline__ bool tm_get(const uint32_t* tm, uint32_t i) { return (tm[i >> 5] >> (i & 31u)) & 1u; }
__device__ __forceinline__ void tm_set(uint32_t* tm, uint32_t i) { tm[i >> 5] |= 1u << (i & 31u); }
__device__ __forceinline__ void tm_clr(uint32_t* tm, uint32_t i) { tm[i >> 5] &= ~(1u << (i & 31u)); }

__global__ __launch_bounds__(64) void k_snappy_fix(const SnappyJob* __restrict__ jobs, SnapWin* __restrict__ win,
                                                   uint32_t* __restrict__ lane_out, uint32_t* __restrict__ splits,
                                                   int* __restrict__ fb) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SNAP_WSTAGE];
    __shared__ uint32_t s_x[FIX_MAXW], s_ent[FIX_MAXW], s_c[FIX_MAXW], s_pre[FIX_MAXW + 1];
    __shared__ uint8_t s_rr[FIX_MAXW], s_fl[FIX_MAXW], s_tr[FIX_MAXW];
    __shared__ uint32_t s_end;
    const int j = blockIdx.x;
    const int lane = threadIdx.x;
    const SnappyJob job = jobs[j];
    if (fb[j] == FB_SERIAL) return;
    const uint32_t nw = job.n_win;
    const uint64_t n = job.src_len;
    SnapWin* Wn = win + job.win_base;
    uint32_t* LO = lane_out + size_t(job.win_base) * 64;
    if (nw > uint32_t(FIX_MAXW) || (Wn[0].flags & WIN_BROKEN)) {
        if (lane == 0) fb[j] = FB_SERIAL;
        return;
    }
    bool ok = false;
    for (int round = 0; round < FIX_ROUNDS; round++) {
        for (uint32_t w = lane; w < nw; w += 64) {
            const SnapWin sw = Wn[w];
            s_x[w] = sw.exit;
            s_c[w] = sw.entry;
            s_fl[w] = uint8_t(sw.flags);
            s_rr[w] = 0;
        }
        __syncthreads();
        if (lane == 0) {
            // True entries along the chain, assuming each window's exit is right. While the entry is
            // trusted (derived from exact windows only), a window whose first token already leaves
            // it (a long literal) is resolved right here, so literal-only runs settle in one round.
            uint32_t e = s_x[0];
            bool trusted = true;
            for (uint32_t w = 1; w < nw; w++) {
                s_ent[w] = e;
                s_tr[w] = trusted;
                const uint64_t wend = min(uint64_t(w + 1) * SNAP_WIN, n);
                if (uint64_t(e) >= wend) continue;
                if (e == s_c[w] && !(s_fl[w] & (WIN_PASS | WIN_BROKEN))) { e = s_x[w]; continue; }
                if (trusted) {
                    const uint64_t x = e + snap_tok(glb_read8(job.src, n, e)).tl;
                    if (x >= wend && x <= n) { s_rr[w] = 2; e = uint32_t(x); continue; }
                }
                trusted = false;
                e = s_x[w];
            }
            for (uint32_t w = 0; w < nw; w++) TRACEF(0xEEEE0000u | uint32_t(round), w, w ? s_ent[w] : 0u, s_c[w], s_x[w], uint32_t(s_fl[w]) | (uint32_t(s_rr[w]) << 8));
        }
        __syncthreads();
        int changed = 0, serial = 0;
        for (uint32_t w = 1 + lane; w < nw; w += 64) {
            const uint32_t e = s_ent[w];
            const uint32_t W0 = w * SNAP_WIN;
            const uint64_t wend = min(uint64_t(W0) + SNAP_WIN, n);
            uint32_t* tm = job.tokmap + size_t(w) * SNAP_WWORDS;
            uint32_t* lo = LO + size_t(w) * 64;
            const uint32_t c = s_c[w], x0 = s_x[w], fl = s_fl[w];
            const bool pass = fl & WIN_PASS;
            // entry not known yet (an earlier window's exit is being re-derived this round): keep
            // this window's index results untouched for the next round
            if (e == SNAP_INVALID) continue;
            if (e >= wend) {   // jumped over by a literal: no token starts in this window
                if (!pass || c != e) {
                    for (int q = 0; q < 64; q++) { reinterpret_cast<uint4*>(tm)[q] = make_uint4(0, 0, 0, 0); lo[q] = 0; }
                    Wn[w] = SnapWin{e, e, 0, WIN_PASS};
                }
                continue;
            }
            if (e == c && !pass) continue;   // verified against this entry before
            uint64_t q = e;
            uint32_t acc = 0;
            bool merged = false, bad = false;
            if (s_rr[w] == 2) {   // a single token spans the rest of the window
                const SnapTok t = snap_tok(glb_read8(job.src, n, q));
                acc = t.ol;
                q += t.tl;
            } else {   // walk the true chain from e until it meets the window's chain
                int steps = 0;
                // a broken guessed chain has no trustworthy exit: never merge into it
                const bool nomerge = pass || (fl & WIN_BROKEN);
                while (q < wend && steps < MERGE_STEPS) {
                    if (!nomerge && tm_get(tm, uint32_t(q) - W0)) { merged = true; break; }
                    const SnapTok t = snap_tok(glb_read8(job.src, n, q));
                    acc += t.ol;
                    q += t.tl;
                    steps++;
                    if (q > n) { bad = true; break; }
                }
            }
            TRACEF(0xFFFF0000u | (bad ? 1u : 0u) | (merged ? 2u : 0u) | (q >= wend ? 4u : 0u), w, e, uint32_t(q), acc);
            if (bad) {   // the chain from e leaves the stream: corrupt if e is known true, else a bad guess
                if (s_tr[w]) serial = 1;
            } else if (merged) {
                const SnapWin sw = Wn[w];
                uint32_t rem = 0;
                for (uint64_t p = c; p < q;) {   // the guessed chain's tokens before the meeting point
                    const SnapTok t = snap_tok(glb_read8(job.src, n, p));
                    tm_clr(tm, uint32_t(p) - W0);
                    lo[(uint32_t(p) - W0) / SNAP_RB] -= t.ol;
                    rem += t.ol;
                    p += t.tl;
                }
                for (uint64_t p = e; p < q;) {   // the true ones
                    const SnapTok t = snap_tok(glb_read8(job.src, n, p));
                    tm_set(tm, uint32_t(p) - W0);
                    lo[(uint32_t(p) - W0) / SNAP_RB] += t.ol;
                    p += t.tl;
                }
                Wn[w] = SnapWin{e, sw.exit, sw.out - rem + acc, sw.flags};
            } else if (q >= wend) {   // the true chain crosses the window without meeting it
                for (int r = 0; r < 64; r++) { reinterpret_cast<uint4*>(tm)[r] = make_uint4(0, 0, 0, 0); lo[r] = 0; }
                for (uint64_t p = e; p < q;) {
                    const SnapTok t = snap_tok(glb_read8(job.src, n, p));
                    tm_set(tm, uint32_t(p) - W0);
                    lo[(uint32_t(p) - W0) / SNAP_RB] += t.ol;
                    p += t.tl;
                }
                Wn[w] = SnapWin{e, uint32_t(q), acc, 0};
                if (uint32_t(q) != x0) changed = 1;
            } else {
                s_rr[w] = 1;   // long divergence: re-parse below
            }
        }
        __threadfence();   // other lanes read these windows' tables next
        __syncthreads();
        for (uint32_t w = 1; w < nw; w++) {   // re-parse windows from their entry (whole wave)
            if (s_rr[w] != 1) continue;
            const uint32_t W0 = w * SNAP_WIN;
            const uint32_t e = s_ent[w];
            __syncthreads();
            const uint32_t woff = snap_stage(stage, job.src, n, W0, SNAP_WSTAGE, lane);
            __syncthreads();
            WinLane L;
            uint32_t fl;
            const uint32_t X = win_parse(stage, woff, W0, n, e, L, fl);
            store_window(job.tokmap + size_t(w) * SNAP_WWORDS, LO + size_t(w) * 64, L, lane);
            const uint32_t sum = wave_sum_sat(L.out);
            if (lane == 0) Wn[w] = SnapWin{e, X, sum, fl};
            if (lane == 0) TRACEF(0x99990000u, w, e, X, fl);
            if (X != s_x[w]) changed = 1;
        }
        if (__any(serial)) {
            if (lane == 0) fb[j] = FB_SERIAL;
            return;
        }
        const bool any_changed = __any(changed);
        __threadfence();
        __syncthreads();
        if (!any_changed) { ok = true; break; }
    }
    if (lane == 0) {   // the converged chain: every window entered where verified, none broken
        uint32_t e = Wn[0].exit;
        for (uint32_t w = 1; w < nw && ok; w++) {
            const SnapWin sw = Wn[w];
            if (uint64_t(e) >= min(uint64_t(w + 1) * SNAP_WIN, n)) continue;
            if (sw.entry != e || (sw.flags & (WIN_PASS | WIN_BROKEN))) ok = false;
            e = sw.exit;
        }
        s_end = ok ? e : SNAP_INVALID;
    }
    __syncthreads();
    // totals
    uint32_t run = 0;
    for (uint32_t w0 = 0; w0 < nw; w0 += 64) {
        const uint32_t w = w0 + lane;
        const uint32_t o = w < nw ? Wn[w].out : 0u;
        uint32_t x = o;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (w < nw) s_pre[w] = run + x - o;
        run += __shfl(x, 63, 64);
    }
    if (s_end != n || run != job.dst_len) {
        if (lane == 0) fb[j] = FB_SERIAL;
        return;
    }
    __syncthreads();
    // input position of the token starting at each 64 KiB output boundary
    uint32_t* sp = splits + job.split_base;
    for (uint32_t k = 1 + lane; k < job.n_pieces; k += 64) {
        const uint32_t B = k * SNAP_BLOCK;
        uint32_t a = 0, b = nw;   // last window with s_pre <= B
        while (b - a > 1) {
            const uint32_t m = (a + b) / 2;
            if (s_pre[m] <= B) a = m; else b = m;
        }
        const uint32_t w = a;
        uint32_t cum = s_pre[w];
        const uint32_t* lo = LO + size_t(w) * 64;
        int l = 0;
        for (; l < 63; l++) {
            const uint32_t v = lo[l];
            if (B < cum + v) break;
            cum += v;
        }
        const uint32_t rs = w * SNAP_WIN + uint32_t(l) * SNAP_RB;
        const uint32_t* tm = job.tokmap + size_t(w) * SNAP_WWORDS + l * 4;
        uint32_t found = SNAP_INVALID;
        bool done = false;
        for (int wd = 0; wd < 4 && !done; wd++) {
            uint32_t m = tm[wd];
            while (m) {
                const uint32_t p = rs + uint32_t(wd) * 32 + uint32_t(__ffs(m) - 1);
                m &= m - 1;
                if (cum == B) { found = p; done = true; break; }
                if (cum > B) { done = true; break; }
                cum += snap_tok(glb_read8(job.src, n, p)).ol;
            }
        }
        sp[k] = found;
    }
}

// ======================================================================== executor


constexpr uint32_t XRING = 8192;     // output ring (LDS)
constexpr uint32_t XRMASK = XRING - 1;
constexpr uint32_t XSLOT = 2048;     // flush granule
constexpr uint32_t XCHUNK = 1024;    // input bytes whose tokens are enumerated at once
constexpr uint32_t XSTAGE = XCHUNK + 64 + 16;

__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Batch-parallel executor step limits. A batch writes at most XPAR_OUT bytes into the ring, so
// with op - F < XSLOT at its start, a copy reaching back <= XNEAR still finds its source in the
// ring and any longer copy reads output flushed >= 2 KiB earlier.
constexpr uint32_t XPAR_OUT = 2048;
constexpr uint32_t XPAR_TOK = 64;
constexpr uint32_t XNEAR = XRING - XPAR_OUT;

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

// One batch-parallel executor step (all 64 lanes; lane t holds token t of the sub-batch: `take`,
// kind, output length ol, literal source position or copy offset, output position otok).
// Literals are independent and go first; copies then run in dependency rounds: a copy runs once
// no pending copy of the batch writes a byte it reads ([a, b); for offset < length only the
// first `off` bytes before it). Returns false on a copy reaching before the piece.
__device__ __forceinline__ bool par_step(uint8_t* ring, const uint8_t* stage, uint8_t* dst, uint32_t woff, uint32_t I,
                                         uint32_t out_start, uint32_t op, uint32_t& F, bool take, uint32_t kd,
                                         uint32_t ol, uint32_t srcv, uint32_t off, uint32_t otok, uint32_t btot,
                                         int lane) {
    wait_vmem();   // flushed output is visible to far copies
    if (take && kd == 0) {
        const uint32_t sb = woff + (srcv - I);
        for (uint32_t j = 0; j < ol; j++) ring[(otok + j) & XRMASK] = stage[sb + j];
    }
    __syncthreads();
    const bool cp = take && kd != 0;
    if (__any(cp && (off == 0 || off > otok - out_start))) return false;
    const uint32_t a = otok - off;
    const uint32_t b = a + min(ol, off);
    const uint32_t kb = lanes_below(take ? otok : 0xffffffffu, b);            // outputs starting before b
    const uint32_t ka = lanes_below(take ? otok + ol : 0xffffffffu, a + 1);  // outputs ending by a
    const uint64_t dep = (cp && kb > ka) ? (lane_mask_lt(kb) & ~lane_mask_lt(ka)) : 0ull;
    uint64_t pend = __ballot(cp);
    while (pend) {
        const bool ready = cp && ((pend >> lane) & 1ull) && (dep & pend) == 0ull;
        if (ready) {
            const bool near = off <= XNEAR;
            uint32_t r = 0;
            for (uint32_t j = 0; j < ol; j++) {
                const uint32_t s = a + r;
                const uint8_t v = near ? ring[s & XRMASK] : dst[s];   // far: flushed >= 2 KiB ago
                ring[(otok + j) & XRMASK] = v;
                r = r + 1 == off ? 0u : r + 1;
            }
        }
        pend &= ~__ballot(ready);
        __syncthreads();
    }
    const uint32_t upto = op + btot;
    while (upto - F >= XSLOT) {
        const uint32_t a0 = F + uint32_t(lane) * 32u;
        const uint4 v0 = *reinterpret_cast<const uint4*>(ring + (a0 & XRMASK));
        const uint4 v1 = *reinterpret_cast<const uint4*>(ring + ((a0 + 16u) & XRMASK));
        *reinterpret_cast<uint4*>(dst + a0) = v0;
        *reinterpret_cast<uint4*>(dst + a0 + 16) = v1;
        F += XSLOT;
    }
    return true;
}

__global__ __launch_bounds__(64) void k_snappy_exec(const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                                    const uint32_t* __restrict__ splits, int* __restrict__ fb, int mode) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[XRING];
    __shared__ __attribute__((aligned(16))) uint8_t stage[XSTAGE];
    __shared__ uint16_t tokpos[XCHUNK / 2];
    const int lane = threadIdx.x;
    int j, k;
    if (mode == 0) { const int2 pc = pieces[blockIdx.x]; j = pc.x; k = pc.y; }
    else { j = blockIdx.x; k = 0; }
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
    const uint16_t* tm16 = reinterpret_cast<const uint16_t*>(job.tokmap);
    uint32_t op = out_start, F = out_start;
#ifdef PF_SNAP_TRACE
    const bool tr = false;
    TRACE(0xAAAA0000u, uint32_t(k), ip, out_start, out_end);
#endif
    bool bad = false;
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
        uint32_t ex = cnt;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(ex, d, 64);
            if (lane >= d) ex += y;
        }
        const uint32_t T = __shfl(ex, 63, 64);
        uint32_t q = ex - cnt;
        while (bits) {
            const uint32_t b = uint32_t(__ffs(bits) - 1);
            bits &= bits - 1;
            tokpos[q++] = uint16_t(16u * uint32_t(lane) + b);
        }
        __syncthreads();
        if (T == 0) { bad = true; break; }
        bool stop = false;
        for (uint32_t sb = 0; sb < T && !stop && !bad; sb += 64) {
            const uint32_t t = sb + uint32_t(lane);
            const bool v = t < T;
            const uint32_t pos = v ? uint32_t(tokpos[t]) : 0u;
            const SnapTok tk = snap_tok(lds_read8(stage, woff + pos));
            const uint32_t ol = v ? tk.ol : 0u;
            const uint64_t start = uint64_t(I) + pos;
            const unsigned long long endp = start + tk.tl;
            const unsigned long long prev = __shfl_up(endp, 1, 64);
            uint32_t inc = ol;
            #pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d, 64);
                if (lane >= d) inc += y;
            }
            const uint32_t otok = op + inc - ol;
            const bool take = v && otok < out_end;
            const unsigned long long tb = __ballot(take);
            const int nt = __popcll(tb);
            const bool wrong = take && ((lane == 0 ? start != ip : start != prev) || endp > n || op + inc > out_end);
            if (__any(wrong)) { bad = true; break; }
            if (nt == 0) break;   // the previous sub-batch ended exactly at out_end
            if (uint32_t(nt) < min(T - sb, 64u)) stop = true;
            TRACE(0xBBBB0000u | uint32_t(k), I, ip, T, sb, uint32_t(nt), op, F);
            const uint32_t srcv = tk.kind == 0 ? uint32_t(start) + tk.arg : tk.arg;
            const uint32_t kd = tk.kind;
            const uint32_t btot = __builtin_amdgcn_readlane(inc, nt - 1);
            const bool lit = take && kd == 0;
            // Batch-parallel step: every token of the sub-batch at once, one lane per token. Taken
            // when the batch is short (no token > XPAR_TOK bytes, <= XPAR_OUT bytes in all) and
            // every literal is staged; otherwise the token-serial step below.
            const bool par = btot <= XPAR_OUT &&
                             !__any(take && (ol > XPAR_TOK ||
                                             (lit && uint64_t(srcv) + ol > uint64_t(I) + XCHUNK + 64)));
            if (par) {
                if (!par_step(ring, stage, dst, woff, I, out_start, op, F, take, kd, ol, srcv, tk.arg, otok, btot, lane)) {
                    bad = true;
                    break;
                }
            } else
            for (int i = 0; i < nt; i++) {
                const uint32_t k_i = __builtin_amdgcn_readlane(kd, i);
                const uint32_t l_i = __builtin_amdgcn_readlane(ol, i);
                const uint32_t s_i = __builtin_amdgcn_readlane(srcv, i);
                const uint32_t o_i = __builtin_amdgcn_readlane(otok, i);
                if (o_i + l_i + 64 >= out_end || o_i < out_start + 64) TRACE(0xCCCC0000u | (uint32_t(k) << 8) | k_i, l_i, s_i, o_i, F);
                if (k_i == 0) {
                    const bool staged = uint64_t(s_i) + l_i <= uint64_t(I) + XCHUNK + 64;
                    for (uint32_t d = 0; d < l_i; d += 1024) {
                        const uint32_t c = min(l_i - d, 1024u);
                        if (staged) {   // uniform: LDS -> LDS
                            const uint32_t sb0 = woff + (s_i - I) + d;
                            for (uint32_t qq = uint32_t(lane); qq < c; qq += 64)
                                ring[(o_i + d + qq) & XRMASK] = stage[sb0 + qq];
                        } else {        // long literal straight from HBM
                            const uint8_t* ib = in + s_i + d;
                            for (uint32_t qq = uint32_t(lane); qq < c; qq += 64)
                                ring[(o_i + d + qq) & XRMASK] = __builtin_nontemporal_load(ib + qq);
                        }
                        const uint32_t upto = o_i + d + c;
                        while (upto - F >= XSLOT) {
                            wait_vmem();   // earlier flushes have landed: far copies may read them
                            const uint32_t a0 = F + uint32_t(lane) * 32u;
                            const uint4 v0 = *reinterpret_cast<const uint4*>(ring + (a0 & XRMASK));
                            const uint4 v1 = *reinterpret_cast<const uint4*>(ring + ((a0 + 16u) & XRMASK));
                            *reinterpret_cast<uint4*>(dst + a0) = v0;
                            *reinterpret_cast<uint4*>(dst + a0 + 16) = v1;
                            F += XSLOT;
                        }
                    }
                } else {
                    if (s_i == 0 || s_i > o_i - out_start) { bad = true; break; }
                    uint32_t jj = uint32_t(lane);
                    if (s_i < l_i) jj = jj % s_i;            // overlapping copy repeats its pattern
                    const uint32_t sa = o_i - s_i + jj;
                    uint8_t byte = 0;
                    if (s_i <= XRING) {
                        if (uint32_t(lane) < l_i) byte = ring[sa & XRMASK];
                    } else {
                        if (uint32_t(lane) < l_i) byte = dst[sa];   // flushed: >= 6 KiB behind F
                    }
                    if (uint32_t(lane) < l_i) ring[(o_i + uint32_t(lane)) & XRMASK] = byte;
#ifdef PF_SNAP_SAFE
                    __syncthreads();
#endif
                    const uint32_t upto = o_i + l_i;
                    while (upto - F >= XSLOT) {
                        wait_vmem();
                        const uint32_t a0 = F + uint32_t(lane) * 32u;
                        const uint4 v0 = *reinterpret_cast<const uint4*>(ring + (a0 & XRMASK));
                        const uint4 v1 = *reinterpret_cast<const uint4*>(ring + ((a0 + 16u) & XRMASK));
                        *reinterpret_cast<uint4*>(dst + a0) = v0;
                        *reinterpret_cast<uint4*>(dst + a0 + 16) = v1;
                        F += XSLOT;
                    }
                }
            }
            if (bad) break;
#ifdef PF_SNAP_SAFE
            __syncthreads();
#endif
            op += __builtin_amdgcn_readlane(inc, nt - 1);
            ip = uint32_t(__shfl(endp, nt - 1, 64));
            if (op >= out_end) stop = true;
        }
    }
    if (bad) {
        if (lane == 0) atomicMax(&fb[j], whole ? FB_SERIAL : FB_REDO);
        return;
    }
    TRACE(0xDDDD0000u | uint32_t(k), op, F, ip, out_end);
    // tail: bytes [F, op)
    for (uint32_t a = F + uint32_t(lane) * 16u; a + 16u <= op; a += 1024u)
        *reinterpret_cast<uint4*>(dst + a) = *reinterpret_cast<const uint4*>(ring + (a & XRMASK));
    for (uint32_t a = F + ((op - F) & ~15u) + uint32_t(lane); a < op; a += 64) dst[a] = ring[a & XRMASK];
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

// All Snappy work of one batch, in stream order. fb must be zero on entry.
void launch_snappy(const SnappyJob* d_jobs, int n_jobs, const int2* d_wins, int n_wins, SnapWin* d_win,
                   uint32_t* d_lane_out, const int2* d_pieces, int n_pieces, uint32_t* d_splits, int* d_fb,
                   DevChunkResult* d_res, hipStream_t s) {
    if (n_jobs <= 0) return;
    hipLaunchKernelGGL(k_snappy_index, dim3(n_wins), dim3(64), 0, s, d_jobs, d_wins, d_win, d_lane_out, d_fb);
    hipLaunchKernelGGL(k_snappy_fix, dim3(n_jobs), dim3(64), 0, s, d_jobs, d_win, d_lane_out, d_splits, d_fb);
    hipLaunchKernelGGL(k_snappy_exec, dim3(n_pieces), dim3(64), 0, s, d_jobs, d_pieces, (const uint32_t*)d_splits, d_fb, 0);
    hipLaunchKernelGGL(k_snappy_exec, dim3(n_jobs), dim3(64), 0, s, d_jobs, d_pieces, (const uint32_t*)d_splits, d_fb, 1);
    launch_snappy_serial(d_jobs, n_jobs, d_fb, d_res, s);
}

}  // namespace pf
