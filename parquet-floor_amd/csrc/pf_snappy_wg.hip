// pf_snappy_wg.hip — K1 executor: one 1024-thread workgroup per 64 KiB Snappy piece.
//
// Replaces snappy-java's Snappy.uncompress for one output block of a page body
// (src/main/java/org/apache/hadoop/io/compress/DecompressorStream.java:101-173 hands the page to
// it). The parse kernels (pf_snappy_par.hip) have already marked every token start of the page
// (tokmap) and found the input position of the token at each 64 KiB output boundary (splits).
// Google Snappy never copies across a 64 KiB block, so a piece decodes on its own.
//
// The single-wave executor (k_snappy_exec2) walks a piece's tokens 64 at a time; a dense piece
// (~10 k tokens of sorted or small integers) takes ~0.8 ms that way. Here the whole piece is
// decoded at once by 16 waves with its 64 KiB output image in LDS:
//
//   1. tokens: every thread takes 32-bit words of the piece's token-start bitmap; a block scan
//      numbers the tokens and their output lengths, so each token's output start is known.
//      Each thread decodes the tokens of its word from a 64-byte LDS copy of that input.
//      The token ends are OR-ed into a second bitmap, which must equal the start bitmap
//      shifted by one token (the tokens tile the piece's input exactly) — else the page is
//      redone by the serial-order executor (FB_REDO), as k_snappy_exec2 does.
//   2. bytes, 4 KiB of output per batch, 4 bytes per thread: a byte's token comes from the
//      output-start bitmap (word prefix counts + popcount). A literal byte is loaded from the
//      input; a copy byte whose source lies before the batch is read from the LDS image; a copy
//      byte whose source lies inside the batch points at that byte. Pointer chains are
//      followed without barriers (every entry is always a valid ancestor or a terminal, and
//      threads compress the paths they walk), ending at a literal byte or a resolved value.
//   3. every batch is written to HBM with coalesced 4-byte stores as soon as it is final.
//
// Pieces the workgroup cannot hold (more than 16 Ki tokens, input or output spans over 64 KiB,
// pages in whole-page mode) are left to k_snappy_exec2 (pdone[piece] stays 0).
#include <hip/hip_runtime.h>

#include "pf_snappy_par.h"

namespace pf {

#ifdef PF_STAMPS
// diagnostics build: per-phase s_memtime cycle sums over the workgroups (thread 0's view, so a
// phase includes the barrier that waits for the slowest wave); [15] = pieces, [14] = max chase steps
__device__ unsigned long long pf_wstamps[16];
extern "C" int pf_debug_wstamps(unsigned long long* out, int n, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_wstamps), sizeof(unsigned long long) * (n < 16 ? n : 16)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pf_wstamps), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#define WT_DECL unsigned long long wt_ = __builtin_amdgcn_s_memtime()
#define WT(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (threadIdx.x == 0) atomicAdd(&pf_wstamps[i], t_ - wt_); wt_ = t_; } while (0)
#define WADD(i, v) atomicAdd(&pf_wstamps[i], (unsigned long long)(v))
#define WMAX(i, v) atomicMax(&pf_wstamps[i], (unsigned long long)(v))
#else
#define WT_DECL ((void)0)
#define WT(i) ((void)0)
#define WADD(i, v) ((void)0)
#define WMAX(i, v) ((void)0)
#endif

constexpr int XW_T = 1024;                    // threads per workgroup (16 waves)
constexpr int XW_WAVES = XW_T / 64;
constexpr uint32_t XW_OUT = 65536;            // output image (one Snappy block)
constexpr uint32_t XW_TCAP = 16384;           // tokens held per piece
constexpr uint32_t XW_S = 4 * XW_T;           // output bytes per resolution batch
constexpr uint32_t XW_OWORDS = XW_OUT / 32;   // output-start bitmap words
constexpr uint32_t XW_EWORDS = XW_OUT / 32 + 8;   // token-end bitmap (input span + word slack)
// resolution entries (u16): pointer (< XW_S) to a byte of the batch | T_VAL + value
constexpr uint32_t T_VAL = 0x8000u;

__device__ __forceinline__ uint32_t xw_dpp_scan(uint32_t v) {   // inclusive wave scan
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

// Barrier for LDS hand-offs only: global loads stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Exclusive block scan of two counters at once (all XW_T threads); totals returned.
__device__ __forceinline__ void xw_scan2(uint32_t a, uint32_t b, uint32_t* red, uint32_t& ea, uint32_t& eb, uint32_t& ta,
                                         uint32_t& tb) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t ia = xw_dpp_scan(a), ib = xw_dpp_scan(b);
    if (lane == 63) { red[wid] = ia; red[XW_WAVES + wid] = ib; }
    lds_barrier();
    uint32_t ba = 0, bb = 0, sa = 0, sb = 0;
    #pragma unroll
    for (int w = 0; w < XW_WAVES; w++) {
        const uint32_t va = red[w], vb = red[XW_WAVES + w];
        ba += w < wid ? va : 0u;
        bb += w < wid ? vb : 0u;
        sa += va;
        sb += vb;
    }
    lds_barrier();
    ea = ba + ia - a;
    eb = bb + ib - b;
    ta = sa;
    tb = sb;
}

// x mod d for 0 <= x < 64, 1 <= d <= 64.
__device__ __forceinline__ uint32_t xw_mod_small(uint32_t x, uint32_t d) {
    const uint32_t q = uint32_t((float(x) + 0.5f) * __builtin_amdgcn_rcpf(float(d)));
    return x - q * d;
}

struct XwLds {
    uint8_t val[XW_OUT];               // piece output image; per-thread input staging in step 1
    uint16_t o16[XW_TCAP];             // token output start (relative to the piece)
    uint16_t a16[XW_TCAP];             // copy offset, or literal data start relative to ip0
    uint32_t kbits[XW_TCAP / 32];      // 1 = literal
    uint32_t obits[XW_OWORDS];         // output-start bitmap
    uint16_t wpre[XW_OWORDS];          // tokens starting in earlier obits words
    union {
        uint16_t P[XW_S];              // resolution entries of the batch
        uint32_t ebits[XW_EWORDS];     // token-end bitmap (step 1), words relative to the first bitmap word
    } u;
    uint32_t red[2 * XW_WAVES];
};
static_assert(sizeof(XwLds) <= 163840, "LDS budget");

__global__ __launch_bounds__(XW_T) void k_snappy_exec_wg(const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                                        const uint32_t* __restrict__ splits, int* __restrict__ fb,
                                                        int* __restrict__ pdone) {
    __shared__ __attribute__((aligned(16))) XwLds S;
    const int tid = threadIdx.x;
    const int2 pc = pieces[blockIdx.x];
    const int j = pc.x, k = pc.y;
    if (fb[j] != FB_OK) return;   // whole-page / redo / serial pages: k_snappy_exec2 and the fallback
    const SnappyJob job = jobs[j];
    const uint8_t* in = job.src;
    const uint64_t n = job.src_len;
    const uint32_t* sp = splits + job.split_base;
    uint64_t pos0 = 0, ulen = 0;
    if (!uvarint(in, n, pos0, ulen) || ulen != job.dst_len) return;   // k_snappy_exec2 marks the page
    if (k > 0 && sp[k] == SNAP_INVALID) return;                      // an earlier piece covers it
    const uint32_t ip0 = k == 0 ? uint32_t(pos0) : sp[k];
    const uint32_t out_start = uint32_t(k) * SNAP_BLOCK;
    uint32_t out_end = job.dst_len, ip1 = uint32_t(n);
    for (uint32_t k2 = k + 1; k2 < job.n_pieces; k2++)
        if (sp[k2] != SNAP_INVALID) { out_end = k2 * SNAP_BLOCK; ip1 = sp[k2]; break; }
    const uint32_t span = out_end - out_start;
    if (span == 0 || span > XW_OUT || ip1 <= ip0 || ip1 - ip0 > XW_OUT - 1 || ip1 > n) return;

    WT_DECL;
    PF_GLOBAL uint8_t* gdst = gptr(job.dst) + out_start;
    const PF_GLOBAL uint8_t* gin = gptr(in);
    {   // a piece that is one literal (incompressible data, e.g. bit-packed dictionary ids): a copy
        const SnapTok t0 = snap_tok(glb_read8(in, n, ip0));
        if (t0.kind == 0 && t0.ol == span && uint64_t(ip0) + t0.tl == ip1) {
            const uint32_t s0 = ip0 + t0.arg;   // literal data [s0, s0 + span) of the input
            const uintptr_t base = reinterpret_cast<uintptr_t>(in) + s0;
            const uintptr_t last = base + span - 1;   // its last byte: an aligned dword holding it is readable
            const uint32_t sh = uint32_t(base & 3u);
            const PF_GLOBAL uint32_t* a0 = (const PF_GLOBAL uint32_t*)(base & ~uintptr_t(3));
            for (uint32_t d = uint32_t(tid); 4u * d < span; d += XW_T) {
                const uint32_t lo = a0[d];
                const uint32_t hi = sh && (base & ~uintptr_t(3)) + 4u * d + 4u <= last ? a0[d + 1] : 0u;
                const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);
                if (4u * d + 4u <= span) {
                    *(PF_GLOBAL uint32_t*)(gdst + 4u * d) = v;
                } else {
                    for (uint32_t i = 0; 4u * d + i < span; i++) gdst[4u * d + i] = uint8_t(v >> (8 * i));
                }
            }
            if (tid == 0) { pdone[blockIdx.x] = 1; WADD(9, 1); }
            return;
        }
    }
    // ---------------------------------------------------------------- 1. tokens
    const uint32_t w_lo = ip0 >> 5, w_hi = (ip1 - 1) >> 5;   // bitmap words of [ip0, ip1)
    const uint32_t nw = w_hi - w_lo + 1;                     // <= 2049: at most 3 words per thread
    const PF_GLOBAL uint32_t* tm = (const PF_GLOBAL uint32_t*)job.tokmap;
    for (uint32_t i = uint32_t(tid); i < XW_EWORDS; i += XW_T) S.u.ebits[i] = 0;
    for (uint32_t i = uint32_t(tid); i < XW_OWORDS; i += XW_T) S.obits[i] = 0;
    for (uint32_t i = uint32_t(tid); i < XW_TCAP / 32; i += XW_T) S.kbits[i] = 0;
    __syncthreads();
    uint8_t* const slot = S.val + 64 * tid;   // this thread's 64 bytes of staged input (val is free until step 2)
    uint32_t keep[3] = {0u, 0u, 0u};          // the masked start bits of this thread's words
    uint32_t tbase = 0, obase = 0;            // tokens / output bytes of earlier rounds
    bool bad = false, full = false;
    #pragma unroll
    for (int r = 0; r < 3; r++) {
        const uint32_t wi = uint32_t(r) * XW_T + uint32_t(tid);
        if (uint32_t(r) * XW_T >= nw) break;   // block-uniform
        const uint32_t w = w_lo + wi;
        const uint32_t b0 = 32u * w;
        uint32_t bits = 0, woff = 0;
        if (wi < nw) {
            // the word's start bits and input bytes [32 w, 32 w + 40) (+ alignment), loaded together;
            // 16-byte chunks wholly past the stream are never read (a chunk holding a valid byte does
            // not cross a page)
            const uintptr_t a = reinterpret_cast<uintptr_t>(in) + b0;
            woff = uint32_t(a & 15u);
            const PF_GLOBAL u32x4* src = (const PF_GLOBAL u32x4*)(a - woff);
            const int64_t first = int64_t(b0) - int64_t(woff);
            u32x4 v[4];
            #pragma unroll
            for (int c = 0; c < 4; c++) {
                v[c] = u32x4{0u, 0u, 0u, 0u};
                if (first + 16 * c < int64_t(n)) v[c] = src[c];
            }
            bits = tm[w];
            if (b0 < ip0) bits &= ~0u << (ip0 - b0);
            if (b0 + 32u > ip1) bits &= ip1 - b0 >= 32u ? ~0u : ((1u << (ip1 - b0)) - 1u);
            #pragma unroll
            for (int c = 0; c < 4; c++) reinterpret_cast<u32x4*>(slot)[c] = v[c];
        }
        keep[r] = bits;
        const uint32_t cnt = uint32_t(__popc(bits));
        uint32_t et, e2, tt, t2;
        xw_scan2(cnt, 0u, S.red, et, e2, tt, t2);
        if (tbase + tt > XW_TCAP) { full = true; break; }   // block-uniform
        // pass A: token records with output starts relative to the word; token ends into ebits
        uint32_t lo = 0;
        {
            uint32_t m = bits, t = tbase + et;
            while (m) {
                const uint32_t b = uint32_t(__ffs(m) - 1);
                m &= m - 1;
                const SnapTok tk = snap_tok(lds_read8(slot, woff + b));
                const uint64_t end = uint64_t(b0 + b) + tk.tl;
                if (end > ip1 || lo + tk.ol > XW_OUT) { bad = true; break; }
                const uint32_t e = uint32_t(end) - 32u * w_lo;   // < XW_EWORDS * 32
                atomicOr(&S.u.ebits[e >> 5], 1u << (e & 31u));
                const bool lit = tk.kind == 0;
                S.o16[t] = uint16_t(lo);
                S.a16[t] = uint16_t(lit ? b0 + b + tk.arg - ip0 : min(tk.arg, 0xffffu));
                if (lit) atomicOr(&S.kbits[t >> 5], 1u << (t & 31u));
                lo += tk.ol;
                t++;
            }
        }
        uint32_t eo, e3, to, t3;
        xw_scan2(lo, 0u, S.red, eo, e3, to, t3);
        // pass C: absolute output starts, copies must not reach before the piece
        if (!bad) {
            const uint32_t base = obase + eo;
            for (uint32_t t = tbase + et; t < tbase + et + cnt; t++) {
                const uint32_t o = uint32_t(S.o16[t]) + base;
                const bool lit = (S.kbits[t >> 5] >> (t & 31u)) & 1u;
                const uint32_t off = S.a16[t];
                if (o >= span || (!lit && (off == 0 || off > o))) { bad = true; break; }
                S.o16[t] = uint16_t(o);
                atomicOr(&S.obits[o >> 5], 1u << (o & 31u));
            }
        }
        tbase += tt;
        obase += to;
        if (obase > XW_OUT) break;   // block-uniform; corrupt
    }
    if (full) return;   // more tokens than the LDS tables hold: k_snappy_exec2
    WT(0);
    // checks: output total, and the tiling of [ip0, ip1): the end bitmap must be the start bitmap
    // without ip0, plus ip1 (nw + 1 words: ip1 may lie in the word after the last)
    {
        bool mis = bad || obase != span;
        #pragma unroll
        for (int r = 0; r < 3; r++) {
            const uint32_t wi = uint32_t(r) * XW_T + uint32_t(tid);
            if (wi > nw) break;
            const uint32_t b0 = 32u * (w_lo + wi);
            uint32_t sb = keep[r];
            const bool has0 = ip0 >= b0 && ip0 < b0 + 32u;
            if (has0 && !((sb >> (ip0 - b0)) & 1u)) mis = true;   // the first token starts at ip0
            if (has0) sb &= ~(1u << (ip0 - b0));
            if (ip1 >= b0 && ip1 < b0 + 32u) sb |= 1u << (ip1 - b0);
            if (S.u.ebits[wi] != sb) mis = true;
        }
        if (__syncthreads_or(mis)) {
            if (tid == 0) atomicMax(&fb[j], FB_REDO);
            return;
        }
    }
    WT(1);
    // word prefix counts of the output-start bitmap
    {
        const uint32_t w0 = 2u * uint32_t(tid);
        const uint32_t c0 = __popc(S.obits[w0]), c1 = __popc(S.obits[w0 + 1]);
        uint32_t e, e2, t1, t2;
        xw_scan2(c0 + c1, 0u, S.red, e, e2, t1, t2);
        S.wpre[w0] = uint16_t(e);
        S.wpre[w0 + 1] = uint16_t(e + c0);
    }
    __syncthreads();
    WT(2);

    // ---------------------------------------------------------------- 2. literal bytes
    // Thread tid owns output bytes [4 tid + 4096 g, +4) for g = 0..15 (the same bytes in step 3).
    // All literal bytes of the piece are loaded in two bursts of 32 loads per thread (one memory
    // latency each) and placed in the image; non-literal bytes are filled in step 3.
    const PF_GLOBAL uint8_t* gsrc = gin + ip0;
    #pragma unroll
    for (int h = 0; h < 2; h++) {
        uint32_t lb[32];
        #pragma unroll
        for (int g = 0; g < 8; g++) {
            const uint32_t x0 = 4u * uint32_t(tid) + XW_S * uint32_t(8 * h + g);
            const uint32_t xx0 = x0 < span ? x0 : 0u;
            const uint32_t wd = xx0 >> 5;
            const uint32_t ob = S.obits[wd], pre = S.wpre[wd];
            #pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t x = xx0 + uint32_t(i) < span ? xx0 + uint32_t(i) : xx0;
                const uint32_t t = pre + __popc(ob & ((2u << (x & 31u)) - 1u)) - 1u;
                const bool lit = (S.kbits[t >> 5] >> (t & 31u)) & 1u;
                const uint32_t srcoff = lit && x0 < span ? uint32_t(S.a16[t]) + (x - uint32_t(S.o16[t])) : 0u;
                lb[4 * g + i] = gsrc[srcoff];
            }
        }
        #pragma unroll
        for (int g = 0; g < 8; g++) {
            const uint32_t x0 = 4u * uint32_t(tid) + XW_S * uint32_t(8 * h + g);
            if (x0 < span)
                *reinterpret_cast<uint32_t*>(&S.val[x0]) =
                    lb[4 * g] | (lb[4 * g + 1] << 8) | (lb[4 * g + 2] << 16) | (lb[4 * g + 3] << 24);
        }
    }
    __syncthreads();
    WT(3);

    // ---------------------------------------------------------------- 3. copy bytes
    for (uint32_t b0 = 0; b0 < span; b0 += XW_S) {
        const uint32_t xr = 4u * uint32_t(tid);   // batch-relative position of this thread's first byte
        const uint32_t x0 = b0 + xr;
        uint32_t st[4];
        if (x0 < span) {
            const uint32_t wd = x0 >> 5;
            const uint32_t ob = S.obits[wd], pre = S.wpre[wd];
            const uint32_t cur = *reinterpret_cast<const uint32_t*>(&S.val[x0]);
            #pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t x = x0 + uint32_t(i) < span ? x0 + uint32_t(i) : x0;
                const uint32_t t = pre + __popc(ob & ((2u << (x & 31u)) - 1u)) - 1u;
                const bool lit = (S.kbits[t >> 5] >> (t & 31u)) & 1u;
                if (lit) {
                    st[i] = T_VAL | ((cur >> (8 * i)) & 0xffu);
                } else {
                    const uint32_t ot = S.o16[t], a = S.a16[t];
                    const uint32_t jj = x - ot;
                    const uint32_t m = a <= 64u ? xw_mod_small(jj & 63u, a) : jj;
                    const uint32_t y = ot - a + m;
                    st[i] = y < b0 ? (T_VAL | uint32_t(S.val[y])) : (y - b0);
                }
            }
            *reinterpret_cast<uint2*>(&S.u.P[xr]) = make_uint2(st[0] | (st[1] << 16), st[2] | (st[3] << 16));
        } else {
            #pragma unroll
            for (int i = 0; i < 4; i++) st[i] = T_VAL;
        }
        lds_barrier();
        WT(4);
        // follow pointer chains (entries only ever move to an ancestor or a terminal value; relaxed
        // workgroup-scope atomics keep every step an LDS access)
#ifdef PF_STAMPS
        uint32_t steps = 0;
#endif
        #pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t e = st[i];
            while (e < T_VAL) {
                e = __hip_atomic_load(&S.u.P[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(&S.u.P[xr + uint32_t(i)], uint16_t(e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef PF_STAMPS
                steps++;
#endif
            }
            st[i] = e;
        }
#ifdef PF_STAMPS
        if ((tid & 63) == 0) { WADD(13, steps); WMAX(14, steps); }
#endif
        const uint32_t v = (st[0] & 0xffu) | ((st[1] & 0xffu) << 8) | ((st[2] & 0xffu) << 16) | ((st[3] & 0xffu) << 24);
        if (x0 < span) {
            *reinterpret_cast<uint32_t*>(&S.val[x0]) = v;
            if (x0 + 4u <= span) {
                *(PF_GLOBAL uint32_t*)(gdst + x0) = v;
            } else {
                #pragma unroll
                for (int i = 0; i < 4; i++)
                    if (x0 + uint32_t(i) < span) gdst[x0 + uint32_t(i)] = uint8_t(v >> (8 * i));
            }
        }
        lds_barrier();
        WT(5);
        if (tid == 0) WADD(12, 1);
    }
    if (tid == 0) pdone[blockIdx.x] = 1;
    if (tid == 0) { WADD(15, 1); WADD(11, span); WADD(10, tbase); }
}

void launch_snappy_exec_wg(const SnappyJob* d_jobs, const int2* d_pieces, int n_pieces, const uint32_t* d_splits, int* d_fb,
                           int* d_pdone, hipStream_t s) {
    if (n_pieces <= 0) return;
    hipLaunchKernelGGL(k_snappy_exec_wg, dim3(n_pieces), dim3(XW_T), 0, s, d_jobs, d_pieces, d_splits, d_fb, d_pdone);
}

}  // namespace pf
