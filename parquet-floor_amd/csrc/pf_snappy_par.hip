// pf_snappy_par.hip — K1 (parallel path): Snappy page decompression split into independent
// 64 KiB blocks.
//
// Google Snappy (what snappy-java wraps) compresses its input in independent 64 KiB blocks:
// no copy reaches back across a block boundary, and a token starts exactly at every multiple of
// 65536 in the output. Decoding therefore runs as:
//   k_snappy_index : one wave per page larger than 64 KiB; wave-parallel speculative parse
//                    (pf_snappy_par.h) of the token stream that records, for each multiple of
//                    65536, the input position of the token starting there;
//   k_snappy_exec  : one 256-thread workgroup per 64 KiB piece. Per window (<= 2 KiB of input,
//                    <= 8 KiB of output): wave 0 parses and emits token records; all threads
//                    give every output byte a source pointer (an input byte, or an earlier output
//                    byte: position - offset, taken modulo the offset inside overlapping copies);
//                    pointer jumping through the window's pointers resolves copy-of-copy chains
//                    in log(depth) rounds; finally every byte is gathered from its root (the
//                    staged input, or already-final HBM output) and stored. Literals longer than
//                    1 KiB end a window and are copied straight to HBM;
//   k_snappy_serial: (pf_snappy.hip) re-decodes, serially, any page whose stream breaks the
//                    block assumption or looks corrupt — so arbitrary valid Snappy streams still
//                    decode bit-exactly and corrupt ones get the precise error.
// Replaces snappy-java's Snappy.uncompress behind the Hadoop codec shim
// (src/main/java/org/apache/hadoop/io/compress/DecompressorStream.java:61-70,101-173).
#include <hip/hip_runtime.h>

// Diagnostic build only (make stamps): per-phase s_memtime cycle sums, never in the product .so.
#ifdef PF_STAMPS
__device__ unsigned long long pf_stamps[16];
#define PF_STAMPS_COUNT pf_stamps
#endif

#include "pf_snappy_par.h"

namespace pf {

#ifdef PF_STAMPS
#define STAMP_DECL unsigned long long t_prev_ = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                                   \
    do {                                                                           \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                      \
        if (threadIdx.x == 0) atomicAdd(&pf_stamps[i], t_ - t_prev_);              \
        t_prev_ = t_;                                                              \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i)
#endif

constexpr uint32_t BLOCK = 65536;
constexpr int XNT = 256;                     // threads of the executor workgroup
constexpr uint32_t WOUT = 8192;              // output bytes (pointer slots) per window
constexpr int PER_T = int(WOUT) / XNT;       // pointer slots per thread (strided by XNT)
constexpr uint32_t BIGLIT = 1024;            // longer literals end a window, copied straight to HBM
constexpr uint32_t LPIECE = 64;              // literal records are split into <= 64-byte pieces
constexpr int REC_CAP = 64 * 16 + int(WOUT / LPIECE) + 64;
constexpr uint32_t INPUT = 0x80000000u;      // pointer tag: input byte position

struct SnapRec {
    uint32_t out;     // output position (page-absolute)
    uint32_t src;     // literal: input position; copy: offset
    uint32_t len;     // bit 31: literal
};

__device__ __forceinline__ bool preamble(const uint8_t* in, uint64_t n, uint64_t& pos, uint64_t& ulen) {
    pos = 0;
    return uvarint(in, n, pos, ulen);
}

__device__ __forceinline__ uint32_t sbyte(const SnapSeg& S, int b) { return (S.w[b >> 2] >> (8 * (b & 3))) & 0xffu; }

// Exact output length of the token at segment position b (static b), from registers.
__device__ __forceinline__ uint32_t seg_outlen(const SnapSeg& S, int b) {
    if (pk(S.tl, b) != 255u) return pk(S.ol, b);
    const uint32_t nb = (sbyte(S, b) >> 2) - 59u;
    uint32_t v = sbyte(S, b + 1);
    if (nb > 1) v |= sbyte(S, b + 2) << 8;
    if (nb > 2) v |= sbyte(S, b + 3) << 16;
    if (nb > 3) v |= sbyte(S, b + 4) << 24;
    return v + 1u;
}

// ---------------------------------------------------------------- k_snappy_index
__global__ __launch_bounds__(64) void k_snappy_index(const SnappyJob* __restrict__ jobs, const int* __restrict__ list,
                                                     uint32_t* splits, int* fallback) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SNAP_STAGE];
    const int j = list[blockIdx.x];
    const SnappyJob job = jobs[j];
    const int lane = threadIdx.x;
    uint64_t pos, ulen;
    if (!preamble(job.src, job.src_len, pos, ulen) || ulen != job.dst_len) {
        if (lane == 0) fallback[j] = 1;
        return;
    }
    uint32_t* sp = splits + job.split_base;
    uint64_t out = 0;
    const uint64_t n = job.src_len;
    STAMP_DECL
    while (pos < n) {
        __syncthreads();
        const uint32_t woff = snap_stage_window(stage, job.src, n, pos, lane, 64);
        __syncthreads();
        STAMP(5);
        SnapLane L;
        SnapSeg S;
        const uint32_t exit = snap_parse_window(stage, woff, n - pos, L, S);
        STAMP(6);
        if (job.tokmap && L.valid) {   // publish token starts for the executor
            const uint64_t gp = pos + uint64_t(lane) * SNAP_SEG;
            const uint32_t sh = uint32_t(gp & 31u);
            atomicOr(job.tokmap + (gp >> 5), L.valid << sh);
            if (sh) atomicOr(job.tokmap + (gp >> 5) + 1, L.valid >> (32u - sh));
        }
        uint64_t lsum = 0;
        #pragma unroll
        for (int b = 0; b < 32; b++)
            if ((L.valid >> b) & 1u) lsum += seg_outlen(S, b);
        uint64_t x = lsum;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        const uint64_t base = out + x - lsum;
        if (lsum && ((base + lsum - 1) / BLOCK != base / BLOCK || base % BLOCK == 0)) {
            uint64_t o = base;
            #pragma unroll
            for (int b = 0; b < 32; b++) {
                if ((L.valid >> b) & 1u) {
                    if (o % BLOCK == 0 && o > 0 && o < ulen) {
                        const uint64_t k = o / BLOCK;
                        if (k < job.n_pieces) sp[k] = uint32_t(pos + uint32_t(lane) * SNAP_SEG + uint32_t(b));
                    }
                    o += seg_outlen(S, b);
                }
            }
        }
        out += __shfl(x, 63, 64);
        if (exit == SNAP_FAR) { pos = n + 1; break; }
        pos += exit;
        STAMP(7);
    }
    if (lane == 0 && (out != ulen || pos != n)) fallback[j] = 1;
}

// ---------------------------------------------------------------- k_snappy_exec
__global__ __launch_bounds__(XNT) void k_snappy_exec(const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                                     const uint32_t* __restrict__ splits, int* fallback) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SNAP_STAGE];
    __shared__ uint32_t P[WOUT];
    __shared__ SnapRec rec[REC_CAP];
    __shared__ uint32_t s_nrec, s_wout, s_exit, s_bad, s_big_out, s_big_src, s_big_len;

    const int2 pc = pieces[blockIdx.x];
    const int j = pc.x, k = pc.y;
    const SnappyJob job = jobs[j];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t* sp = splits + job.split_base;
    if (k > 0 && sp[k] == 0xffffffffu) return;          // merged into an earlier piece
    uint64_t p0, ulen;
    if (!preamble(job.src, job.src_len, p0, ulen) || ulen != job.dst_len) { if (tid == 0) fallback[j] = 1; return; }
    const uint8_t* in = job.src;
    uint8_t* dst = job.dst;
    uint64_t in_pos = k == 0 ? p0 : sp[k];
    const uint32_t out_start = uint32_t(k) * BLOCK;
    uint64_t in_end = job.src_len;
    uint32_t out_end = uint32_t(ulen);
    for (uint32_t k2 = k + 1; k2 < job.n_pieces; k2++)
        if (sp[k2] != 0xffffffffu) { in_end = sp[k2]; out_end = k2 * BLOCK; break; }
    if (in_pos > in_end || out_start > out_end) { if (tid == 0) fallback[j] = 1; return; }

    uint32_t op = out_start;
    bool bad = false;
    STAMP_DECL
    while (in_pos < in_end) {
        __syncthreads();
        const uint32_t woff = snap_stage_window(stage, in, in_end, in_pos, tid, XNT);
        __syncthreads();
        STAMP(0);
        const uint32_t wbase = op;
        // ---------------- wave 0: parse + records (all from registers) ----------------
        if (wid == 0) {
            SnapLane L;
            SnapSeg S;
            if (job.tokmap) {
                // indexed page: token starts come from k_snappy_index's bitmap, no re-parse
                snap_seg_init(S, stage, woff, lane);
                const uint64_t limit = in_end - in_pos;
                const uint32_t ss = uint32_t(lane) * SNAP_SEG;
                const uint32_t lim = limit >= ss + 32 ? 32u : (limit <= ss ? 0u : uint32_t(limit - ss));
                const uint64_t gp = in_pos + ss;
                const uint32_t sh = uint32_t(gp & 31u);
                uint32_t m = job.tokmap[gp >> 5] >> sh;
                if (sh) m |= job.tokmap[(gp >> 5) + 1] << (32u - sh);
                m &= lim >= 32 ? 0xffffffffu : ((1u << lim) - 1u);
                uint32_t own = 0;
                #pragma unroll
                for (int b = 0; b < 32; b++) {
                    if ((m >> b) & 1u) {
                        uint32_t il = pk(S.tl, b);
                        if (il == 255u) { uint32_t olen; snap_long_literal(stage + woff, ss + uint32_t(b), il, olen); }
                        own = il == SNAP_FAR ? SNAP_FAR : ss + uint32_t(b) + il;
                    }
                }
                #pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(own, d, 64);
                    if (lane >= d) own = max(own, y);
                }
                L.valid = m;
                L.committed = 1;
                L.exit = own;
            } else {
                (void)snap_parse_window(stage, woff, in_end - in_pos, L, S);
            }
            uint32_t osum = 0, cnt = 0, bigl = 0;
            #pragma unroll
            for (int b = 0; b < 32; b++) {
                if ((L.valid >> b) & 1u) {
                    const uint32_t ol = seg_outlen(S, b);
                    const bool lit = (sbyte(S, b) & 3u) == 0;
                    if (lit && ol > BIGLIT) bigl = ol;
                    else { osum += ol; cnt += lit ? (ol + LPIECE - 1) / LPIECE : 1u; }
                }
            }
            uint32_t x = osum, xc = cnt;
            #pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64), yc = __shfl_up(xc, d, 64);
                if (lane >= d) { x += y; xc += yc; }
            }
            const unsigned long long comm = __ballot(L.committed);
            int f2 = 64 - __clzll(comm);
            const unsigned long long over = __ballot(L.committed && x > WOUT);
            if (over) f2 = min(f2, __ffsll(over) - 1);
            const unsigned long long big = __ballot(L.committed && bigl != 0);
            if (big) f2 = min(f2, __ffsll(big));              // include the big literal's lane
            bool lbad = false;
            if (lane < f2) {
                uint32_t o = wbase + x - osum;
                uint32_t ri = xc - cnt;
                const uint64_t lin = in_pos + uint32_t(lane) * SNAP_SEG;
                #pragma unroll
                for (int b = 0; b < 32; b++) {
                    if ((L.valid >> b) & 1u) {
                        const uint32_t tag = sbyte(S, b);
                        const uint32_t ol = seg_outlen(S, b);
                        if ((tag & 3u) == 0) {
                            const uint32_t hdr = (tag >> 2) < 60 ? 1u : 1u + ((tag >> 2) - 59u);
                            const uint64_t s = lin + uint32_t(b) + hdr;
                            if (s + ol > in_end) lbad = true;
                            if (ol > BIGLIT) {
                                s_big_out = o; s_big_src = uint32_t(s); s_big_len = ol;
                            } else {
                                for (uint32_t q = 0; q < ol; q += LPIECE)
                                    rec[ri++] = SnapRec{o + q, uint32_t(s + q), min(LPIECE, ol - q) | 0x80000000u};
                                o += ol;
                            }
                        } else {
                            uint32_t off;
                            if ((tag & 3u) == 1) off = ((tag >> 5) << 8) | sbyte(S, b + 1);
                            else if ((tag & 3u) == 2) off = sbyte(S, b + 1) | sbyte(S, b + 2) << 8;
                            else off = sbyte(S, b + 1) | sbyte(S, b + 2) << 8 | sbyte(S, b + 3) << 16 | sbyte(S, b + 4) << 24;
                            if (off == 0 || off > o - out_start) lbad = true;   // reaches before the piece
                            rec[ri++] = SnapRec{o, off, ol};
                            o += ol;
                        }
                    }
                }
            }
            const bool anybad = __any(lbad);
            const int src_lane = f2 > 0 ? f2 - 1 : 0;
            const uint32_t t_nrec = __shfl(xc, src_lane, 64);
            const uint32_t t_wout = __shfl(x, src_lane, 64);
            const uint32_t t_exit = __shfl(L.exit, src_lane, 64);
            if (lane == 0) {
                s_bad = (anybad || f2 <= 0) ? 1u : 0u;
                s_nrec = t_nrec;
                s_wout = t_wout;
                s_exit = t_exit;
                if (!(big && f2 == __ffsll(big))) s_big_len = 0;
            }
        }
        __syncthreads();
        STAMP(1);
        const uint32_t nrec = s_nrec, wout = s_wout, wexit = s_exit, blen = s_big_len;
        if (s_bad || uint64_t(wbase) + wout + blen > out_end || wexit == 0 || wexit == SNAP_FAR) { bad = true; break; }
        // ---------------- pointers: one slot per output byte ----------------
        for (uint32_t r = tid; r < nrec; r += XNT) {
            const SnapRec t = rec[r];
            const uint32_t len = t.len & 0x7fffffffu;
            uint32_t* pd = P + (t.out - wbase);
            if (t.len & 0x80000000u) {
                for (uint32_t q = 0; q < len; q++) pd[q] = INPUT | (t.src + q);
            } else if (t.src >= len) {
                const uint32_t s0 = t.out - t.src;
                for (uint32_t q = 0; q < len; q++) pd[q] = s0 + q;
            } else {
                const uint32_t s0 = t.out - t.src;
                uint32_t jj = 0;
                for (uint32_t q = 0; q < len; q++) {
                    pd[q] = s0 + jj;
                    jj = (jj + 1 == t.src) ? 0u : jj + 1;
                }
            }
        }
        __syncthreads();
        STAMP(2);
        // ---------------- pointer jumping (loads batched for ILP) ----------------
        for (;;) {
            int pending = 0;
            #pragma unroll
            for (int h = 0; h < PER_T; h += 16) {
                uint32_t v[16];
                #pragma unroll
                for (int i = 0; i < 16; i++) {
                    const uint32_t b = uint32_t(tid) + uint32_t(XNT) * uint32_t(h + i);
                    v[i] = b < wout ? P[b] : INPUT;
                }
                uint32_t u[16];
                #pragma unroll
                for (int i = 0; i < 16; i++) u[i] = (!(v[i] & INPUT) && v[i] >= wbase) ? P[v[i] - wbase] : v[i];
                #pragma unroll
                for (int i = 0; i < 16; i++) {
                    if (u[i] != v[i]) {
                        P[uint32_t(tid) + uint32_t(XNT) * uint32_t(h + i)] = u[i];
                        pending |= !(u[i] & INPUT) && u[i] >= wbase;
                    }
                }
            }
            if (!__syncthreads_or(pending)) break;
        }
        STAMP(3);
        // ---------------- gather + store (loads batched) ----------------
        const uint64_t stage_first = in_pos - woff;
        #pragma unroll
        for (int h = 0; h < PER_T; h += 16) {
            uint32_t v[16];
            #pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t b = uint32_t(tid) + uint32_t(XNT) * uint32_t(h + i);
                v[i] = b < wout ? P[b] : 0u;
            }
            uint8_t by[16];
            #pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t b = uint32_t(tid) + uint32_t(XNT) * uint32_t(h + i);
                by[i] = 0;
                if (b < wout) {
                    if (v[i] & INPUT) {
                        const uint64_t ip = v[i] & ~INPUT;
                        by[i] = (ip >= stage_first && ip < stage_first + SNAP_STAGE) ? stage[ip - stage_first] : in[ip];
                    } else {
                        by[i] = dst[v[i]];
                    }
                }
            }
            #pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t b = uint32_t(tid) + uint32_t(XNT) * uint32_t(h + i);
                if (b < wout) dst[wbase + b] = by[i];
            }
        }
        for (uint32_t q = tid; q < blen; q += XNT) dst[s_big_out + q] = in[s_big_src + q];
        STAMP(4);
        op = wbase + wout + blen;
        in_pos += wexit;
    }
    __syncthreads();
    if ((bad || op != out_end || in_pos != in_end) && tid == 0) fallback[j] = 1;
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

// ---------------------------------------------------------------- launchers
void launch_snappy_index(const SnappyJob* d_jobs, const int* d_index_list, int n_index, uint32_t* d_splits,
                         int* d_fallback, hipStream_t s) {
    if (n_index > 0) hipLaunchKernelGGL(k_snappy_index, dim3(n_index), dim3(64), 0, s, d_jobs, d_index_list, d_splits, d_fallback);
}
void launch_snappy_exec(const SnappyJob* d_jobs, const int2* d_pieces, int n_pieces, const uint32_t* d_splits,
                        int* d_fallback, hipStream_t s) {
    if (n_pieces > 0) hipLaunchKernelGGL(k_snappy_exec, dim3(n_pieces), dim3(XNT), 0, s, d_jobs, d_pieces, d_splits, d_fallback);
}

}  // namespace pf
