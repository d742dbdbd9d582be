// pf_snappy_par.hip — K1 (parallel path): Snappy page decompression split into independent
// 64 KiB blocks.
//
// Google Snappy (what snappy-java wraps) compresses its input in independent 64 KiB blocks:
// no copy reaches back across a block boundary, and a token starts exactly at every multiple of
// 65536 in the output. Decoding therefore runs as:
//   k_snappy_index : one wave per page larger than 64 KiB; wave-parallel speculative parse
//                    (pf_snappy_par.h) of the token stream that records, for each multiple of
//                    65536, the input position of the token starting there;
//   k_snappy_exec  : one wave per 64 KiB piece; parses its tokens the same way and executes them
//                    in dependency rounds out of a 32 KiB LDS ring, flushing finished bytes to
//                    HBM with 16-byte stores;
//   k_snappy_serial: (pf_snappy.hip) re-decodes, serially, any page whose stream breaks the
//                    block assumption or looks corrupt — so arbitrary valid Snappy streams still
//                    decode bit-exactly and corrupt ones get the precise error.
// Replaces snappy-java's Snappy.uncompress behind the Hadoop codec shim
// (src/main/java/org/apache/hadoop/io/compress/DecompressorStream.java:61-70,101-173).
#include <hip/hip_runtime.h>

#include "pf_snappy_par.h"

namespace pf {

constexpr uint32_t BLOCK = 65536;
constexpr uint32_t PRING = 32768;
constexpr uint32_t PRMASK = PRING - 1;
constexpr uint32_t FAR = PRING - 4160;       // offsets beyond this read the flushed HBM output
constexpr uint32_t FLUSH_LAG = 8192;
constexpr int REC_CAP = 1152;
constexpr uint32_t LIT_PIECE = 64;
constexpr uint32_t LONG_LIT = 512;

struct SnapRec {
    uint32_t out;     // output position (page-absolute)
    uint32_t src;     // literal: input position; copy: offset
    uint32_t len;     // bit 31: literal
};

__device__ __forceinline__ bool preamble(const uint8_t* in, uint64_t n, uint64_t& pos, uint64_t& ulen) {
    pos = 0;
    return uvarint(in, n, pos, ulen);
}

// ---------------------------------------------------------------- k_snappy_index
__global__ __launch_bounds__(64) void k_snappy_index(const SnappyJob* __restrict__ jobs, const int* __restrict__ list,
                                                     uint32_t* splits, int* fallback) {
    __shared__ __attribute__((aligned(16))) uint8_t win[SNAP_WIN + SNAP_SLACK];
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
    while (pos < n) {
        __syncthreads();
        snap_load_window(win, job.src, n, pos);
        __syncthreads();
        SnapLane L;
        uint64_t exit = snap_parse_window(win, n - pos, L);
        // output bytes of this lane's tokens
        uint64_t lsum = 0;
        uint32_t v = L.valid;
        while (v) {
            int b = __ffs(v) - 1;
            v &= v - 1;
            lsum += snap_outlen(win, uint32_t(lane) * SNAP_SEG + b);
        }
        uint64_t x = lsum;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        uint64_t base = out + x - lsum;
        // boundaries k*BLOCK inside [base, base + lsum): find the token starting exactly there
        if (lsum && ((base + lsum - 1) / BLOCK != base / BLOCK || base % BLOCK == 0)) {
            uint64_t o = base;
            uint32_t v2 = L.valid;
            while (v2) {
                int b = __ffs(v2) - 1;
                v2 &= v2 - 1;
                if (o % BLOCK == 0 && o > 0 && o < ulen) {
                    uint64_t k = o / BLOCK;
                    if (k < job.n_pieces) sp[k] = uint32_t(pos + uint32_t(lane) * SNAP_SEG + b);
                }
                o += snap_outlen(win, uint32_t(lane) * SNAP_SEG + b);
            }
        }
        out += __shfl(x, 63, 64);
        pos += exit;
    }
    if (lane == 0 && (out != ulen || pos != n)) fallback[j] = 1;
}

// ---------------------------------------------------------------- k_snappy_exec
__device__ __forceinline__ void ring_flush(const uint8_t* ring, uint8_t* dst, uint32_t from, uint32_t to) {
    const int lane = threadIdx.x & 63;
    uint32_t head = min(to, (from + 15u) & ~15u);
    for (uint32_t q = from + lane; q < head; q += 64) dst[q] = ring[q & PRMASK];
    uint32_t body_end = head + ((to > head ? to - head : 0) & ~15u);
    for (uint32_t q = head + uint32_t(lane) * 16u; q < body_end; q += 64 * 16u) {
        uint32_t r = q & PRMASK;   // 16-aligned and the ring size is a multiple of 16: no wrap inside
        *reinterpret_cast<uint4*>(dst + q) = *reinterpret_cast<const uint4*>(ring + r);
    }
    for (uint32_t q = body_end + lane; q < to; q += 64) dst[q] = ring[q & PRMASK];
}

__global__ __launch_bounds__(64) void k_snappy_exec(const SnappyJob* __restrict__ jobs, const int2* __restrict__ pieces,
                                                    const uint32_t* __restrict__ splits, int* fallback) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[PRING];
    __shared__ __attribute__((aligned(16))) uint8_t win[SNAP_WIN + SNAP_SLACK];
    __shared__ SnapRec rec[REC_CAP];

    const int2 pc = pieces[blockIdx.x];
    const int j = pc.x, k = pc.y;
    const SnappyJob job = jobs[j];
    const int lane = threadIdx.x;
    const uint32_t* sp = splits + job.split_base;
    if (k > 0 && sp[k] == 0xffffffffu) return;          // merged into an earlier piece
    uint64_t p0, ulen;
    if (!preamble(job.src, job.src_len, p0, ulen) || ulen != job.dst_len) { if (lane == 0) fallback[j] = 1; return; }
    const uint8_t* in = job.src;
    const uint64_t n = job.src_len;
    uint8_t* dst = job.dst;
    uint64_t in_pos = k == 0 ? p0 : sp[k];
    const uint32_t out_start = uint32_t(k) * BLOCK;
    uint64_t in_end = n;
    uint32_t out_end = uint32_t(ulen);
    for (uint32_t k2 = k + 1; k2 < job.n_pieces; k2++)
        if (sp[k2] != 0xffffffffu) { in_end = sp[k2]; out_end = k2 * BLOCK; break; }
    if (in_pos > in_end || out_start > out_end) { if (lane == 0) fallback[j] = 1; return; }

    uint32_t op = out_start, flushed = out_start;
    bool bad = false;
    while (in_pos < in_end && !bad) {
        __syncthreads();
        snap_load_window(win, in, in_end, in_pos);
        __syncthreads();
        SnapLane L;
        const uint64_t limit = in_end - in_pos;
        uint64_t exit = snap_parse_window(win, limit, L);
        // records: one per copy, literals split into 64-byte pieces (>512 B: one LONG record)
        uint32_t cnt = 0;
        uint64_t osum = 0;
        {
            uint32_t v = L.valid;
            while (v) {
                int b = __ffs(v) - 1;
                v &= v - 1;
                uint32_t p = uint32_t(lane) * SNAP_SEG + b;
                uint64_t ol = snap_outlen(win, p);
                bool lit = (win[p] & 3) == 0;
                cnt += (lit && ol <= LONG_LIT) ? uint32_t((ol + LIT_PIECE - 1) / LIT_PIECE) : 1u;
                osum += ol;
            }
        }
        uint32_t xc = cnt;
        uint64_t xo = osum;
        #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t yc = __shfl_up(xc, d, 64);
            uint64_t yo = __shfl_up(xo, d, 64);
            if (lane >= d) { xc += yc; xo += yo; }
        }
        const uint32_t total_rec = __shfl(xc, 63, 64);
        const uint64_t total_out = __shfl(xo, 63, 64);
        if (total_rec > REC_CAP || uint64_t(op) + total_out > out_end) { bad = true; break; }
        {
            uint32_t ri = xc - cnt;
            uint64_t o = uint64_t(op) + (xo - osum);
            uint32_t v = L.valid;
            while (v) {
                int b = __ffs(v) - 1;
                v &= v - 1;
                uint32_t p = uint32_t(lane) * SNAP_SEG + b;
                uint32_t tag = win[p];
                uint64_t ol = snap_outlen(win, p);
                uint64_t ip = in_pos + p;
                if ((tag & 3) == 0) {
                    uint32_t hdr = (tag >> 2) < 60 ? 1u : 1u + ((tag >> 2) - 59);
                    uint64_t s = ip + hdr;
                    if (s + ol > in_end) bad = true;
                    if (ol > LONG_LIT) {
                        rec[ri++] = SnapRec{uint32_t(o), uint32_t(s), uint32_t(ol) | 0x80000000u};
                    } else {
                        for (uint64_t q = 0; q < ol; q += LIT_PIECE)
                            rec[ri++] = SnapRec{uint32_t(o + q), uint32_t(s + q),
                                                uint32_t(min<uint64_t>(LIT_PIECE, ol - q)) | 0x80000000u};
                    }
                } else {
                    uint32_t off;
                    if ((tag & 3) == 1) off = ((tag >> 5) << 8) | win[p + 1];
                    else if ((tag & 3) == 2) off = uint32_t(win[p + 1]) | uint32_t(win[p + 2]) << 8;
                    else off = uint32_t(win[p + 1]) | uint32_t(win[p + 2]) << 8 | uint32_t(win[p + 3]) << 16 |
                               uint32_t(win[p + 4]) << 24;
                    if (off == 0 || off > o - out_start) bad = true;   // before the piece: not independent
                    rec[ri++] = SnapRec{uint32_t(o), off, uint32_t(ol)};
                }
                o += ol;
            }
        }
        if (__any(bad)) { bad = true; break; }
        __syncthreads();
        // ---- execute records in order: batches of 64, dependency rounds ----
        for (uint32_t b0 = 0; b0 < total_rec; b0 += 64) {
            const uint32_t ri = b0 + lane;
            const bool has = ri < total_rec;
            SnapRec r = has ? rec[ri] : SnapRec{0, 0, 0};
            const bool lit = r.len & 0x80000000u;
            const uint32_t len = r.len & 0x7fffffffu;
            const bool longlit = has && lit && len > LONG_LIT;
            // LONG literals: finish the records before them, flush, copy straight to HBM
            unsigned long long longs = __ballot(longlit);
            unsigned long long pending = __ballot(has);
            // process lanes in segments separated by LONG records
            while (pending) {
                int first_long = longs ? __ffsll(longs) - 1 : 64;
                unsigned long long seg = first_long >= 64 ? pending : (pending & ((1ull << first_long) - 1));
                // ring capacity / flush: bytes of this segment must fit after the unflushed lag
                if (seg) {
                    int last = 63 - __clzll(seg);
                    uint32_t seg_end = __shfl(r.out + len, last, 64);
                    uint32_t seg_start = __shfl(r.out, __ffsll(seg) - 1, 64);
                    if (seg_start - flushed > FLUSH_LAG || seg_end - flushed > PRING) {
                        __syncthreads();
                        ring_flush(ring, dst, flushed, seg_start);
                        flushed = seg_start;
                        __syncthreads();
                    }
                }
                while (seg) {
                    const int fpl = __ffsll(seg) - 1;
                    const uint32_t fp = __shfl(r.out, fpl, 64);
                    const bool mine = (seg >> lane) & 1ull;
                    bool ready = false;
                    if (mine) ready = lit || (r.out - r.src + min(len, r.src) <= fp);
                    unsigned long long rdy = __ballot(ready) & seg;
                    if (ready) {
                        if (lit) {
                            const uint32_t wb = uint32_t(r.src - in_pos);
                            if (r.src >= in_pos && wb + len <= uint32_t(SNAP_WIN + SNAP_SLACK)) {
                                for (uint32_t q = 0; q < len; q++) ring[(r.out + q) & PRMASK] = win[wb + q];
                            } else {
                                for (uint32_t q = 0; q < len; q++) ring[(r.out + q) & PRMASK] = in[r.src + q];
                            }
                        } else {
                            const uint32_t off = r.src;
                            const uint32_t s0 = r.out - off;
                            uint32_t jj = 0;
                            if (off <= FAR) {
                                for (uint32_t q = 0; q < len; q++) {
                                    ring[(r.out + q) & PRMASK] = ring[(s0 + jj) & PRMASK];
                                    if (++jj == off) jj = 0;
                                }
                            } else {
                                for (uint32_t q = 0; q < len; q++) {
                                    ring[(r.out + q) & PRMASK] = dst[s0 + jj];
                                    if (++jj == off) jj = 0;
                                }
                            }
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    seg &= ~rdy;
                    pending &= ~rdy;
                }
                if (first_long < 64) {
                    // everything before the LONG literal is in the ring: flush it, copy the literal
                    const uint32_t lo = __shfl(r.out, first_long, 64);
                    const uint32_t ls = __shfl(r.src, first_long, 64);
                    const uint32_t ll = __shfl(len, first_long, 64);
                    __syncthreads();
                    ring_flush(ring, dst, flushed, lo);
                    for (uint32_t q = lane; q < ll; q += 64) dst[lo + q] = in[ls + q];
                    // keep the literal's tail in the ring for later copies
                    const uint32_t keep = min(ll, PRING);
                    for (uint32_t q = lane; q < keep; q += 64) {
                        uint32_t o2 = lo + ll - keep + q;
                        ring[o2 & PRMASK] = in[ls + ll - keep + q];
                    }
                    flushed = lo + ll;
                    __syncthreads();
                    pending &= ~(1ull << first_long);
                    longs &= ~(1ull << first_long);
                }
            }
        }
        op += uint32_t(total_out);
        in_pos += exit;
        if (op - flushed >= FLUSH_LAG) {
            __syncthreads();
            ring_flush(ring, dst, flushed, op);
            flushed = op;
        }
    }
    if (bad || op != out_end || in_pos != in_end) {
        if (lane == 0) fallback[j] = 1;
        return;
    }
    __syncthreads();
    ring_flush(ring, dst, flushed, op);
}

// ---------------------------------------------------------------- launcher
void launch_snappy_index(const SnappyJob* d_jobs, const int* d_index_list, int n_index, uint32_t* d_splits,
                         int* d_fallback, hipStream_t s) {
    if (n_index > 0) hipLaunchKernelGGL(k_snappy_index, dim3(n_index), dim3(64), 0, s, d_jobs, d_index_list, d_splits, d_fallback);
}
void launch_snappy_exec(const SnappyJob* d_jobs, const int2* d_pieces, int n_pieces, const uint32_t* d_splits,
                        int* d_fallback, hipStream_t s) {
    if (n_pieces > 0) hipLaunchKernelGGL(k_snappy_exec, dim3(n_pieces), dim3(64), 0, s, d_jobs, d_pieces, d_splits, d_fallback);
}

}  // namespace pf
