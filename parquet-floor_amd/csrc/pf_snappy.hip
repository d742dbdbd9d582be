// pf_snappy.hip — K1: Snappy page decompression on gfx950.
//
// Replaces snappy-java's Snappy.uncompress (JNI into Google Snappy), which parquet-mr reaches
// per page through the Hadoop codec shim (src/main/java/org/apache/hadoop/io/compress/
// DecompressorStream.java:61-70,101-173; CodecPool.java:6-8; ReflectionUtils.java:10-21).
//
// Raw Snappy: varint uncompressed length, then tags
//   00 literal  (len-1 in tag>>2; 60..63 -> 1..4 LE length bytes follow)
//   01 copy     (len 4..11 = 4 + (tag>>2 & 7), offset = (tag>>5)<<8 | next byte)
//   10 copy     (len (tag>>2)+1, 16-bit LE offset)
//   11 copy     (len (tag>>2)+1, 32-bit LE offset)
// Copies may overlap their own output (offset < length).
//
// Design (one 64-lane wave per page, no output staging):
//  * tokens are parsed in batches of 256 by lane 0 into LDS (4 KiB), then executed in order by
//    the wave directly in the HBM output: literals lane-parallel from the input, copies by 64
//    lanes at once (byte j of a copy reads position out - off + (j mod off), which always precedes
//    out, so a copy never reads its own bytes even when it overlaps itself);
//  * a workgroup barrier (release/acquire at workgroup scope) between tokens makes every lane's
//    stores visible to the next token's loads.
// This serial kernel is the FALLBACK: it only runs for pages the block-parallel path
// (pf_snappy_par.hip) could not decode (corrupt streams — it produces the precise error status).
// It is launched on every batch and nearly always finds nothing to do, so it holds almost no LDS:
// a launch that needs a large LDS allocation waits for CUs the other contexts' kernels occupy.
#include <hip/hip_runtime.h>

#include "pf_snappy_par.h"

namespace pf {

constexpr int TOK_BATCH = 256;

struct Token {
    uint32_t src;    // literal: input byte position; copy: offset
    uint32_t len;
    uint32_t out;    // output position
    uint32_t lit;
};

// One page, serially, by one wave (LDS passed in by the kernel).
__device__ void serial_page(const SnappyJob& job, DevChunkResult* res, Token* toks, int& ntok_s,
                            int& err_s, uint32_t& ip_s) {
    const uint8_t* in = job.src;
    const uint64_t n = job.src_len;
    uint8_t* dst = job.dst;
    const int lane = threadIdx.x;

    // preamble: uncompressed length
    uint64_t pos = 0, ulen = 0;
    bool ok = uvarint(in, n, pos, ulen) && ulen == job.dst_len;
    if (!ok) {
        if (lane == 0) set_status(res, job.chunk, ST_CORRUPT, job.page);
        return;
    }
    if (lane == 0) { ip_s = uint32_t(pos); err_s = 0; }
    __syncthreads();

    uint32_t op = 0;
    for (;;) {
        // ---- parse a batch of tokens (lane 0, serial) ----
        if (lane == 0) {
            uint64_t ip = ip_s;
            uint32_t o = op;
            int nt = 0, err = 0;
            while (nt < TOK_BATCH && ip < n) {
                uint32_t tag = in[ip++];
                Token t;
                t.out = o;
                if ((tag & 3) == 0) {
                    uint32_t len = tag >> 2;
                    if (len >= 60) {
                        uint32_t nb = len - 59;
                        if (ip + nb > n) { err = 1; break; }
                        len = 0;
                        for (uint32_t k = 0; k < nb; k++) len |= uint32_t(in[ip + k]) << (8 * k);
                        ip += nb;
                    }
                    uint64_t l64 = uint64_t(len) + 1;
                    if (ip + l64 > n || o + l64 > ulen) { err = 1; break; }
                    t.src = uint32_t(ip); t.len = uint32_t(l64); t.lit = 1;
                    ip += l64;
                } else {
                    uint32_t len, off;
                    if ((tag & 3) == 1) {
                        if (ip + 1 > n) { err = 1; break; }
                        len = 4 + ((tag >> 2) & 7);
                        off = ((tag >> 5) << 8) | in[ip];
                        ip += 1;
                    } else if ((tag & 3) == 2) {
                        if (ip + 2 > n) { err = 1; break; }
                        len = (tag >> 2) + 1;
                        off = uint32_t(in[ip]) | uint32_t(in[ip + 1]) << 8;
                        ip += 2;
                    } else {
                        if (ip + 4 > n) { err = 1; break; }
                        len = (tag >> 2) + 1;
                        off = ld32le(in, ip, n);
                        ip += 4;
                    }
                    if (off == 0 || off > o || uint64_t(o) + len > ulen) { err = 1; break; }
                    t.src = off; t.len = len; t.lit = 0;
                }
                o += t.len;
                toks[nt++] = t;
            }
            ntok_s = nt;
            ip_s = uint32_t(ip);
            err_s = err;
        }
        __syncthreads();
        const int nt = ntok_s;
        if (err_s) break;
        // ---- execute tokens in order, in the HBM output ----
        for (int i = 0; i < nt; i++) {
            const Token t = toks[i];
            if (t.lit) {
                for (uint32_t j = lane; j < t.len; j += WAVE) dst[t.out + j] = in[t.src + j];
            } else if (uint32_t(lane) < t.len) {
                dst[t.out + lane] = dst[t.out - t.src + (uint32_t(lane) % t.src)];
            }
            __syncthreads();   // this token's bytes are visible to the next token's reads
            op = t.out + t.len;
        }
        if (nt < TOK_BATCH) break;   // input exhausted
    }
    __syncthreads();
    if (err_s || op != ulen) {
        if (lane == 0) set_status(res, job.chunk, ST_CORRUPT, job.page);
        return;
    }
}



// Grid-stride over the jobs with a small grid: nearly every page was decoded by the parallel path.
constexpr int SERIAL_GRID = 64;

__global__ __launch_bounds__(64) void k_snappy_serial(const SnappyJob* __restrict__ jobs, const int* __restrict__ fallback,
                                                      int n_jobs, DevChunkResult* res) {
    __shared__ Token toks[TOK_BATCH];
    __shared__ int ntok_s, err_s;
    __shared__ uint32_t ip_s;
    for (int j = blockIdx.x; j < n_jobs; j += gridDim.x) {
        if (fallback[j] != FB_SERIAL) continue;   // the block-parallel path decoded this page
        const SnappyJob job = jobs[j];
        serial_page(job, res, toks, ntok_s, err_s, ip_s);
        __syncthreads();
    }
}

void launch_snappy_serial(const SnappyJob* d_jobs, int n_jobs, const int* d_fallback, DevChunkResult* d_res,
                          hipStream_t s) {
    if (n_jobs > 0)
        hipLaunchKernelGGL(k_snappy_serial, dim3(n_jobs < SERIAL_GRID ? n_jobs : SERIAL_GRID), dim3(64), 0, s, d_jobs,
                           d_fallback, n_jobs, d_res);
}

}  // namespace pf
