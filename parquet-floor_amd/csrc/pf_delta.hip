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

struct MiniBlock {
    uint64_t bitpos;     // absolute bit position of the miniblock's packed data
    int64_t min_delta;
    uint32_t first;      // index (within the page's value stream) of its first delta's value
    int32_t width;
};

__global__ __launch_bounds__(DNT) void k_delta(const DevChunk* __restrict__ chunks, DevPage* pages, const int* page_list,
                                               DevChunkResult* res) {
    __shared__ MiniBlock mb[MB_CAP];
    __shared__ int nmb, err, done;
    __shared__ uint64_t wpos, vpm_s, total_s, have_s, nmini_s;
    __shared__ uint64_t carry;
    __shared__ uint64_t wsum[DNT / 64];
    __shared__ int64_t cur_min;
    __shared__ int blk_left;     // miniblocks left in the current block
    __shared__ uint8_t widths[256];

    const int pi = page_list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (res[pg.chunk].status != 0) return;
    const bool is64 = ck.ptype == 2;
    // values section (v1 pages: after the levels)
    const uint8_t* p;
    uint64_t n;
    {
        if (pg.flags & PG_V2) { p = pg.body; n = pg.body_len; }
        else {
            uint64_t pos = 0; n = pg.body_len; p = pg.body;
            bool bad = false;
            for (int which = 0; which < 2; which++) {
                int maxl = which == 0 ? ck.max_rep : ck.max_def;
                if (maxl == 0) continue;
                int enc = which == 0 ? pg.rep_enc : pg.def_enc;
                uint64_t len;
                if (enc == 3) { if (pos + 4 > n) { bad = true; break; } len = ld32le(p, pos, n); pos += 4; }
                else if (enc == 4) len = (uint64_t(pg.num_values) * bit_width(maxl) + 7) / 8;
                else { bad = true; break; }
                if (len > n - pos) { bad = true; break; }
                pos += len;
            }
            if (bad) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
            p += pos; n -= pos;
        }
    }
    uint64_t* out = reinterpret_cast<uint64_t*>(pg.aux);
    if (threadIdx.x == 0) {
        err = 0; done = 0;
        uint64_t pos = 0, block, nmini, total, zz;
        if (!uvarint(p, n, pos, block) || !uvarint(p, n, pos, nmini) || !uvarint(p, n, pos, total) ||
            !uvarint(p, n, pos, zz) || nmini == 0 || block == 0 || block % 128 || nmini > 256 ||
            (block / nmini) % 32 || total > uint64_t(pg.aux_cap)) {
            err = 1;
        } else {
            vpm_s = block / nmini; nmini_s = nmini; total_s = total;
            uint64_t first = uint64_t(unzigzag(zz));
            if (!is64) first = uint64_t(uint32_t(first));
            if (total > 0) out[0] = first;
            have_s = total > 0 ? 1 : 0;
            wpos = pos; blk_left = 0;
            carry = first;
        }
    }
    __syncthreads();
    if (err) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    const uint64_t vpm = vpm_s, total = total_s;
    while (true) {
        // ---- lane 0: collect up to MB_CAP miniblocks ----
        if (threadIdx.x == 0) {
            int k = 0;
            uint64_t have = have_s, pos = wpos;
            while (have < total && k < MB_CAP) {
                if (blk_left == 0) {
                    uint64_t mz;
                    if (!uvarint(p, n, pos, mz) || pos + nmini_s > n) { err = 1; break; }
                    int64_t md = unzigzag(mz);
                    if (!is64) md = int32_t(md);
                    cur_min = md;
                    for (uint64_t m = 0; m < nmini_s; m++) widths[m] = p[pos + m];
                    pos += nmini_s;
                    blk_left = int(nmini_s);
                }
                int w = widths[nmini_s - blk_left];
                if (w > (is64 ? 64 : 32)) { err = 1; break; }
                uint64_t nb = vpm * uint64_t(w) / 8;
                if (pos + nb > n) { err = 1; break; }
                mb[k].bitpos = pos * 8; mb[k].width = w; mb[k].min_delta = cur_min; mb[k].first = uint32_t(have);
                k++;
                pos += nb;
                blk_left--;
                have += vpm;
                if (have > total) have = total;
            }
            nmb = k; wpos = pos;
            if (have >= total) done = 1;
            // round boundary: values [have_s, have) are covered by these k miniblocks
            total_s = total;   // unchanged
            vpm_s = vpm;
            // stash the end in first_s slot-free variable
            wsum[0] = have;    // temp: end of this round (read below before reuse)
        }
        __syncthreads();
        if (err) break;
        const uint64_t r0 = have_s, r1 = wsum[0];
        const int nk = nmb;
        __syncthreads();
        // ---- all threads: deltas -> values, tile by tile with a carried prefix ----
        for (uint64_t t0 = r0; t0 < r1; t0 += DNT) {
            uint64_t i = t0 + threadIdx.x;
            uint64_t d = 0;
            if (i < r1) {
                uint64_t j = i - r0;                       // delta index within this round
                uint64_t m = j / vpm, q = j % vpm;
                if (m < uint64_t(nk)) {
                    const MiniBlock& b = mb[m];
                    d = uint64_t(b.min_delta) + bits_le64(p, n, b.bitpos - 0 + q * uint64_t(b.width) - 0, b.width);
                }
            }
            // inclusive scan of d across the workgroup
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            uint64_t x = d;
            #pragma unroll
            for (int s = 1; s < 64; s <<= 1) {
                uint64_t y = __shfl_up(x, s, 64);
                if (lane >= s) x += y;
            }
            __syncthreads();
            if (lane == 63) wsum[wid] = x;
            __syncthreads();
            uint64_t base = carry;
            for (int w2 = 0; w2 < wid; w2++) base += wsum[w2];
            uint64_t v = base + x;
            if (!is64) v = uint64_t(uint32_t(v));
            if (i < r1) out[i] = v;
            __syncthreads();
            if (threadIdx.x == DNT - 1 || (i + 1 == r1)) { if (i < r1 && i + 1 == min<uint64_t>(r1, t0 + DNT)) carry = v; }
            __syncthreads();
        }
        if (threadIdx.x == 0) { have_s = r1; }
        __syncthreads();
        if (done) break;
    }
    if (err && threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi);
}

void launch_delta(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                  hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_delta, dim3(n), dim3(DNT), 0, st, d_chunks, d_pages, d_list, d_res);
}

}  // namespace pf
