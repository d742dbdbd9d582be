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
constexpr int DVPT = 8;        // values per thread per tile

struct MiniBlock {
    uint64_t bitpos;     // absolute bit position of the miniblock's packed data
    int64_t min_delta;
    uint32_t first;      // index (within the page's value stream) of its first delta's value
    int32_t width;
};

struct DbpLds {
    MiniBlock mb[MB_CAP];
    int nmb, err, done;
    uint64_t wpos, vpm_s, total_s, have_s, nmini_s, rend;
    uint64_t carry;
    uint64_t wsum[DNT / 64];
    int64_t cur_min;
    int blk_left;        // miniblocks left in the current block
    uint8_t widths[256];
};

// Values section of a data page (v1: after the rep/def level sections).
__device__ bool values_section(const DevPage& pg, const DevChunk& ck, const uint8_t*& p, uint64_t& n) {
    if (pg.flags & PG_V2) { p = pg.body; n = pg.body_len; return true; }
    uint64_t pos = 0;
    n = pg.body_len; p = pg.body;
    for (int which = 0; which < 2; which++) {
        const int maxl = which == 0 ? ck.max_rep : ck.max_def;
        if (maxl == 0) continue;
        const int enc = which == 0 ? pg.rep_enc : pg.def_enc;
        uint64_t len;
        if (enc == 3) { if (pos + 4 > n) return false; len = ld32le(p, pos, n); pos += 4; }
        else if (enc == 4) len = (uint64_t(pg.num_values) * bit_width(maxl) + 7) / 8;
        else return false;
        if (len > n - pos) return false;
        pos += len;
    }
    p += pos; n -= pos;
    return true;
}

// Workgroup-wide DELTA_BINARY_PACKED decode of [p, p + n) (parquet-mr DeltaBinaryPackingValuesReader
// semantics): values v[0, min(total, cap)) -> out (64-bit; INT32 streams wrap mod 2^32). A
// miniblock is consumed whole while any value remains, so `end` (the byte after the last one read)
// is where a following section (DELTA_LENGTH_BYTE_ARRAY chars, DELTA_BYTE_ARRAY suffixes) starts.
// strict: total > cap is an error (INT pages); otherwise values past cap are parsed, not stored.
// Returns false on a malformed stream. All DNT threads must call.
__device__ bool dbp_decode_wg(DbpLds& S, const uint8_t* p, uint64_t n, bool is64, uint64_t* out, uint64_t cap,
                              bool strict, uint64_t& total_out, uint64_t& end_out) {
    if (threadIdx.x == 0) {
        S.err = 0; S.done = 0;
        uint64_t pos = 0, block, nmini, total, zz;
        if (!uvarint(p, n, pos, block) || !uvarint(p, n, pos, nmini) || !uvarint(p, n, pos, total) ||
            !uvarint(p, n, pos, zz) || nmini == 0 || block == 0 || block % nmini || nmini > 256 || nmini > block ||
            (block / nmini) % 8 || (strict && total > cap)) {   // parquet-mr: miniblock size a multiple of 8
            S.err = 1;
        } else {
            S.vpm_s = block / nmini; S.nmini_s = nmini; S.total_s = total;
            uint64_t first = uint64_t(unzigzag(zz));
            if (!is64) first = uint64_t(uint32_t(first));
            if (total > 0 && cap > 0) out[0] = first;
            S.have_s = total > 0 ? 1 : 0;
            S.wpos = pos; S.blk_left = 0;
            S.carry = first;
        }
    }
    __syncthreads();
    if (S.err) return false;
    const uint64_t vpm = S.vpm_s, total = S.total_s;
    while (true) {
        // ---- thread 0: collect up to MB_CAP miniblock headers ----
        if (threadIdx.x == 0) {
            int k = 0;
            uint64_t have = S.have_s, pos = S.wpos;
            while (have < total && k < MB_CAP) {
                if (S.blk_left == 0) {
                    uint64_t mz;
                    if (!uvarint(p, n, pos, mz) || pos + S.nmini_s > n) { S.err = 1; break; }
                    int64_t md = unzigzag(mz);
                    if (!is64) md = int32_t(md);
                    S.cur_min = md;
                    for (uint64_t m = 0; m < S.nmini_s; m++) S.widths[m] = p[pos + m];
                    pos += S.nmini_s;
                    S.blk_left = int(S.nmini_s);
                }
                const int w = S.widths[S.nmini_s - S.blk_left];
                if (w > (is64 ? 64 : 32)) { S.err = 1; break; }
                const uint64_t nb = vpm * uint64_t(w) / 8;
                if (pos + nb > n) { S.err = 1; break; }
                S.mb[k].bitpos = pos * 8; S.mb[k].width = w; S.mb[k].min_delta = S.cur_min; S.mb[k].first = uint32_t(have);
                k++;
                pos += nb;
                S.blk_left--;
                have += vpm;
                if (have > total) have = total;
            }
            S.nmb = k; S.wpos = pos;
            if (have >= total) S.done = 1;
            S.rend = have;   // values [have_s, have) are covered by these k miniblocks
        }
        __syncthreads();
        if (S.err) break;
        const uint64_t r0 = S.have_s, r1 = S.rend;
        const int nk = S.nmb;
        // ---- all threads: deltas -> values, tile by tile with a carried prefix; DVPT consecutive
        // values per thread (one workgroup scan per DNT * DVPT values) ----
        for (uint64_t t0 = r0; t0 < r1; t0 += uint64_t(DNT) * DVPT) {
            const uint64_t i0 = t0 + uint64_t(threadIdx.x) * DVPT;
            uint64_t d[DVPT];
            uint64_t tsum = 0;
            #pragma unroll
            for (int k = 0; k < DVPT; k++) {
                const uint64_t i = i0 + k;
                uint64_t dk = 0;
                if (i < r1) {
                    const uint64_t j = i - r0;                       // delta index within this round
                    const uint64_t m = j / vpm, q = j % vpm;
                    if (m < uint64_t(nk)) {
                        const MiniBlock& b = S.mb[m];
                        dk = uint64_t(b.min_delta) + bits_le64(p, n, b.bitpos + q * uint64_t(b.width), b.width);
                    }
                }
                tsum += dk;
                d[k] = tsum;                                         // inclusive within the thread
            }
            // exclusive scan of the thread sums across the workgroup
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            uint64_t x = tsum;
            #pragma unroll
            for (int sh = 1; sh < 64; sh <<= 1) {
                const uint64_t y = __shfl_up(x, sh, 64);
                if (lane >= sh) x += y;
            }
            if (lane == 63) S.wsum[wid] = x;
            __syncthreads();
            uint64_t base = S.carry, all = 0;
            for (int w2 = 0; w2 < DNT / 64; w2++) {
                const uint64_t ws = S.wsum[w2];
                if (w2 < wid) base += ws;
                all += ws;
            }
            base += x - tsum;
            #pragma unroll
            for (int k = 0; k < DVPT; k++) {
                const uint64_t i = i0 + k;
                uint64_t v = base + d[k];
                if (!is64) v = uint64_t(uint32_t(v));
                if (i < r1 && i < cap) out[i] = v;
            }
            __syncthreads();   // every thread read carry and wsum
            if (threadIdx.x == 0) S.carry = S.carry + all;
            __syncthreads();
        }
        if (threadIdx.x == 0) S.have_s = r1;
        __syncthreads();
        if (S.done) break;
    }
    total_out = total;
    end_out = S.wpos;
    const bool ok = !S.err;
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(DNT) void k_delta(const DevChunk* __restrict__ chunks, DevPage* pages, const int* page_list,
                                               DevChunkResult* res) {
    __shared__ DbpLds S;
    const int pi = page_list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    if (res[pg.chunk].status != 0) return;
    const uint8_t* p;
    uint64_t n, total, end;
    if (!values_section(pg, ck, p, n)) { if (threadIdx.x == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    if (!dbp_decode_wg(S, p, n, ck.ptype == 2, reinterpret_cast<uint64_t*>(pg.aux), uint64_t(pg.aux_cap), true, total,
                       end) && threadIdx.x == 0)
        set_status(res, pg.chunk, ST_CORRUPT, pi);
}

// ---- DELTA_LENGTH_BYTE_ARRAY (6) / DELTA_BYTE_ARRAY (7) BYTE_ARRAY pages -------------------------
// Replaces parquet-mr's DeltaLengthByteArrayValuesReader / DeltaByteArrayReader (behind
// ColumnReader.getBinary, src/main/java/blue/strategic/parquet/ParquetReader.java:151-157).
// k_dlen (before k_count), one workgroup per page: the length stream(s) -> pg.dx:
//   cpos[k] = chars of values [0, k) (u64, k <= T; saturates past 2^62 on a bad length),
//   lenA[k] = DLBA length / DBA prefix length, lenB[k] = DBA suffix length,
// dx_data = where the chars (DLBA) / suffixes (DBA) start in the values section, dx_bad = the
// first value that violates the oracle's checks (length < 0 as int32, prefix longer than the
// previous value, data past the section end). k_count then checks the page's present values
// against T and dx_bad and takes the page's chars from cpos. k_decode writes offsets and, for DLBA,
// the chars; k_dba_chars materialises DELTA_BYTE_ARRAY values (prefix of the previous value +
// suffix) in value order.
constexpr uint64_t CPOS_BAD = 1ull << 62;

__global__ __launch_bounds__(DNT) void k_dlen(const DevChunk* __restrict__ chunks, DevPage* pages, const int* page_list,
                                              DevChunkResult* res) {
    __shared__ DbpLds S;
    __shared__ uint64_t wtot[DNT / 64];
    __shared__ uint64_t s_carry, s_carry_sfx;
    __shared__ uint32_t s_prevlen;
    const int pi = page_list[blockIdx.x];
    DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int tid = threadIdx.x;
    if (res[pg.chunk].status != 0) return;
    const bool dba = pg.encoding == 7;
    const uint8_t* p;
    uint64_t n;
    const uint64_t cap = uint64_t(pg.aux_cap);
    uint64_t* cpos = pg.dx;
    uint64_t* la = cpos + cap + 1;
    uint64_t* lb = la + cap;
    uint64_t t1 = 0, e1 = 0, t2 = 0, e2 = 0;
    bool ok = values_section(pg, ck, p, n);
    if (ok) ok = dbp_decode_wg(S, p, n, false, la, cap, false, t1, e1);
    if (ok && dba) ok = dbp_decode_wg(S, p + e1, n - e1, false, lb, cap, false, t2, e2);
    if (!ok) { if (tid == 0) set_status(res, pg.chunk, ST_CORRUPT, pi); return; }
    const uint64_t T = dba ? min(t1, t2) : t1;     // values both streams hold
    const uint64_t data = e1 + e2;                  // chars / suffixes start
    const uint64_t avail = n - data;
    const uint64_t m = min(T, cap);
    if (tid == 0) { s_carry = 0; s_carry_sfx = 0; s_prevlen = 0; pg.dx_bad = int64_t(m); }
    __syncthreads();
    // per-value checks + prefix sums of the value lengths (and of DBA suffix lengths)
    for (uint64_t t0 = 0; t0 < m; t0 += DNT) {
        const uint64_t k = t0 + uint64_t(tid);
        const bool in = k < m;
        const uint32_t a = in ? uint32_t(la[k]) : 0u, b = in && dba ? uint32_t(lb[k]) : 0u;
        bool bad = in && (int32_t(a) < 0 || int32_t(b) < 0);
        const uint64_t len = uint64_t(a) + uint64_t(b);
        const uint64_t sfx = dba ? b : a;           // bytes this value takes from the data section
        // inclusive scans (wave, then across waves)
        const int lane = tid & 63, wid = tid >> 6;
        uint64_t x = len, y = sfx;
        #pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            const uint64_t xu = __shfl_up(x, sh, 64), yu = __shfl_up(y, sh, 64);
            if (lane >= sh) { x += xu; y += yu; }
        }
        if (lane == 63) { wtot[wid] = x; S.wsum[wid] = y; }
        __syncthreads();
        uint64_t bx = s_carry, by = s_carry_sfx;
        for (int w2 = 0; w2 < wid; w2++) { bx += wtot[w2]; by += S.wsum[w2]; }
        const uint64_t cend = bx + x, send = by + y;   // after value k
        if (in) {
            if (send > avail) bad = true;
            if (dba) {   // prefix <= previous value's length
                const uint32_t prev = k == 0 ? 0u : (k == t0 ? s_prevlen : uint32_t(la[k - 1]) + uint32_t(lb[k - 1]));
                if (a > prev) bad = true;
            }
            cpos[k + 1] = min(cend, CPOS_BAD);
            if (k == 0) cpos[0] = 0;
        }
        if (bad) atomicMin(reinterpret_cast<unsigned long long*>(&pg.dx_bad), (unsigned long long)k);
        __syncthreads();
        if (in && (k + 1 == min(m, t0 + DNT))) { s_carry = cend; s_carry_sfx = send; s_prevlen = uint32_t(len); }
        __syncthreads();
    }
    if (tid == 0) {
        if (m == 0) cpos[0] = 0;
        pg.dx_total = int64_t(T);
        pg.dx_data = uint32_t(data);
    }
}

// One wave per DELTA_BYTE_ARRAY page, after k_scan: value k = the first prefix[k] bytes of value
// k-1 + its suffix, written at chars + char_start + cpos[k]. The previous value is kept in LDS
// (values longer than XV_CAP re-read it from the chars just written) and the suffix stream is
// staged through LDS in XS_WIN windows.
constexpr uint32_t XV_CAP = 4096;
constexpr uint32_t XS_WIN = 8192;

__global__ __launch_bounds__(64) void k_dba_chars(const DevChunk* __restrict__ chunks, DevPage* pages,
                                                  const int* page_list, DevChunkResult* res) {
    __shared__ __attribute__((aligned(16))) uint8_t vbuf[2][XV_CAP];
    __shared__ __attribute__((aligned(16))) uint8_t sw[XS_WIN];
    const int pi = page_list[blockIdx.x];
    const DevPage& pg = pages[pi];
    const DevChunk& ck = chunks[pg.chunk];
    const int lane = threadIdx.x;
    if (res[pg.chunk].status != 0 || !ck.chars || !pg.dx) return;
    const uint8_t* p;
    uint64_t n;
    if (!values_section(pg, ck, p, n)) return;   // k_dlen reported it
    const uint64_t nv = uint64_t(pg.n_values);
    const uint64_t cap = uint64_t(pg.aux_cap);
    const uint64_t* cpos = pg.dx;
    const uint64_t* la = cpos + cap + 1;
    const uint64_t* lb = la + cap;
    const uint8_t* sfx = p + pg.dx_data;
    const uint64_t sfx_n = n - pg.dx_data;
    uint8_t* out = ck.chars + pg.char_start;
    uint64_t sp = 0;            // suffix stream position
    uint64_t ws = 0, we = 0;    // staged window [ws, we)
    int cur = 0;
    uint32_t plen = 0;          // previous value's length
    for (uint64_t k = 0; k < nv; k++) {
        const uint32_t pl = uint32_t(la[k]), sl = uint32_t(lb[k]);
        const uint32_t len = pl + sl;
        uint8_t* o = out + cpos[k];
        const bool fits = len <= XV_CAP && plen <= XV_CAP;
        if (sl > 0 && (sp < ws || sp + sl > we)) {   // restage the suffix window at sp
            if (sl <= XS_WIN) {
                ws = sp;
                we = min<uint64_t>(sp + XS_WIN, sfx_n);
                for (uint64_t i = uint64_t(lane); i < we - ws; i += 64) sw[i] = sfx[ws + i];
                __syncthreads();
            }
        }
        const bool staged = sp >= ws && sp + sl <= we;
        if (!fits) __threadfence_block();            // previous value re-read from the chars just written
        const uint8_t* prev = vbuf[cur ^ 1];
        uint8_t* keep = vbuf[cur];
        for (uint32_t j = uint32_t(lane); j < len; j += 64) {
            uint8_t b;
            if (j < pl) b = fits ? prev[j] : out[cpos[k - 1] + j];
            else b = staged ? sw[sp - ws + (j - pl)] : sfx[sp + (j - pl)];
            o[j] = b;
            if (len <= XV_CAP) keep[j] = b;
        }
        __syncthreads();
        sp += sl;
        plen = len;
        cur ^= 1;
    }
}

void launch_delta(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                  hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_delta, dim3(n), dim3(DNT), 0, st, d_chunks, d_pages, d_list, d_res);
}
void launch_dlen(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                 hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_dlen, dim3(n), dim3(DNT), 0, st, d_chunks, d_pages, d_list, d_res);
}
void launch_dba_chars(const DevChunk* d_chunks, DevPage* d_pages, const int* d_list, int n, DevChunkResult* d_res,
                      hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_dba_chars, dim3(n), dim3(64), 0, st, d_chunks, d_pages, d_list, d_res);
}

}  // namespace pf
