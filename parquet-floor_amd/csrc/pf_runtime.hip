// pf_runtime.hip — context, batch planning and kernel orchestration behind include/pfloor.h.
//
// One pf_ctx per GPU (one HIP stream, growable HBM arenas, pinned staging). A decode batch is
// any set of column chunks (a row group's selected columns, or several row groups): the host
// turns the descriptors into flat DevChunk / DevPage / SnappyJob tables, uploads them in one
// copy, and enqueues
//   k_snappy -> k_ba (dictionaries) -> k_delta -> k_count -> k_ba (PLAIN pages) -> k_scan -> k_flat -> k_decode
// on the context stream. Nothing synchronises until pf_wait.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "pf_encode.h"
#include "pf_host.h"
#include "pf_snappy_par.h"
#include "pfloor.h"

namespace pf {
void launch_snappy(const SnappyJob*, int, const int2*, int, SnapWin*, SnapEnt*, uint32_t*, const int2*, int, uint32_t*,
                   int*, DevChunkResult*, int, int, hipStream_t);
void launch_snappy_parse(const SnappyJob*, int, const int2*, int, SnapWin*, SnapEnt*, uint32_t*, uint32_t*, int*, int,
                         hipStream_t);
void launch_snappy_exec(const SnappyJob*, int, const int2*, int, uint32_t*, int*, DevChunkResult*, int, hipStream_t);
void launch_ba(BaJob*, int, const int2*, int, DevChunkResult*, hipStream_t, bool);
void launch_snappy_head(SnappyJob*, int, DevPage*, const DevChunk*, int*, const DevChunkResult*, hipStream_t);
void launch_snappy_litcopy(const SnappyJob*, const int*, int, const int*, hipStream_t);
void launch_delta(const DevChunk*, DevPage*, const int*, int, int, DevChunkResult*, hipStream_t);
void launch_dlen(const DevChunk*, DevPage*, const int*, int, DevChunkResult*, hipStream_t);
void launch_dba_chars(const DevChunk*, DevPage*, const int*, int, DevChunkResult*, hipStream_t);
void launch_count(const DevChunk*, DevPage*, const int*, int, int, const int2*, int, DevChunkResult*, BaJob*, hipStream_t, int);
void launch_scan(DevChunk*, DevPage*, const int*, int, DevChunkResult*, uint8_t*, uint64_t, unsigned long long*, hipStream_t);
void launch_flat(const DevChunk*, DevPage*, const int*, int, int, int, int, int*, DevChunkResult*, hipStream_t, NullCaps, int);
void launch_lvl(const DevChunk*, DevPage*, const int*, int, DevChunkResult*, hipStream_t, bool, NullCaps);
void launch_runs(const DevChunk*, DevPage*, const int*, int, DevChunkResult*, hipStream_t);
void launch_decode(const DevChunk*, DevPage*, const int*, int, int, DevChunkResult*, hipStream_t, int);
void launch_nest_lvl(const DevChunk*, DevPage*, const int*, int, int, DevChunkResult*, hipStream_t, bool);
void launch_nest_count(const DevChunk*, DevPage*, const int*, int, const int2*, int, DevChunkResult*, hipStream_t);
void launch_nest_decode(const DevChunk*, DevPage*, const int2*, int, DevChunkResult*, hipStream_t);
void launch_page_scan(const ScanChunk*, int, pf_page_desc*, ScanCrc*, ScanResult*, hipStream_t);
void launch_page_crc(const ScanCrc*, const int*, int, ScanResult*, int32_t*, hipStream_t);
}  // namespace pf

using namespace pf;

namespace {

thread_local std::string g_err;

int fail(pf_ctx* ctx, int code, const std::string& msg);

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        size_t want = std::max<size_t>(n + n / 4, 1 << 20);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

struct HostBuf {
    void* p = nullptr;
    void* d = nullptr;   // the device's address of the pinned pages (kernels read / write them over PCIe)
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; d = nullptr; cap = 0; }
        size_t want = std::max<size_t>(n + n / 4, 1 << 16);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) {
            cap = want;
            if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) d = nullptr;
        }
        return e;
    }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; d = nullptr; cap = 0; }
};

// Copies between pinned host pages and device memory by a kernel on the decode stream: two ranges
// of 8-byte words, grid-stride. The batch's metadata upload and its results download were SDMA /
// blit copies on the stream (PF_ZC=0): config 1 0.41 -> 0.39 ms, the others unchanged.
// (An upload stream of its own, event-joined, made every config slower: SF1 3.13 -> 4.4 ms.)
__global__ __launch_bounds__(256) void k_copy_words(uint64_t* __restrict__ d0, const uint64_t* __restrict__ s0, uint32_t n0,
                                                    uint64_t* __restrict__ d1, const uint64_t* __restrict__ s1, uint32_t n1) {
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n0 + n1; i += stride) {
        if (i < n0) d0[i] = s0[i];
        else d1[i - n0] = s1[i - n0];
    }
}
static_assert(sizeof(DevChunkResult) % 8 == 0 && sizeof(DevChunk) % 8 == 0, "k_copy_words moves 8-byte words");
// The batch's metadata upload (pinned host words -> device) and the zeroing of its validity arena and
// window hand-over words in one launch (round 5: two hipMemsetAsync fills were two more dependent
// launches at the head of every batch's chain). z0 / z1: 8-byte aligned, nz0 / nz1 bytes.
__global__ __launch_bounds__(256) void k_upload(uint64_t* __restrict__ d, const uint64_t* __restrict__ s, uint32_t n,
                                                uint8_t* __restrict__ z0, uint32_t nz0, uint8_t* __restrict__ z1, uint32_t nz1) {
    const uint32_t stride = gridDim.x * 256u;
    const uint32_t w0 = (nz0 + 7u) / 8u, w1 = (nz1 + 7u) / 8u;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n + w0 + w1; i += stride) {
        if (i < n) { d[i] = s[i]; continue; }
        const bool first = i < n + w0;
        uint8_t* z = first ? z0 : z1;
        const uint32_t w = first ? i - n : i - n - w0, nz = first ? nz0 : nz1;
        if (8u * w + 8u <= nz) reinterpret_cast<uint64_t*>(z)[w] = 0;
        else for (uint32_t b = 8u * w; b < nz; b++) z[b] = 0;
    }
}
inline void copy_words(void* d0, const void* s0, size_t b0, void* d1, const void* s1, size_t b1, hipStream_t st) {
    const uint32_t n0 = uint32_t(b0 / 8), n1 = uint32_t(b1 / 8);
    const uint32_t grid = std::max(1u, std::min(1024u, (n0 + n1 + 255u) / 256u));
    hipLaunchKernelGGL(k_copy_words, dim3(grid), dim3(256), 0, st, static_cast<uint64_t*>(d0), static_cast<const uint64_t*>(s0), n0,
                       static_cast<uint64_t*>(d1), static_cast<const uint64_t*>(s1), n1);
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// A decoded batch into pinned host memory by a kernel writing through the pages' device address
// (round 6): the SDMA engines move one direction at a time on this link -- an SDMA H2D and an SDMA D2H
// together make 57 GB/s, an SDMA H2D beside this kernel's D2H 86 GB/s (profiles/r06_e2e/duplex.txt) --
// so the next batch's H2D (pf_decode_row_group's SDMA copy) runs under this batch's download. Up to
// three ranges (the output arenas), 16-byte chunks grid-stride, the ranges' last < 16 bytes by block 0.
struct DlRange {
    uint8_t* d;
    const uint8_t* s;
    uint64_t n;
};
__global__ __launch_bounds__(256) void k_download(DlRange r0, DlRange r1, DlRange r2) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const uint64_t c0 = r0.n >> 4, c1 = r1.n >> 4, c2 = r2.n >> 4;
    const uint64_t stride = uint64_t(gridDim.x) * 256u;
    for (uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x; i < c0 + c1 + c2; i += stride) {
        const DlRange& r = i < c0 ? r0 : (i < c0 + c1 ? r1 : r2);
        const uint64_t j = i < c0 ? i : (i < c0 + c1 ? i - c0 : i - c0 - c1);
        reinterpret_cast<u4*>(r.d)[j] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(r.s) + j);
    }
    if (blockIdx.x == 0 && threadIdx.x < 48) {
        const DlRange& r = threadIdx.x < 16 ? r0 : (threadIdx.x < 32 ? r1 : r2);
        const uint64_t b = (r.n & ~uint64_t(15)) + (threadIdx.x & 15u);
        if (b < r.n) r.d[b] = r.s[b];
    }
}

constexpr int N_EVENTS = 11;  // h2d, snappy parse, snappy exec, dict, delta, levels, count, scan, flat, decode
constexpr uint32_t BA_TILE_BYTES = 8192;   // pf_pages.hip BA_TILE
constexpr int64_t FLAT_BLK = 4096;         // pf_pages.hip FBLK   // h2d, snappy, dict, delta, count, scan, flat, decode

}  // namespace

// The HIP stream(s) of a context. Shared by contexts made with pf_ctx_create_shared (the stream
// lives until the last of them is destroyed).
struct Streams {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t exec_stream = nullptr;
    // pf_copy_batch_async's downloads (made on first use): the next batch's H2D and kernels on `stream`
    // (a twin context's, with its own arenas) run while this batch's columns go to the host
    hipStream_t copy_stream = nullptr;
    std::mutex mu;
    ~Streams() {
        (void)hipSetDevice(device);
        if (copy_stream) { (void)hipStreamSynchronize(copy_stream); (void)hipStreamDestroy(copy_stream); }
        if (exec_stream) { (void)hipStreamSynchronize(exec_stream); (void)hipStreamDestroy(exec_stream); }
        if (stream) { (void)hipStreamSynchronize(stream); (void)hipStreamDestroy(stream); }
    }
};

struct pf_ctx {
    int device = 0;
    pf::PfOpts opts;                       // defaults; the diagnostics build reads PF_* at creation
    std::shared_ptr<Streams> streams;
    hipStream_t stream = nullptr;          // = streams->stream
    // PF_EXEC_STREAM=1: the Snappy executor runs on a low-priority stream of its own (event-ordered
    // with `stream`, which then gets the high priority), so the short kernels of another context
    // get CUs ahead of this context's executor waves as those retire.
    hipStream_t exec_stream = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    bool zc = true;                        // metadata / results copied by k_copy_words (PF_ZC=0: SDMA copies)
    hipEvent_t ev[N_EVENTS] = {};
    // recorded after the last operation of this context's decode: pf_wait waits for it, not for the
    // stream, so a context sharing the stream can have the next batch enqueued behind this one
    hipEvent_t ev_done = nullptr;
    // recorded after the last enqueued D2H copy of this context's outputs: pf_copy_column / pf_sync
    // wait for it, not for the stream, so a peer's decode queued behind the copies keeps running
    hipEvent_t ev_copy = nullptr;          // after this context's last async copy (on whichever stream)
    hipEvent_t ev_dl = nullptr;            // the decode a download on the copy stream follows
    bool timing = true;                    // per-stage events (pf_last_timing); pf_ctx_set_timing
    std::string err;
    DevBuf d_in, d_scratch, d_out, d_bits, d_chars, d_meta, d_tokmap;
    DevBuf d_scan_in, d_scan;              // pf_scan_pages: host chunk bytes, tables
    DevBuf d_enc, d_enc_sec, d_enc_out;    // pf_encode_chunk / pf_snappy_compress: work arena, values sections, slots
    std::vector<uint8_t> h_enc;            // the last encoded chunk (headers + bodies)
    HostBuf h_meta, h_res;
    HostBuf h_enc_slots;                   // pf_encode_chunk / pf_snappy_compress: compressed slots D2H
    // last batch
    int n_chunks = 0;
    bool pending = false;
    bool copies_pending = false;           // pf_copy_columns_async enqueued, not yet pf_sync'ed
    bool tables_from_decode = false;       // d_meta layout (off_fallback) belongs to a pf_decode_row_group
    bool timing_valid = false;
    std::vector<DevChunk> chunks;          // host copies (device pointers)
    std::vector<DevPage> pages;
    std::vector<SnappyJob> jobs;
    std::vector<int> l_dictbin, l_delta, l_count, l_scan, l_flat, l_decode, l_runs, l_dlen, l_dba, l_lvl, l_djobs, l_nest, l_nseg,
        l_cdict;   // l_cdict: (page, block) pairs of flat dictionary BYTE_ARRAY pages (k_count_dict)
    std::vector<int2> wins, pieces;       // Snappy index windows / 64 KiB pieces (job, index)
    std::vector<BaJob> bajobs;             // PLAIN BYTE_ARRAY walks: dictionary pages, then data pages
    std::vector<int2> ba_tiles;            // (job relative to its batch, tile)
    int n_ba_dict = 0, n_ba_dict_tiles = 0;
    bool ba_short_dict = true, ba_short_data = true;   // every walk job's values average <= BA_SHORT bytes: k_ba_tile
    uint32_t null_dict_lds = 0;            // bytes of the largest nullable-page dictionary that fits k_flat_null's LDS stage
    bool meta_by_kernel = false;   // this batch's metadata went up by k_upload (which also zeroes bits / npub)
    uint32_t null_dcap = 16, null_icap = 16;   // k_flat_null's level / id byte stages (NullCaps)
    int max_snap_win = 1;                  // index windows of the batch's largest Snappy job (k_snappy_chain's tables)
    uint32_t n_splits = 0;
    SnapWin* d_win = nullptr;              // in d_tokmap: bitmap | lane outs | windows | entry tables
    SnapEnt* d_ent = nullptr;
    const uint32_t* d_last_splits = nullptr;   // diagnostics: last pf_snappy_decompress tables
    uint32_t* d_lane_out = nullptr;
    std::vector<int64_t> host_status;      // per chunk host-side planning errors
    std::vector<pf_column_info> info;
    size_t bits_bytes = 0;
    int n_decode_first = 0;                // l_decode: pages that will need k_decode come first
    int n_count_flat = 0;                  // l_count: flat BYTE_ARRAY pages (k_count_flat's grid) come first
    int n_flat_fixed = 0, n_flat_all = 0, n_null4 = 0, n_null8 = 0;   // l_flat: (page, block) pairs of k_flat_fixed,
                                                                     // k_flat_all, k_flat_null<4>, <8>
    size_t off_npub = 0, npub_bytes = 0;   // k_nest_lvl / k_dbp_pos window hand-overs (scratch), zeroed before the batch
    int max_nwin = 0, max_dbp_nwin = 0;
    size_t out_bytes = 0;                  // values / offsets / levels arena extent of the last decode
    size_t off_chunks = 0, off_pages = 0, off_jobs = 0, off_lists = 0, off_res = 0, meta_bytes = 0;
    size_t off_pieces = 0, off_splits = 0, off_fallback = 0, off_wins = 0, off_bajobs = 0, off_batiles = 0, off_nfbq = 0;
    uint64_t chars_need = 0;
    const uint8_t* d_bytes = nullptr;
    int reruns = 0;
};

namespace {

int fail(pf_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    g_err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                     \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(ctx, PF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// stage-timing event: only when the context has timing on (each record is a marker on the stream,
// ~7 us between kernels on MI355X, so the product path leaves them off)
#define EVREC(ctx, ev, st)                                 \
    do {                                                   \
        if ((ctx)->timing) HIPCHK(ctx, hipEventRecord(ev, st)); \
    } while (0)

int type_width(int ptype, int type_length) {
    switch (ptype) {
    case PF_BOOLEAN: return 1;
    case PF_INT32: case PF_FLOAT: return 4;
    case PF_INT64: case PF_DOUBLE: return 8;
    case PF_INT96: return 12;
    case PF_BYTE_ARRAY: return 0;
    case PF_FIXED_LEN_BYTE_ARRAY: return type_length > 0 ? type_length : -1;
    default: return -1;
    }
}

// Enqueue the kernels of the planned batch (metadata already on device).
int enqueue_kernels(pf_ctx* ctx) {
    hipStream_t st = ctx->stream;
    uint8_t* meta = static_cast<uint8_t*>(ctx->d_meta.p);
    DevChunk* d_chunks = reinterpret_cast<DevChunk*>(meta + ctx->off_chunks);
    DevPage* d_pages = reinterpret_cast<DevPage*>(meta + ctx->off_pages);
    SnappyJob* d_jobs = reinterpret_cast<SnappyJob*>(meta + ctx->off_jobs);
    DevChunkResult* d_res = reinterpret_cast<DevChunkResult*>(meta + ctx->off_res);
    int* lists = reinterpret_cast<int*>(meta + ctx->off_lists);
    size_t lo = 0;
    int* d_dictbin = lists + lo; lo += ctx->l_dictbin.size();
    int* d_delta = lists + lo; lo += ctx->l_delta.size();
    int* d_count = lists + lo; lo += ctx->l_count.size();
    int* d_scan = lists + lo; lo += ctx->l_scan.size();
    int* d_flat = lists + lo; lo += ctx->l_flat.size();
    int* d_decode = lists + lo; lo += ctx->l_decode.size();
    int* d_runs = lists + lo; lo += ctx->l_runs.size();
    int* d_dlen = lists + lo; lo += ctx->l_dlen.size();
    int* d_dba = lists + lo; lo += ctx->l_dba.size();
    int* d_lvl = lists + lo; lo += ctx->l_lvl.size();
    int* d_djobs = lists + lo; lo += ctx->l_djobs.size();
    int* d_nest = lists + lo; lo += ctx->l_nest.size();
    const int2* d_nseg = reinterpret_cast<const int2*>(lists + lo); lo += ctx->l_nseg.size();
    const int2* d_cdict = reinterpret_cast<const int2*>(lists + lo); lo += ctx->l_cdict.size();
    const int n_nest = int(ctx->l_nest.size()), n_nseg = int(ctx->l_nseg.size() / 2);
    unsigned long long* used = reinterpret_cast<unsigned long long*>(meta + ctx->meta_bytes - 256);
    const int2* d_pieces = reinterpret_cast<const int2*>(meta + ctx->off_pieces);
    uint32_t* d_splits = reinterpret_cast<uint32_t*>(meta + ctx->off_splits);
    int* d_fallback = reinterpret_cast<int*>(meta + ctx->off_fallback);
    const int2* d_wins = reinterpret_cast<const int2*>(meta + ctx->off_wins);

    // diagnostics build only (bench analysis, results are wrong): stages left out of every batch, so a
    // step's time without them shows what they cost under load
#ifdef PF_DIAG
    const unsigned skip = ctx->opts.debug_skip;
#else
    constexpr unsigned skip = 0;
#endif
    if (!ctx->meta_by_kernel) {   // (the zero-copy upload, k_upload, zeroes them)
        if (ctx->bits_bytes) HIPCHK(ctx, hipMemsetAsync(ctx->d_bits.p, 0, ctx->bits_bytes, st));
        if (ctx->npub_bytes)
            HIPCHK(ctx, hipMemsetAsync(static_cast<uint8_t*>(ctx->d_scratch.p) + ctx->off_npub, 0, ctx->npub_bytes, st));
    }
    EVREC(ctx, ctx->ev[1], st);
    // single-literal pages in place, PLAIN fixed-width pages straight into the column (pf_pages.hip)
    if (!(skip & 1u)) launch_snappy_head(d_jobs, int(ctx->jobs.size()), d_pages, d_chunks, d_fallback, d_res, st);
    if (!(skip & 1u)) launch_snappy_litcopy(d_jobs, d_djobs, int(ctx->l_djobs.size()), d_fallback, st);
    if (!(skip & 1u)) launch_snappy_parse(d_jobs, int(ctx->jobs.size()), d_wins, int(ctx->wins.size()), ctx->d_win, ctx->d_ent,
                        ctx->d_lane_out, d_splits, d_fallback, ctx->max_snap_win, st);
    EVREC(ctx, ctx->ev[2], st);
    if (skip & 2u) {
    } else if (ctx->exec_stream) {
        HIPCHK(ctx, hipEventRecord(ctx->ev_fork, st));
        HIPCHK(ctx, hipStreamWaitEvent(ctx->exec_stream, ctx->ev_fork, 0));
        launch_snappy_exec(d_jobs, int(ctx->jobs.size()), d_pieces, int(ctx->pieces.size()), d_splits, d_fallback, d_res,
                           ctx->opts.exec, ctx->exec_stream);
        HIPCHK(ctx, hipEventRecord(ctx->ev_join, ctx->exec_stream));
        HIPCHK(ctx, hipStreamWaitEvent(st, ctx->ev_join, 0));
    } else {
        launch_snappy_exec(d_jobs, int(ctx->jobs.size()), d_pieces, int(ctx->pieces.size()), d_splits, d_fallback, d_res,
                           ctx->opts.exec, st);
    }
    EVREC(ctx, ctx->ev[3], st);
    BaJob* d_bajobs = reinterpret_cast<BaJob*>(meta + ctx->off_bajobs);
    const int2* d_batiles = reinterpret_cast<const int2*>(meta + ctx->off_batiles);
    const int n_ba = int(ctx->bajobs.size()), n_bt = int(ctx->ba_tiles.size());
    (void)d_dictbin;
    if (!(skip & 4u)) launch_ba(d_bajobs, ctx->n_ba_dict, d_batiles, ctx->n_ba_dict_tiles, d_res, st, ctx->ba_short_dict && ctx->opts.ba_fused);
    EVREC(ctx, ctx->ev[4], st);
    launch_delta(d_chunks, d_pages, d_delta, int(ctx->l_delta.size()), ctx->max_dbp_nwin, d_res, st);
    EVREC(ctx, ctx->ev[5], st);
    if (!(skip & 8u)) launch_runs(d_chunks, d_pages, d_runs, int(ctx->l_runs.size()), d_res, st);
    const NullCaps ncaps{ctx->opts.null_dcap ? ctx->opts.null_dcap : ctx->null_dcap, ctx->null_icap,
                         ctx->opts.null_dict_lds ? ctx->null_dict_lds : 0u};
    if (!(skip & 8u)) launch_lvl(d_chunks, d_pages, d_lvl, int(ctx->l_lvl.size()), d_res, st, ctx->opts.page_null, ncaps);
    launch_dlen(d_chunks, d_pages, d_dlen, int(ctx->l_dlen.size()), d_res, st);
    EVREC(ctx, ctx->ev[6], st);
    launch_nest_lvl(d_chunks, d_pages, d_nest, n_nest, ctx->max_nwin, d_res, st, ctx->opts.nest_timeout);
    if (!(skip & 16u)) launch_count(d_chunks, d_pages, d_count, int(ctx->l_count.size()), ctx->n_count_flat, d_cdict, int(ctx->l_cdict.size() / 2),
                                       d_res, d_bajobs, st, ctx->opts.count_grid);
    launch_nest_count(d_chunks, d_pages, d_nest, n_nest, d_nseg, n_nseg, d_res, st);
    if (!(skip & 4u))
        launch_ba(d_bajobs + ctx->n_ba_dict, n_ba - ctx->n_ba_dict, d_batiles + ctx->n_ba_dict_tiles, n_bt - ctx->n_ba_dict_tiles,
                  d_res, st, ctx->ba_short_data && ctx->opts.ba_fused);
    EVREC(ctx, ctx->ev[7], st);
    launch_scan(d_chunks, d_pages, d_scan, int(ctx->l_scan.size()), d_res, static_cast<uint8_t*>(ctx->d_chars.p),
                ctx->d_chars.cap, used, st);
    EVREC(ctx, ctx->ev[8], st);
    if (!(skip & 32u))
        launch_flat(d_chunks, d_pages, d_flat, ctx->n_flat_fixed, ctx->n_flat_all, ctx->n_null4, ctx->n_null8,
                    reinterpret_cast<int*>(meta + ctx->off_nfbq), d_res, st, ncaps, ctx->opts.null_stagger);
    EVREC(ctx, ctx->ev[9], st);
    if (!(skip & 64u)) launch_decode(d_chunks, d_pages, d_decode, int(ctx->l_decode.size()), ctx->n_decode_first, d_res, st,
                                       ctx->opts.decode_grid);
    launch_nest_decode(d_chunks, d_pages, d_nseg, n_nseg, d_res, st);
    launch_dba_chars(d_chunks, d_pages, d_dba, int(ctx->l_dba.size()), d_res, st);
    EVREC(ctx, ctx->ev[10], st);
    HIPCHK(ctx, hipGetLastError());
    // results + device-written chunk fields (chars base) back to pinned host memory
    const size_t res_pad = align_up(sizeof(DevChunkResult) * ctx->n_chunks, 256);
    if (ctx->zc && ctx->h_res.d) {
        copy_words(ctx->h_res.d, meta + ctx->off_res, sizeof(DevChunkResult) * ctx->n_chunks,
                   static_cast<uint8_t*>(ctx->h_res.d) + res_pad, d_chunks, sizeof(DevChunk) * ctx->n_chunks, st);
    } else {
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_res.p, meta + ctx->off_res, sizeof(DevChunkResult) * ctx->n_chunks,
                                   hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipMemcpyAsync(static_cast<uint8_t*>(ctx->h_res.p) + res_pad, d_chunks, sizeof(DevChunk) * ctx->n_chunks,
                                   hipMemcpyDeviceToHost, st));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev_done, st));
    return PF_OK;
}

// Snappy tables of the batch's jobs: 8 KiB index windows and 64 KiB pieces. d_tokmap holds, per
// window, 1 KiB of token-start bitmap, then 64 lane output counts, then the SnapWin records;
// the index pass writes every word, so nothing needs clearing.
int plan_snappy(pf_ctx* ctx) {
    ctx->wins.clear();
    ctx->pieces.clear();
    ctx->n_splits = 0;
    ctx->max_snap_win = 1;
    uint32_t n_win = 0;
    size_t tw = 0, tp = 0;
    for (SnappyJob& jb : ctx->jobs) {
        jb.n_win = std::max<uint32_t>(1u, uint32_t((uint64_t(jb.src_len) + SNAP_WIN - 1) / SNAP_WIN));
        ctx->max_snap_win = std::max(ctx->max_snap_win, int(std::min<uint32_t>(jb.n_win, 1u << 20)));
        jb.n_pieces = std::max<uint32_t>(1u, uint32_t((uint64_t(jb.dst_len) + SNAP_BLOCK - 1) / SNAP_BLOCK));
        tw += jb.n_win;
        tp += jb.n_pieces;
    }
    ctx->wins.resize(tw);
    ctx->pieces.resize(tp);
    // Dispatch the pieces with the most compressed bytes per 64 KiB of output first (more tokens per
    // piece -> more executor steps), so the longest pieces do not start last (k_snappy_exec alone
    // 1.50 -> 1.39 ms per launch on SF1). PF_PIECE_ORDER=0 keeps page order (A/B).
    const bool lpt = ctx->opts.piece_order;
    std::vector<uint64_t> keyed(lpt ? tp : 0);
    size_t wi = 0, pi = 0;
    for (size_t j = 0; j < ctx->jobs.size(); j++) {
        SnappyJob& jb = ctx->jobs[j];
        jb.win_base = n_win;
        for (uint32_t w = 0; w < jb.n_win; w++) ctx->wins[wi++] = int2{int(j), int(w)};
        n_win += jb.n_win;
        jb.split_base = ctx->n_splits;
        ctx->n_splits += jb.n_pieces;
        const uint64_t cost = uint64_t(jb.src_len) / jb.n_pieces;   // compressed bytes per piece
        for (uint32_t k = 0; k < jb.n_pieces; k++) {
            if (lpt) keyed[pi] = (std::min<uint64_t>(cost, 0xffffffffull) << 32) | uint64_t(pi);
            ctx->pieces[pi++] = int2{int(j), int(k)};
        }
    }
    if (lpt) {   // descending cost in 64-byte buckets (counting sort: O(pieces)), ties in page order
        constexpr uint32_t NB = 4096;
        std::vector<uint32_t> start(NB + 1, 0);
        auto bucket = [](uint64_t k) { return NB - 1 - uint32_t(std::min<uint64_t>((k >> 32) >> 6, NB - 1)); };
        for (size_t i = 0; i < tp; i++) start[bucket(keyed[i]) + 1]++;
        for (uint32_t b = 0; b < NB; b++) start[b + 1] += start[b];
        std::vector<int2> sorted(tp);
        for (size_t i = 0; i < tp; i++) sorted[start[bucket(keyed[i])]++] = ctx->pieces[size_t(uint32_t(keyed[i]))];
        ctx->pieces.swap(sorted);
    }
    const size_t tok_bytes = size_t(n_win) * SNAP_WWORDS * 4, lo_bytes = size_t(n_win) * 64 * 4;
    const size_t win_bytes = align_up(size_t(n_win) * sizeof(SnapWin), 256), ent_bytes = size_t(n_win) * 64 * sizeof(SnapEnt);
    HIPCHK(ctx, ctx->d_tokmap.ensure(tok_bytes + lo_bytes + win_bytes + ent_bytes + 256));
    uint8_t* base = static_cast<uint8_t*>(ctx->d_tokmap.p);
    ctx->d_lane_out = reinterpret_cast<uint32_t*>(base + tok_bytes);
    ctx->d_win = reinterpret_cast<SnapWin*>(base + tok_bytes + lo_bytes);
    ctx->d_ent = reinterpret_cast<SnapEnt*>(base + tok_bytes + lo_bytes + win_bytes);
    for (SnappyJob& jb : ctx->jobs) jb.tokmap = reinterpret_cast<uint32_t*>(base) + size_t(jb.win_base) * SNAP_WWORDS;
    return PF_OK;
}

// Upload metadata tables (results zeroed, arena counter zeroed).
int upload_meta(pf_ctx* ctx) {
    uint8_t* h = static_cast<uint8_t*>(ctx->h_meta.p);
    std::memset(h, 0, ctx->meta_bytes);
    std::memcpy(h + ctx->off_chunks, ctx->chunks.data(), sizeof(DevChunk) * ctx->chunks.size());
    std::memcpy(h + ctx->off_pages, ctx->pages.data(), sizeof(DevPage) * ctx->pages.size());
    std::memcpy(h + ctx->off_jobs, ctx->jobs.data(), sizeof(SnappyJob) * ctx->jobs.size());
    std::memcpy(h + ctx->off_pieces, ctx->pieces.data(), sizeof(int2) * ctx->pieces.size());
    std::memset(h + ctx->off_splits, 0xff, sizeof(uint32_t) * ctx->n_splits);
    std::memcpy(h + ctx->off_wins, ctx->wins.data(), sizeof(int2) * ctx->wins.size());
    {   // data-page walks report their chars into the page record
        BaJob* bj = reinterpret_cast<BaJob*>(h + ctx->off_bajobs);
        std::memcpy(bj, ctx->bajobs.data(), sizeof(BaJob) * ctx->bajobs.size());
        uint8_t* dpages = static_cast<uint8_t*>(ctx->d_meta.p) + ctx->off_pages;
        for (size_t i = size_t(ctx->n_ba_dict); i < ctx->bajobs.size(); i++)
            bj[i].chars_out = reinterpret_cast<int64_t*>(dpages + sizeof(DevPage) * size_t(bj[i].page) + offsetof(DevPage, n_chars));
        std::memcpy(h + ctx->off_batiles, ctx->ba_tiles.data(), sizeof(int2) * ctx->ba_tiles.size());
    }
    int* lists = reinterpret_cast<int*>(h + ctx->off_lists);
    size_t lo = 0;
    for (auto* v : {&ctx->l_dictbin, &ctx->l_delta, &ctx->l_count, &ctx->l_scan, &ctx->l_flat, &ctx->l_decode, &ctx->l_runs,
                    &ctx->l_dlen, &ctx->l_dba, &ctx->l_lvl, &ctx->l_djobs, &ctx->l_nest, &ctx->l_nseg, &ctx->l_cdict}) {
        std::copy(v->begin(), v->end(), lists + lo);
        lo += v->size();
    }
    {   // diagnostics: force_serial = k sends every k-th Snappy job to the serial kernel (tests of
        // k_snappy_serial's grid-stride over many jobs; valid streams never fall back)
        const int k = ctx->opts.force_serial;
        int* fbh = reinterpret_cast<int*>(h + ctx->off_fallback);
        if (k > 0)
            for (size_t j = 0; j < ctx->jobs.size(); j++)
                if (int(j % size_t(k)) == k - 1) fbh[j] = FB_SERIAL;
        // force_redo = k: the block-parallel executor rejects every k-th job (after k_snappy_head), so
        // direct pages are also decoded through the redo path (tests)
        const int kr = ctx->opts.force_redo;
        SnappyJob* jh = reinterpret_cast<SnappyJob*>(h + ctx->off_jobs);
        if (kr > 0)
            for (size_t j = 0; j < ctx->jobs.size(); j++)
                if (int(j % size_t(kr)) == kr - 1) jh[j].dflags |= 1u;
    }
    DevChunkResult* r = reinterpret_cast<DevChunkResult*>(h + ctx->off_res);
    for (int c = 0; c < ctx->n_chunks; c++) {
        r[c].status = int32_t(ctx->host_status[c]);
        r[c].err_page = -1;
        const DevChunk& ck = ctx->chunks[c];
        if (!ck.needs_count) {   // flat fixed width: slots = rows = entries (host-known)
            r[c].num_slots = ck.num_entries;
            r[c].num_rows = ck.num_entries;
        }
    }
    // k_upload counts in 32 bits: an arena of 4 GiB or more takes the copy path (its zero fills below)
    const bool small = ctx->meta_bytes / 8 < (1ull << 31) && ctx->bits_bytes < (1ull << 31) && ctx->npub_bytes < (1ull << 31);
    ctx->meta_by_kernel = ctx->zc && ctx->h_meta.d && small;
    if (ctx->meta_by_kernel) {   // enqueue_kernels follows at once on the same stream
        const uint32_t n = uint32_t(ctx->meta_bytes / 8), nz0 = uint32_t(ctx->bits_bytes), nz1 = uint32_t(ctx->npub_bytes);
        const uint32_t grid = std::max(1u, std::min(1024u, (n + (nz0 + 7u) / 8u + (nz1 + 7u) / 8u + 255u) / 256u));
        hipLaunchKernelGGL(k_upload, dim3(grid), dim3(256), 0, ctx->stream, static_cast<uint64_t*>(ctx->d_meta.p),
                           static_cast<const uint64_t*>(ctx->h_meta.d), n, static_cast<uint8_t*>(ctx->d_bits.p), nz0,
                           static_cast<uint8_t*>(ctx->d_scratch.p) + ctx->off_npub, nz1);
        HIPCHK(ctx, hipGetLastError());
    } else {
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_meta.p, h, ctx->meta_bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    return PF_OK;
}

}  // namespace


// ---------------------------------------------------------------- write path (pf_encode.hip)
namespace {
size_t uvarint_len(uint64_t v) { size_t k = 1; while (v >= 0x80) { v >>= 7; k++; } return k; }
void put_uvarint(std::vector<uint8_t>& o, uint64_t v) {
    while (v >= 0x80) { o.push_back(uint8_t(v | 0x80)); v >>= 7; }
    o.push_back(uint8_t(v));
}

// Snappy-compress `sections` (device, each [off, off + len) of `base`) into SC_BLOCK-job slots;
// returns per section the host stream (varint length + block outputs) in `streams`.
int compress_sections(pf_ctx* ctx, const uint8_t* base, const std::vector<std::pair<uint64_t, uint64_t>>& sections,
                      std::vector<std::vector<uint8_t>>& streams, float* kernel_ms = nullptr) {
    hipStream_t st = ctx->stream;
    std::vector<SnapCJob> jobs;
    std::vector<std::pair<size_t, size_t>> range(sections.size());   // jobs of each section
    for (size_t i = 0; i < sections.size(); i++) {
        range[i].first = jobs.size();
        for (uint64_t o = 0; o < sections[i].second; o += SC_BLOCK) {
            SnapCJob j{};
            j.src = base + sections[i].first + o;
            j.len = uint32_t(std::min<uint64_t>(SC_BLOCK, sections[i].second - o));
            jobs.push_back(j);
        }
        range[i].second = jobs.size();
    }
    const size_t nj = jobs.size();
    size_t m = 0;
    auto take = [](size_t& cur, size_t sz) { size_t o = align_up(cur, 256); cur = o + sz; return o; };
    const size_t o_jobs = take(m, sizeof(SnapCJob) * std::max<size_t>(nj, 1));
    const size_t o_len = take(m, 4 * std::max<size_t>(nj, 1));
    const size_t o_slots = take(m, size_t(SC_SLOT) * std::max<size_t>(nj, 1));
    HIPCHK(ctx, ctx->d_enc_out.ensure(m));
    uint8_t* d = static_cast<uint8_t*>(ctx->d_enc_out.p);
    for (size_t k = 0; k < nj; k++) jobs[k].dst = d + o_slots + k * SC_SLOT;
    // compressed lengths + slots come back into the context's pinned staging (no zero-fill, DMA speed)
    HIPCHK(ctx, ctx->h_enc_slots.ensure(align_up(4 * std::max<size_t>(nj, 1), 256) + nj * size_t(SC_SLOT)));
    uint32_t* lens = static_cast<uint32_t*>(ctx->h_enc_slots.p);
    uint8_t* slots = static_cast<uint8_t*>(ctx->h_enc_slots.p) + align_up(4 * std::max<size_t>(nj, 1), 256);
    if (nj) {
        HIPCHK(ctx, hipMemcpyAsync(d + o_jobs, jobs.data(), sizeof(SnapCJob) * nj, hipMemcpyHostToDevice, st));
        EVREC(ctx, ctx->ev[0], st);
        launch_snappy_compress(reinterpret_cast<const SnapCJob*>(d + o_jobs), int(nj), reinterpret_cast<uint32_t*>(d + o_len), st);
        HIPCHK(ctx, hipGetLastError());
        EVREC(ctx, ctx->ev[1], st);
        HIPCHK(ctx, hipMemcpyAsync(lens, d + o_len, 4 * nj, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipMemcpyAsync(slots, d + o_slots, nj * size_t(SC_SLOT), hipMemcpyDeviceToHost, st));
    }
    HIPCHK(ctx, hipStreamSynchronize(st));
    if (kernel_ms) {
        *kernel_ms = 0.f;
        if (ctx->timing && nj) HIPCHK(ctx, hipEventElapsedTime(kernel_ms, ctx->ev[0], ctx->ev[1]));
    }
    streams.assign(sections.size(), {});
    for (size_t i = 0; i < sections.size(); i++) {
        std::vector<uint8_t>& o = streams[i];
        put_uvarint(o, sections[i].second);
        for (size_t k = range[i].first; k < range[i].second; k++) {
            if (lens[k] > SC_SLOT) return fail(ctx, PF_ERR_HIP, "snappy compress: block overflow");
            const uint8_t* b = slots + k * size_t(SC_SLOT);
            o.insert(o.end(), b, b + lens[k]);
        }
    }
    return PF_OK;
}
}  // namespace

extern "C" int pf_snappy_compress(pf_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    if (!ctx || (!src && n) || !out_len) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "previous decode not waited for");
    if (n > 0xffffffffull) return fail(ctx, PF_ERR_INVALID_ARG, "snappy: buffer too large");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (ctx->copies_pending) HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));
    ctx->copies_pending = false;
    HIPCHK(ctx, ctx->d_enc.ensure(std::max<size_t>(n, 1)));
    if (n) HIPCHK(ctx, hipMemcpyAsync(ctx->d_enc.p, src, n, hipMemcpyHostToDevice, ctx->stream));
    std::vector<std::vector<uint8_t>> streams;
    const int rc = compress_sections(ctx, static_cast<const uint8_t*>(ctx->d_enc.p), {{0, n}}, streams);
    if (rc) return rc;
    *out_len = streams[0].size();
    if (streams[0].size() > cap) return fail(ctx, PF_ERR_CAPACITY, "snappy: destination too small");
    std::memcpy(dst, streams[0].data(), streams[0].size());
    return PF_OK;
}

extern "C" int pf_encode_chunk(pf_ctx* ctx, const pf_encode_column* col, int on_device, pf_encoded_chunk* out) {
    if (!ctx || !col || !out) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "previous decode not waited for");
    const int pt = col->physical_type;
    if (pt != PF_BOOLEAN && pt != PF_INT32 && pt != PF_INT64 && pt != PF_FLOAT && pt != PF_DOUBLE && pt != PF_BYTE_ARRAY)
        return fail(ctx, PF_ERR_UNSUPPORTED_TYPE, "encode: unsupported physical type");
    const int64_t n = col->num_rows;
    if (n < 0 || n > 0x7ffffff0 || (col->max_def != 0 && col->max_def != 1)) return fail(ctx, PF_ERR_INVALID_ARG, "encode: bad shape");
    if (col->codec != PF_CODEC_SNAPPY && col->codec != PF_CODEC_UNCOMPRESSED)
        return fail(ctx, PF_ERR_UNSUPPORTED_CODEC, "encode: codec must be SNAPPY or UNCOMPRESSED");
    const bool str = pt == PF_BYTE_ARRAY;
    if (n > 0 && (str ? (!col->offsets || (!col->chars && col->chars_len > 0) || col->chars_len < 0 || col->chars_len > 0x7fffffff)
                      : !col->values))
        return fail(ctx, PF_ERR_INVALID_ARG, "encode: missing input arrays");
    const int w = pt == PF_BOOLEAN ? 1 : type_width(pt, 0);
    int64_t page_rows = col->page_rows > 0 ? col->page_rows : 20000;
    page_rows = (page_rows + 7) / 8 * 8;   // definition levels of a page start on a validity byte
    // dictionary page limit (parquet.dictionary.page.size, 1 MiB); capped so a dictionary that passes it
    // always fits the 32-bit offsets of the dictionary kernels
    const int64_t dict_limit = std::min<int64_t>(col->dict_page_limit > 0 ? col->dict_page_limit : (1 << 20), 0x7fffffff);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (ctx->copies_pending) HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));
    ctx->copies_pending = false;

    // host copies of validity / offsets (page plan, definition levels)
    const size_t vbytes = size_t((n + 7) / 8);
    std::vector<uint8_t> hval;
    std::vector<int32_t> hoff;
    const bool has_val = col->max_def == 1 && col->validity;
    if (has_val) {
        hval.resize(vbytes);
        if (on_device) HIPCHK(ctx, hipMemcpy(hval.data(), col->validity, vbytes, hipMemcpyDeviceToHost));
        else std::memcpy(hval.data(), col->validity, vbytes);
    }
    if (str && n > 0) {
        hoff.resize(size_t(n) + 1);
        if (on_device) HIPCHK(ctx, hipMemcpy(hoff.data(), col->offsets, 4 * (size_t(n) + 1), hipMemcpyDeviceToHost));
        else std::memcpy(hoff.data(), col->offsets, 4 * (size_t(n) + 1));
        for (int64_t r = 0; r < n; r++)
            if (hoff[r + 1] < hoff[r] || hoff[r] < 0 || hoff[r + 1] > col->chars_len)
                return fail(ctx, PF_ERR_INVALID_ARG, "encode: offsets out of order or outside chars");
    }
    auto present = [&](int64_t r) { return !has_val || ((hval[size_t(r >> 3)] >> (r & 7)) & 1); };
    // page plan: rows, present values, PLAIN byte sizes
    struct PagePlanE { int64_t r0, r1; uint32_t d0, cnt; uint64_t plain; };
    std::vector<PagePlanE> pp;
    uint32_t m = 0;
    for (int64_t r0 = 0; r0 < n || (n == 0 && pp.empty()); r0 += page_rows) {
        PagePlanE p{r0, std::min(n, r0 + page_rows), m, 0, 0};
        for (int64_t r = p.r0; r < p.r1; r++)
            if (present(r)) {
                p.cnt++;
                if (str) p.plain += 4 + uint64_t(hoff[r + 1] - hoff[r]);
            }
        if (!str) p.plain = pt == PF_BOOLEAN ? (p.cnt + 7) / 8 : uint64_t(p.cnt) * w;
        m += p.cnt;
        pp.push_back(p);
        if (n == 0) break;
    }

    // ---- device arena ----
    size_t a_sz = 0;
    auto take = [](size_t& cur, size_t sz) { size_t o = align_up(cur, 256); cur = o + std::max<size_t>(sz, 1); return o; };
    const size_t N1 = size_t(n) + 1;
    const size_t o_in = take(a_sz, str ? 0 : size_t(n) * w), o_vl = take(a_sz, vbytes);
    const size_t o_of = take(a_sz, str ? 4 * N1 : 0), o_ch = take(a_sz, str ? size_t(col->chars_len) : 0);
    const size_t o_flag = take(a_sz, 4 * N1), o_pos = take(a_sz, 4 * N1), o_dense = take(a_sz, size_t(n) * w);
    const size_t o_dsrc = take(a_sz, str ? 4 * N1 : 0), o_dlen = take(a_sz, str ? 4 * N1 : 0);
    const size_t o_vsz = take(a_sz, str ? 4 * N1 : 0), o_vpre = take(a_sz, str ? 4 * N1 : 0);
    const size_t o_key = take(a_sz, 8 * N1), o_skey = take(a_sz, 8 * N1), o_didx = take(a_sz, 4 * N1), o_sidx = take(a_sz, 4 * N1);
    const size_t o_hp = take(a_sz, 4 * N1), o_head = take(a_sz, 4 * N1), o_mark = take(a_sz, 4 * N1), o_did = take(a_sz, 4 * N1);
    const size_t o_dsz = take(a_sz, 4 * N1), o_doff = take(a_sz, 4 * N1), o_ids = take(a_sz, 4 * N1), o_col = take(a_sz, 256);
    size_t temp_bytes = 0;
    HIPCHK(ctx, enc_scan_temp(N1, temp_bytes));
    const size_t o_temp = take(a_sz, temp_bytes);
    HIPCHK(ctx, ctx->d_enc.ensure(a_sz));
    uint8_t* A = static_cast<uint8_t*>(ctx->d_enc.p);
    EncArgs ea{};
    ea.ptype = pt; ea.width = w; ea.n = n;
    if (on_device) {
        ea.values = static_cast<const uint8_t*>(col->values);
        ea.validity = has_val ? col->validity : nullptr;
        ea.offsets = col->offsets;
        ea.chars = col->chars;
    } else {
        if (!str && n) HIPCHK(ctx, hipMemcpyAsync(A + o_in, col->values, size_t(n) * w, hipMemcpyHostToDevice, st));
        if (has_val && vbytes) HIPCHK(ctx, hipMemcpyAsync(A + o_vl, hval.data(), vbytes, hipMemcpyHostToDevice, st));
        if (str && n) {
            HIPCHK(ctx, hipMemcpyAsync(A + o_of, hoff.data(), 4 * N1, hipMemcpyHostToDevice, st));
            if (col->chars_len) HIPCHK(ctx, hipMemcpyAsync(A + o_ch, col->chars, size_t(col->chars_len), hipMemcpyHostToDevice, st));
        }
        ea.values = A + o_in;
        ea.validity = has_val ? A + o_vl : nullptr;
        ea.offsets = reinterpret_cast<const int32_t*>(A + o_of);
        ea.chars = A + o_ch;
    }
    ea.flag = reinterpret_cast<uint32_t*>(A + o_flag); ea.pos = reinterpret_cast<uint32_t*>(A + o_pos);
    ea.dense = A + o_dense;
    ea.dsrc = reinterpret_cast<uint32_t*>(A + o_dsrc); ea.dlen = reinterpret_cast<uint32_t*>(A + o_dlen);
    ea.vsz = reinterpret_cast<uint32_t*>(A + o_vsz); ea.vpre = reinterpret_cast<uint32_t*>(A + o_vpre);
    ea.key = reinterpret_cast<uint64_t*>(A + o_key); ea.skey = reinterpret_cast<uint64_t*>(A + o_skey);
    ea.didx = reinterpret_cast<uint32_t*>(A + o_didx); ea.sidx = reinterpret_cast<uint32_t*>(A + o_sidx);
    ea.headpos = reinterpret_cast<uint32_t*>(A + o_hp); ea.head = reinterpret_cast<uint32_t*>(A + o_head);
    ea.mark = reinterpret_cast<uint32_t*>(A + o_mark); ea.did = reinterpret_cast<uint32_t*>(A + o_did);
    ea.dsz = reinterpret_cast<uint32_t*>(A + o_dsz); ea.doff = reinterpret_cast<uint32_t*>(A + o_doff);
    ea.ids = reinterpret_cast<uint32_t*>(A + o_ids); ea.collide = reinterpret_cast<uint32_t*>(A + o_col);
    void* temp = A + o_temp;

    HIPCHK(ctx, hipMemsetAsync(A + o_col, 0, 256, st));
    if (str) HIPCHK(ctx, hipMemsetAsync(ea.vsz, 0, 4 * N1, st));
    EVREC(ctx, ctx->ev[2], st);
    if (n) HIPCHK(ctx, enc_dense(ea, temp, temp_bytes, st));
    if (str) HIPCHK(ctx, enc_plain_sizes(ea, m, temp, temp_bytes, st));
    // The device sums dictionary bytes in 32 bits: a BYTE_ARRAY column whose dictionary could reach 4 GiB
    // (all values distinct: 4 m + chars) is written PLAIN (conservative: such a dictionary is over any
    // page limit unless most values repeat; parity with parquet-mr's writer is unpinned).
    const bool dict_fits32 = !str || 4ull * uint64_t(m) + uint64_t(col->chars_len) < (1ull << 32);
    const bool want_dict = col->dictionary && pt != PF_BOOLEAN && m > 0 && dict_fits32;
    uint32_t hres[3] = {0, 0, 0};   // collide, dictionary entries, dictionary bytes
    float enc_ms = 0.f;
    if (want_dict) {
        HIPCHK(ctx, enc_dictionary(ea, m, w == 4 ? 32 : 64, temp, temp_bytes, st));
        EVREC(ctx, ctx->ev[3], st);
        HIPCHK(ctx, hipMemcpyAsync(&hres[0], ea.collide, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipMemcpyAsync(&hres[1], ea.did + m, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipMemcpyAsync(&hres[2], ea.doff + m, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipStreamSynchronize(st));
        if (ctx->timing) HIPCHK(ctx, hipEventElapsedTime(&enc_ms, ctx->ev[2], ctx->ev[3]));
    }
    int fallback = 0;
    if (col->dictionary && pt == PF_BOOLEAN) fallback = 3;
    else if (want_dict && hres[0]) fallback = 2;
    else if (col->dictionary && pt != PF_BOOLEAN && m > 0 && !dict_fits32) fallback = 1;
    else if (want_dict && (str ? int64_t(hres[2]) : int64_t(hres[1]) * w) > dict_limit) fallback = 1;   // fixed: D * w on the host
    const bool dict = want_dict && fallback == 0;
    const uint32_t D = dict ? hres[1] : 0, dict_bytes = dict ? (str ? hres[2] : hres[1] * uint32_t(w)) : 0;
    uint32_t bw = 1;
    while (D > 1 && (uint64_t(1) << bw) < D) bw++;

    // ---- values sections: [dictionary page | page 0 | page 1 | ...] in d_enc_out's front ----
    std::vector<EncPage> ep(pp.size());
    std::vector<std::pair<uint64_t, uint64_t>> sections;
    size_t vo = 0;
    const size_t o_dict = take(vo, dict_bytes);
    if (dict) sections.push_back({o_dict, dict_bytes});
    for (size_t i = 0; i < pp.size(); i++) {
        const PagePlanE& p = pp[i];
        uint64_t bytes;
        if (dict) {
            const uint64_t groups = (p.cnt + 7) / 8;
            bytes = p.cnt ? 1 + uvarint_len((groups << 1) | 1) + groups * bw : 1;
        } else {
            bytes = p.plain;
        }
        ep[i] = EncPage{0, p.d0, p.cnt, dict ? 1u : 0u, bw};
        ep[i].out_off = take(vo, bytes);
        sections.push_back({ep[i].out_off, bytes});
    }
    const size_t o_pages = take(vo, sizeof(EncPage) * ep.size());
    HIPCHK(ctx, ctx->d_enc_sec.ensure(vo));
    uint8_t* SEC = static_cast<uint8_t*>(ctx->d_enc_sec.p);
    ea.dict_out = SEC + o_dict;
    ea.vals_out = SEC;
    EVREC(ctx, ctx->ev[4], st);
    if (dict) enc_dictionary_page_and_ids(ea, m, st);
    HIPCHK(ctx, hipMemcpyAsync(SEC + o_pages, ep.data(), sizeof(EncPage) * ep.size(), hipMemcpyHostToDevice, st));
    enc_pages(ea, reinterpret_cast<const EncPage*>(SEC + o_pages), int(ep.size()), st);
    HIPCHK(ctx, hipGetLastError());
    EVREC(ctx, ctx->ev[5], st);
    std::vector<std::vector<uint8_t>> bodies;
    float snap_ms = 0.f;
    if (col->codec == PF_CODEC_SNAPPY) {
        const int rc = compress_sections(ctx, SEC, sections, bodies, &snap_ms);
        if (rc) return rc;
    } else {
        std::vector<uint8_t> all(vo);
        HIPCHK(ctx, hipMemcpyAsync(all.data(), SEC, vo, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipStreamSynchronize(st));
        for (const auto& sct : sections) bodies.emplace_back(all.begin() + sct.first, all.begin() + sct.first + sct.second);
    }

    // ---- page headers + bodies ----
    std::vector<uint8_t>& o = ctx->h_enc;
    o.clear();
    int64_t unc = 0;
    size_t bi = 0;
    out->dictionary_page_offset = -1;
    if (dict) {
        PageHeaderOut h;
        h.page_type = PF_PAGE_DICTIONARY;
        h.uncompressed_size = int32_t(dict_bytes);
        h.compressed_size = int32_t(bodies[0].size());
        h.num_values = int32_t(D);
        h.encoding = PF_ENC_PLAIN;   // parquet-mr PARQUET_2_0: dictionary page PLAIN, data pages RLE_DICTIONARY
        out->dictionary_page_offset = 0;
        const size_t h0 = o.size();
        write_page_header(o, h);
        unc += int64_t(o.size() - h0) + dict_bytes;
        o.insert(o.end(), bodies[0].begin(), bodies[0].end());
        bi = 1;
    }
    out->data_page_offset = int64_t(o.size());
    for (size_t i = 0; i < pp.size(); i++, bi++) {
        const PagePlanE& p = pp[i];
        const int64_t rows = p.r1 - p.r0;
        std::vector<uint8_t> def;
        if (col->max_def == 1) {   // RLE/bit-packed hybrid, bit width 1: one bit-packed run = the validity bits
            const uint64_t groups = uint64_t(rows + 7) / 8;
            put_uvarint(def, (groups << 1) | 1);
            for (uint64_t g = 0; g < groups; g++) {
                uint8_t b = has_val ? hval[size_t(p.r0 / 8 + g)] : 0xff;
                const int64_t left = rows - int64_t(g) * 8;
                if (left < 8) b &= uint8_t((1u << left) - 1u);
                def.push_back(b);
            }
            if (rows == 0) def.clear();
        }
        PageHeaderOut h;
        h.page_type = PF_PAGE_DATA_V2;
        h.uncompressed_size = int32_t(def.size() + sections[bi].second);
        h.compressed_size = int32_t(def.size() + bodies[bi].size());
        h.num_values = int32_t(rows);
        h.num_nulls = int32_t(rows - p.cnt);
        h.num_rows = int32_t(rows);
        h.encoding = dict ? PF_ENC_RLE_DICTIONARY : PF_ENC_PLAIN;
        h.def_bytes = int32_t(def.size());
        h.is_compressed = col->codec == PF_CODEC_SNAPPY;
        const size_t h0 = o.size();
        write_page_header(o, h);
        unc += int64_t(o.size() - h0) + h.uncompressed_size;
        o.insert(o.end(), def.begin(), def.end());
        o.insert(o.end(), bodies[bi].begin(), bodies[bi].end());
    }
    out->bytes = o.data();
    out->size = int64_t(o.size());
    out->total_uncompressed_size = unc;
    out->num_values = n;
    out->n_data_pages = int32_t(pp.size());
    out->dict_entries = int32_t(D);
    out->data_encoding = dict ? PF_ENC_RLE_DICTIONARY : PF_ENC_PLAIN;
    out->fallback = fallback;
    out->codec = col->codec;
    if (ctx->timing) {   // the page kernels' events have completed (the stream was synchronised since)
        float pg_ms = 0.f;
        HIPCHK(ctx, hipEventElapsedTime(&pg_ms, ctx->ev[4], ctx->ev[5]));
        enc_ms += pg_ms;
    }
    out->snappy_ms = snap_ms;
    out->encode_ms = enc_ms;
    out->snappy_in = 0;
    out->snappy_out = 0;
    if (col->codec == PF_CODEC_SNAPPY)
        for (size_t i = 0; i < sections.size(); i++) {
            out->snappy_in += int64_t(sections[i].second);
            out->snappy_out += int64_t(bodies[i].size());
        }
    return PF_OK;
}

extern "C" {

int pf_abi_version(void) { return PF_ABI_VERSION; }

const char* pf_last_error(pf_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int pf_device_count(int* count) {
    if (!count) return fail(nullptr, PF_ERR_INVALID_ARG, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *count = 0; return fail(nullptr, PF_ERR_HIP, hipGetErrorString(e)); }
    *count = n;
    return PF_OK;
}

namespace {
#ifdef PF_DIAG
// Diagnostics build only: the options from the environment (PfOpts, pf_internal.h).
void opts_from_env(pf::PfOpts& o) {
    auto on = [](const char* name, bool dflt) { const char* e = std::getenv(name); return e ? e[0] == '1' : dflt; };
    auto num = [](const char* name, int dflt) { const char* e = std::getenv(name); return e ? std::atoi(e) : dflt; };
    o.exec = num("PF_EXEC", o.exec);
    o.ba_fused = on("PF_BA_FUSED", o.ba_fused);
    o.page_null = on("PF_PAGE_NULL", o.page_null);
    o.null_dict_lds = on("PF_NULL_DICT_LDS", o.null_dict_lds);
    o.nest_timeout = on("PF_DEBUG_NEST_TIMEOUT", o.nest_timeout);
    o.null_dcap = uint32_t(std::max(0, num("PF_NULL_DCAP", 0))) & ~15u;
    o.null_stagger = num("PF_DEBUG_NULL_STAGGER", o.null_stagger);
    o.piece_order = on("PF_PIECE_ORDER", o.piece_order);
    if (const char* e = std::getenv("PF_DEBUG_SKIP")) {
        const char* names[] = {"parse", "exec", "ba", "levels", "count", "flat", "decode"};
        for (int i = 0; i < 7; i++)
            if (std::strstr(e, names[i])) o.debug_skip |= 1u << i;
    }
    o.force_serial = num("PF_DEBUG_FORCE_SERIAL", o.force_serial);
    o.force_redo = num("PF_DEBUG_FORCE_REDO", o.force_redo);
    o.exec_stream = on("PF_EXEC_STREAM", o.exec_stream);
    o.zc = on("PF_ZC", o.zc);
    o.dl_kernel = on("PF_DL_KERNEL", o.dl_kernel);
    o.dl_stream = on("PF_DL_STREAM", o.dl_stream);
    o.h2d_kernel = on("PF_H2D_KERNEL", o.h2d_kernel);
    o.h2d_grid = std::max(1, num("PF_H2D_GRID", o.h2d_grid));
    o.dl_prio = on("PF_DL_PRIO", o.dl_prio);
    o.debug_plan = on("PF_DEBUG_PLAN", o.debug_plan);
    if (const char* e = std::getenv("PF_NEST_SEG")) {
        o.nest_seg = std::atoll(e);
        o.nest_seg_set = true;
    }
    o.dbp_par = on("PF_DBP_PAR", o.dbp_par);
    o.decode_grid = std::max(1, num("PF_DECODE_GRID", o.decode_grid));
    o.count_grid = std::max(1, num("PF_COUNT_GRID", o.count_grid));
    const int fb = num("PF_FIX_BLK", 8192);
    o.fix_shift = fb >= 16384 ? 2 : (fb >= 8192 ? 1 : 0);
}
#endif

int ctx_init(pf_ctx* ctx, pf_ctx* peer) {
#ifdef PF_DIAG
    opts_from_env(ctx->opts);
#endif
    HIPCHK(nullptr, hipSetDevice(ctx->device));
    if (peer) {
        ctx->streams = peer->streams;
    } else {
        ctx->streams = std::make_shared<Streams>();
        ctx->streams->device = ctx->device;
        if (ctx->opts.exec_stream) {
            int least = 0, greatest = 0;
            HIPCHK(nullptr, hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIPCHK(nullptr, hipStreamCreateWithPriority(&ctx->streams->stream, hipStreamNonBlocking, greatest));
            HIPCHK(nullptr, hipStreamCreateWithPriority(&ctx->streams->exec_stream, hipStreamNonBlocking, least));
        } else {
            HIPCHK(nullptr, hipStreamCreateWithFlags(&ctx->streams->stream, hipStreamNonBlocking));
        }
    }
    ctx->stream = ctx->streams->stream;
    ctx->exec_stream = ctx->streams->exec_stream;
    ctx->zc = ctx->opts.zc;
    if (ctx->exec_stream) {
        HIPCHK(nullptr, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
        HIPCHK(nullptr, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
    }
    HIPCHK(nullptr, hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming));
    HIPCHK(nullptr, hipEventCreateWithFlags(&ctx->ev_copy, hipEventDisableTiming));
    HIPCHK(nullptr, hipEventCreateWithFlags(&ctx->ev_dl, hipEventDisableTiming));
    for (auto& e : ctx->ev) HIPCHK(nullptr, hipEventCreate(&e));
    return PF_OK;
}

int ctx_create(int device, pf_ctx* peer, pf_ctx** out) {
    pf_ctx* ctx = new pf_ctx();
    ctx->device = device;
    const int rc = ctx_init(ctx, peer);
    if (rc != PF_OK) {   // release whatever streams / events were created before the failure
        const std::string msg = g_err;
        pf_ctx_destroy(ctx);
        g_err = msg;
        return rc;
    }
    *out = ctx;
    return PF_OK;
}
}  // namespace

int pf_ctx_create(int device, pf_ctx** out) {
    if (!out) return fail(nullptr, PF_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(nullptr, PF_ERR_INVALID_ARG, "no such HIP device");
    return ctx_create(device, nullptr, out);
}

int pf_ctx_create_shared(pf_ctx* peer, pf_ctx** out) {
    if (!out || !peer) return fail(nullptr, PF_ERR_INVALID_ARG, "null arg");
    *out = nullptr;
    return ctx_create(peer->device, peer, out);
}

int pf_ctx_set_timing(pf_ctx* ctx, int on) {
    if (!ctx) return fail(nullptr, PF_ERR_INVALID_ARG, "null ctx");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "decode in flight");
    ctx->timing = on != 0;
    ctx->timing_valid = false;
    return PF_OK;
}

int pf_ctx_destroy(pf_ctx* ctx) {
    if (!ctx) return PF_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);   // this context's work and any peer's ahead of it
    if (ctx->exec_stream) (void)hipStreamSynchronize(ctx->exec_stream);
    if (ctx->copies_pending) (void)hipEventSynchronize(ctx->ev_copy);   // (a download on the copy stream)
    for (DevBuf* b : {&ctx->d_in, &ctx->d_scratch, &ctx->d_out, &ctx->d_bits, &ctx->d_chars, &ctx->d_meta, &ctx->d_tokmap,
                      &ctx->d_scan_in, &ctx->d_scan, &ctx->d_enc, &ctx->d_enc_sec, &ctx->d_enc_out})
        b->release();
    ctx->h_meta.release();
    ctx->h_res.release();
    ctx->h_enc_slots.release();
    for (auto& e : ctx->ev) if (e) (void)hipEventDestroy(e);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
    if (ctx->ev_copy) (void)hipEventDestroy(ctx->ev_copy);
    if (ctx->ev_dl) (void)hipEventDestroy(ctx->ev_dl);
    ctx->streams.reset();   // destroys the stream(s) when no other context shares them
    delete ctx;
    return PF_OK;
}

int pf_host_alloc(pf_ctx* ctx, size_t bytes, void** out) {
    if (!out) return fail(ctx, PF_ERR_INVALID_ARG, "null out");
    if (ctx) (void)hipSetDevice(ctx->device);
    HIPCHK(ctx, hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    return PF_OK;
}

int pf_host_free(pf_ctx* ctx, void* ptr) {
    if (ptr) HIPCHK(ctx, hipHostFree(ptr));
    return PF_OK;
}

int pf_device_alloc(pf_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipMalloc(out, bytes + 256));   // slack: 16-byte staging loads may read past the end
    return PF_OK;
}

int pf_device_free(pf_ctx* ctx, void* ptr) {
    if (ptr) HIPCHK(ctx, hipFree(ptr));
    return PF_OK;
}

int pf_memcpy_h2d(pf_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return fail(ctx, PF_ERR_INVALID_ARG, "null ctx");
    HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    return PF_OK;
}

int pf_decode_row_group(pf_ctx* ctx, const pf_chunk_desc* cds, int n_chunks, const uint8_t* bytes, size_t n_bytes,
                        int bytes_on_device) {
    if (!ctx) return fail(nullptr, PF_ERR_INVALID_ARG, "null ctx");
    if (n_chunks < 0 || (n_chunks > 0 && (!cds || !bytes))) return fail(ctx, PF_ERR_INVALID_ARG, "bad arguments");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "previous decode not waited for");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // diagnostics: PF_DEBUG_PLAN=1 prints the host time of each planning phase (microseconds)
    const bool dbg_plan = ctx->opts.debug_plan;
    using clk = std::chrono::steady_clock;
    clk::time_point tp[8];
    int ntp = 0;
    auto mark = [&]() { if (dbg_plan && ntp < 8) tp[ntp++] = clk::now(); };
    mark();
    ctx->n_chunks = n_chunks;
    ctx->chunks.assign(n_chunks, DevChunk{});
    ctx->pages.clear(); ctx->jobs.clear();
    ctx->l_dictbin.clear(); ctx->l_delta.clear(); ctx->l_count.clear(); ctx->l_scan.clear(); ctx->l_flat.clear(); ctx->l_decode.clear();
    ctx->l_runs.clear(); ctx->l_dlen.clear(); ctx->l_dba.clear(); ctx->l_lvl.clear(); ctx->l_djobs.clear(); ctx->l_cdict.clear();
    ctx->null_dict_lds = 0;
    ctx->null_dcap = ctx->null_icap = 16;
    ctx->l_nest.clear(); ctx->l_nseg.clear();
    // nested pages: entries per segment (k_nest_*); PF_NEST_SEG=n (tests) sets it and sends every
    // eligible nested page, one segment or more, down the segment path (0: none)
    int64_t nest_seg_len = NEST_SEG;
    bool nest_seg_forced = false;
    if (ctx->opts.nest_seg_set) {
        nest_seg_len = ctx->opts.nest_seg;
        nest_seg_forced = nest_seg_len > 0;
        if (nest_seg_len <= 0) nest_seg_len = int64_t(1) << 40;   // every page stays on k_count / k_decode
    }
    ctx->wins.clear(); ctx->pieces.clear(); ctx->n_splits = 0;
    ctx->host_status.assign(n_chunks, 0);
    ctx->info.assign(n_chunks, pf_column_info{});
    ctx->reruns = 0;
    ctx->timing_valid = false;

    // ---- input bytes on device ----
    // stage "h2d" (ev[0] -> ev[1]): the input copy when there is one, the metadata upload and the
    // memsets; for device-resident input it starts at the metadata upload (not before the host plan)
    const bool input_h2d = !bytes_on_device && n_bytes;
    if (input_h2d) EVREC(ctx, ctx->ev[0], st);
    const uint8_t* d_bytes = bytes;
    if (!bytes_on_device && n_bytes) {
        HIPCHK(ctx, ctx->d_in.ensure(n_bytes));
        // pinned pages with a 16-byte aligned device address: read by a kernel (k_download's loop), so the
        // link runs both ways at once beside the downloads (an SDMA H2D waited behind them, r06 trace)
        void* hd = nullptr;
        if (ctx->opts.h2d_kernel && hipHostGetDevicePointer(&hd, const_cast<uint8_t*>(bytes), 0) == hipSuccess && hd &&
            (reinterpret_cast<uintptr_t>(hd) & 15u) == 0) {
            const DlRange r0{static_cast<uint8_t*>(ctx->d_in.p), static_cast<const uint8_t*>(hd), uint64_t(n_bytes)};
            const DlRange rz{nullptr, nullptr, 0};
            hipLaunchKernelGGL(k_download, dim3(ctx->opts.h2d_grid), dim3(256), 0, st, r0, rz, rz);
            HIPCHK(ctx, hipGetLastError());
        } else {
            (void)hipGetLastError();
            HIPCHK(ctx, hipMemcpyAsync(ctx->d_in.p, bytes, n_bytes, hipMemcpyHostToDevice, st));
        }
        d_bytes = static_cast<const uint8_t*>(ctx->d_in.p);
    }
    ctx->d_bytes = d_bytes;

    // ---- plan: sizes of scratch / outputs ----
    struct PagePlan { uint64_t scratch_off; uint64_t aux_off; int is_dict; uint64_t rt_off; uint64_t dx_off; uint64_t lt_off; uint64_t seg_off; int32_t nseg, seg_len, nwin; uint64_t pub_off; uint64_t dbp_off, dbp_pub_off; int32_t dbp_nwin; uint32_t dbp_bcap; };
    std::vector<PagePlan> pplan;
    size_t scratch = 0, out = 0, bits = 0;
    uint64_t nest_pub = 0;
    ctx->max_nwin = 0;
    ctx->max_dbp_nwin = 0;
    // PF_DBP_PAR=0: every DELTA_BINARY_PACKED page on the one-workgroup k_delta (tests)
    const bool dbp_par = ctx->opts.dbp_par;
    uint64_t chars_hint = 0;
    struct OutPlan { size_t values, validity, offsets, list_offsets, list_validity, def, rep; };
    std::vector<OutPlan> oplan(n_chunks);
    auto take = [](size_t& cursor, size_t n, size_t a = 256) { size_t o = align_up(cursor, a); cursor = o + n; return o; };

    for (int c = 0; c < n_chunks; c++) {
        const pf_chunk_desc& cd = cds[c];
        DevChunk& ck = ctx->chunks[c];
        ck.ptype = cd.physical_type; ck.type_length = cd.type_length;
        ck.width = type_width(cd.physical_type, cd.type_length);
        ck.max_def = cd.max_def; ck.max_rep = cd.max_rep; ck.repeated_def = cd.repeated_def;
        ck.list_null_def = cd.list_null_def; ck.codec = cd.codec;
        ck.dict_page = -1;
        ck.first_page = int(ctx->pages.size());
        int64_t& hs = ctx->host_status[c];
        if (ck.width < 0) hs = PF_ERR_UNSUPPORTED_TYPE;
        else if (cd.codec != PF_CODEC_UNCOMPRESSED && cd.codec != PF_CODEC_SNAPPY) hs = PF_ERR_UNSUPPORTED_CODEC;
        else if (cd.max_def < 0 || cd.max_def > 255 || cd.max_rep < 0 || cd.max_rep > 255 || cd.n_pages < 0 ||
                 (cd.n_pages > 0 && !cd.pages) || cd.chunk_offset + cd.chunk_size > n_bytes)
            hs = PF_ERR_INVALID_ARG;
        ck.needs_count = (cd.physical_type == PF_BYTE_ARRAY || cd.max_rep > 0) ? 1 : 0;
        int64_t entries = 0;
        int dict_global = -1;
        if (hs == 0) {
            for (int i = 0; i < cd.n_pages; i++) {
                const pf_page_desc& pd = cd.pages[i];
                if (pd.offset + pd.compressed_size > cd.chunk_size) { hs = PF_ERR_CORRUPT_PAGE; break; }
                if (pd.uncompressed_size > (1u << 29) || pd.compressed_size > (1u << 30)) { hs = PF_ERR_CORRUPT_PAGE; break; }
                bool is_dict = pd.page_type == PF_PAGE_DICTIONARY;
                bool v2 = pd.page_type == PF_PAGE_DATA_V2;
                if (!is_dict && pd.page_type != PF_PAGE_DATA && !v2) continue;   // index pages
                if (is_dict && (dict_global >= 0 || ck.n_pages > 0)) { hs = PF_ERR_CORRUPT_PAGE; break; }
                DevPage pg{};
                pg.chunk = c;
                pg.ba_job = -1;
                pg.encoding = pd.encoding; pg.def_enc = pd.def_encoding; pg.rep_enc = pd.rep_encoding;
                pg.num_values = pd.num_values;
                pg.flags = (v2 ? PG_V2 : 0) | (is_dict ? PG_DICT : 0);
                if (pd.num_values < 0) { hs = PF_ERR_CORRUPT_PAGE; break; }
                const uint8_t* src = d_bytes + cd.chunk_offset + pd.offset;
                uint32_t lvl = v2 ? uint32_t(pd.rep_bytes) + uint32_t(pd.def_bytes) : 0;
                if (v2 && (pd.rep_bytes < 0 || pd.def_bytes < 0 || lvl > pd.compressed_size || lvl > pd.uncompressed_size)) {
                    hs = PF_ERR_CORRUPT_PAGE; break;
                }
                bool compressed = cd.codec == PF_CODEC_SNAPPY && (!v2 || pd.is_compressed);
                PagePlan pp{0, ~0ull, is_dict, ~0ull, ~0ull, ~0ull, ~0ull, 0, 0, 0, 0, ~0ull, 0, 0, 0};
                if (v2) { pg.lvl = src; pg.rep_len = uint32_t(pd.rep_bytes); pg.def_len = uint32_t(pd.def_bytes); }
                if (compressed) {
                    pp.scratch_off = take(scratch, pd.uncompressed_size - lvl, 16);
                    pg.flags |= PG_COMPRESSED;
                    pg.body_len = pd.uncompressed_size - lvl;
                    SnappyJob j{};
                    j.src = src + lvl; j.src_len = pd.compressed_size - lvl; j.dst_len = pd.uncompressed_size - lvl;
                    j.page = int(ctx->pages.size()); j.chunk = c;
                    ctx->jobs.push_back(j);   // dst patched after scratch allocation
                } else {
                    pg.body = src + lvl;
                    pg.body_len = pd.compressed_size - lvl;
                }
                if (is_dict) {
                    dict_global = int(ctx->pages.size());
                    ck.dict_page = dict_global;
                    ck.dict_n = pd.num_values;
                    if (pd.encoding != PF_ENC_PLAIN && pd.encoding != PF_ENC_PLAIN_DICTIONARY) { hs = PF_ERR_UNSUPPORTED_ENCODING; break; }
                    if (cd.physical_type == PF_BOOLEAN) { hs = PF_ERR_UNSUPPORTED_ENCODING; break; }
                    if (cd.physical_type == PF_BYTE_ARRAY) {
                        pp.aux_off = take(scratch, 8ull * (pd.num_values + 1), 256);
                        ctx->l_dictbin.push_back(c);
                    } else if (uint64_t(pd.num_values) * ck.width > pg.body_len) { hs = PF_ERR_CORRUPT_PAGE; break; }
                } else {
                    pg.entry_start = entries;
                    entries += pd.num_values;
                    ck.n_pages++;
                    if (cd.physical_type == PF_BYTE_ARRAY)   // value positions / ids + per-block chars (k_flat)
                        pp.aux_off = take(scratch, 4ull * pd.num_values + 16 + 8ull * (uint64_t(pd.num_values) / FLAT_BLK + 2), 256);
                    else if (pd.encoding == PF_ENC_DELTA_BINARY_PACKED && (cd.physical_type == PF_INT32 || cd.physical_type == PF_INT64)) {
                        pp.aux_off = take(scratch, 8ull * pd.num_values + 8, 256);
                        if (pd.num_values >= DBP_PAR_MIN && dbp_par) {   // block-parallel decode (k_dbp_*)
                            pp.dbp_bcap = uint32_t(pd.num_values / 8 + 2);
                            pp.dbp_off = take(scratch, 12ull * pp.dbp_bcap + 16, 256);
                            pp.dbp_nwin = int32_t((uint64_t(std::max(pd.uncompressed_size, pd.compressed_size)) + DBP_WIN - 1) / DBP_WIN + 1);
                            pp.dbp_pub_off = nest_pub;
                            nest_pub += uint64_t(pp.dbp_nwin) * sizeof(WinPub);
                        }
                    }
                    if (cd.physical_type == PF_BYTE_ARRAY) chars_hint += pd.uncompressed_size;
                    if (cd.physical_type == PF_BYTE_ARRAY &&
                        (pd.encoding == PF_ENC_DELTA_LENGTH_BYTE_ARRAY || pd.encoding == PF_ENC_DELTA_BYTE_ARRAY))
                        pp.dx_off = take(scratch, 8ull * (3ull * uint64_t(pd.num_values) + 1), 256);   // k_dlen
                    if (cd.max_rep == 0 && cd.physical_type != PF_BOOLEAN &&
                        (pd.encoding == PF_ENC_PLAIN_DICTIONARY || pd.encoding == PF_ENC_RLE_DICTIONARY))
                        pp.rt_off = take(scratch, RT_BYTES, 256);   // k_runs table
                    if (cd.max_rep == 0 && cd.max_def > 0 && cd.physical_type != PF_BOOLEAN && cd.physical_type != PF_BYTE_ARRAY &&
                        pd.num_nulls != 0 &&   // v2 header / v1 page statistics say when no level is null (-1: unknown)
                        (pd.encoding == PF_ENC_PLAIN || pd.encoding == PF_ENC_PLAIN_DICTIONARY || pd.encoding == PF_ENC_RLE_DICTIONARY))
                        pp.lt_off = take(scratch, 16 + 16ull * lvl_table_cap(pd.num_values) +
                                                      4ull * LT_BT_WORDS * (uint64_t(pd.num_values) / FLAT_BLK + 1), 256);   // k_lvl tables
                    {   // nested pages decoded in segments (k_nest_*): PLAIN fixed width, dictionary, DELTA_BINARY_PACKED ints
                        const int e = pd.encoding;
                        const bool enc_ok = (e == PF_ENC_PLAIN && cd.physical_type != PF_BYTE_ARRAY) ||
                                            e == PF_ENC_PLAIN_DICTIONARY || e == PF_ENC_RLE_DICTIONARY ||
                                            (e == PF_ENC_DELTA_BINARY_PACKED && (cd.physical_type == PF_INT32 || cd.physical_type == PF_INT64));
                        if (cd.max_rep > 0 && cd.physical_type != PF_BOOLEAN && enc_ok && pd.num_values > 0) {
                            const int64_t sl = std::max<int64_t>(nest_seg_len, (int64_t(pd.num_values) + NEST_MAX_SEGS - 1) / NEST_MAX_SEGS);
                            const int64_t ns = (int64_t(pd.num_values) + sl - 1) / sl;
                            if (ns >= 2 || nest_seg_forced) {
                                pp.seg_len = int32_t(sl);
                                pp.nseg = int32_t(ns);
                                pp.seg_off = take(scratch, nest_seg_bytes(pp.nseg), 256);
                                // windows over the longer level stream (v2: its length is in the header; v1: the page bounds it)
                                const uint64_t lvl_bytes = v2 ? uint64_t(std::max(pd.rep_bytes, pd.def_bytes))
                                                              : uint64_t(std::max(pd.uncompressed_size, pd.compressed_size));
                                pp.nwin = int32_t((lvl_bytes + NEST_WIN - 1) / NEST_WIN + 1);
                                pp.pub_off = nest_pub;   // (the window hand-overs of all pages: one block, zeroed per batch)
                                nest_pub += 2ull * uint64_t(pp.nwin) * sizeof(WinPub);
                            }
                        }
                    }
                }
                pplan.push_back(pp);
                ctx->pages.push_back(pg);
            }
        }
        if (hs != 0) {   // drop this chunk's pages from every list
            while (int(ctx->pages.size()) > ck.first_page) { ctx->pages.pop_back(); pplan.pop_back(); }
            while (!ctx->jobs.empty() && ctx->jobs.back().chunk == c) ctx->jobs.pop_back();
            if (!ctx->l_dictbin.empty() && ctx->l_dictbin.back() == c) ctx->l_dictbin.pop_back();
            ck.n_pages = 0; ck.dict_page = -1; entries = 0;
        }
        if (ck.dict_page >= 0) ck.first_page = ck.dict_page + 1;
        ck.num_entries = entries;
        // outputs
        OutPlan& op = oplan[c];
        op = OutPlan{~size_t(0), ~size_t(0), ~size_t(0), ~size_t(0), ~size_t(0), ~size_t(0), ~size_t(0)};
        if (hs == 0) {
            if (ck.width > 0) op.values = take(out, size_t(entries) * ck.width);
            if (cd.max_def > 0) op.validity = take(bits, align_up((entries + 7) / 8, 4), 256);
            if (cd.physical_type == PF_BYTE_ARRAY) op.offsets = take(out, 4 * size_t(entries + 1));
            if (cd.max_rep == 1) {
                op.list_offsets = take(out, 4 * size_t(entries + 1));
                op.list_validity = take(bits, align_up((entries + 7) / 8, 4), 256);
            }
            if (cd.max_rep > 0) { op.def = take(out, entries); op.rep = take(out, entries); }
        }
    }
    mark();
    // ---- PLAIN BYTE_ARRAY walk jobs: dictionary pages first, then PLAIN data pages ----
    ctx->bajobs.clear();
    ctx->ba_tiles.clear();
    ctx->ba_short_dict = ctx->ba_short_data = true;
    // k_ba_tile links values of up to ~124 bytes within a tile; pages of longer values would all take
    // the exact fallback walk there, so a batch with such pages keeps the multi-kernel walk
    constexpr uint64_t BA_SHORT = 48;
    std::vector<size_t> ba_bm;
    for (int pass = 0; pass < 2; pass++) {
        for (size_t i = 0; i < ctx->pages.size(); i++) {
            DevPage& pg = ctx->pages[i];
            const DevChunk& ck = ctx->chunks[pg.chunk];
            if (ck.ptype != PF_BYTE_ARRAY || ctx->host_status[pg.chunk] != 0) continue;
            const bool is_dict = pg.flags & PG_DICT;
            if (pass == 0 ? !is_dict : (is_dict || pg.encoding != PF_ENC_PLAIN)) continue;
            BaJob J{};
            J.n_cap = pg.body_len;
            J.n_tiles = std::max<uint32_t>(1u, (pg.body_len + BA_TILE_BYTES - 1) / BA_TILE_BYTES);
            J.chunk = pg.chunk;
            J.page = int32_t(i);
            J.state = BA_SKIP;
            const size_t words = size_t(J.n_tiles) * (BA_TILE_BYTES / 32);
            ba_bm.push_back(take(scratch, 4 * (3 * words + J.n_tiles), 256));
            const int rel = int(ctx->bajobs.size()) - (pass == 0 ? 0 : ctx->n_ba_dict);
            for (uint32_t t = 0; t < J.n_tiles; t++) ctx->ba_tiles.push_back(int2{rel, int(t)});
            if (pass == 1) pg.ba_job = int32_t(ctx->bajobs.size());
            if (uint64_t(pg.body_len) > BA_SHORT * uint64_t(std::max<int64_t>(1, pg.num_values)))
                (pass == 0 ? ctx->ba_short_dict : ctx->ba_short_data) = false;
            ctx->bajobs.push_back(J);
        }
        if (pass == 0) { ctx->n_ba_dict = int(ctx->bajobs.size()); ctx->n_ba_dict_tiles = int(ctx->ba_tiles.size()); }
    }
    mark();
    // ---- allocate arenas ----
    size_t chars_cap = std::max<size_t>(size_t(2 * chars_hint) + (16u << 20), ctx->chars_need);
    if (ctx->copies_pending) {
        if (out > ctx->d_out.cap || bits > ctx->d_bits.cap || chars_cap > ctx->d_chars.cap)
            HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));   // a growing output arena must not be freed under a pending D2H copy
        else
            HIPCHK(ctx, hipStreamWaitEvent(st, ctx->ev_copy, 0));   // (a download on the copy stream reads the arenas)
    }
    ctx->copies_pending = false;
    ctx->npub_bytes = size_t(nest_pub);
    ctx->off_npub = take(scratch, ctx->npub_bytes, 256);
    HIPCHK(ctx, ctx->d_scratch.ensure(std::max<size_t>(scratch, 1)));
    HIPCHK(ctx, ctx->d_out.ensure(std::max<size_t>(out, 1)));
    HIPCHK(ctx, ctx->d_bits.ensure(std::max<size_t>(bits, 1)));
    HIPCHK(ctx, ctx->d_chars.ensure(chars_cap));
    ctx->bits_bytes = bits;
    ctx->out_bytes = out;
    uint8_t* S = static_cast<uint8_t*>(ctx->d_scratch.p);
    uint8_t* O = static_cast<uint8_t*>(ctx->d_out.p);
    uint8_t* B = static_cast<uint8_t*>(ctx->d_bits.p);
    {
        size_t ji = 0;
        for (size_t i = 0; i < ctx->pages.size(); i++) {
            DevPage& pg = ctx->pages[i];
            const PagePlan& pp = pplan[i];
            if (pg.flags & PG_COMPRESSED) {
                pg.body = S + pp.scratch_off;
                while (ji < ctx->jobs.size() && ctx->jobs[ji].page != int(i)) ji++;
                if (ji < ctx->jobs.size()) ctx->jobs[ji].dst = S + pp.scratch_off;
            }
            if (pp.aux_off != ~0ull) {
                pg.aux = reinterpret_cast<uint32_t*>(S + pp.aux_off);
                pg.aux_cap = pg.num_values;
            }
            if (pp.rt_off != ~0ull) {
                pg.runtab = reinterpret_cast<uint32_t*>(S + pp.rt_off);
                ctx->l_runs.push_back(int(i));
            }
            if (pp.lt_off != ~0ull) {
                pg.lvltab = reinterpret_cast<uint32_t*>(S + pp.lt_off);
                pg.lvl_cap = lvl_table_cap(pg.num_values);
                ctx->l_lvl.push_back(int(i));
                const DevChunk& lc = ctx->chunks[size_t(pg.chunk)];
                const uint64_t db = uint64_t(std::max<int64_t>(lc.dict_n, 0)) * uint64_t(std::max(lc.width, 0));
                if (lc.dict_page >= 0 && db > 0 && db <= NULL_DICT_LDS)
                    ctx->null_dict_lds = std::max(ctx->null_dict_lds, uint32_t(align_up(db, 256)));
                // level / id byte stages: FBLK values of the level width / the dictionary's id width
                // (bit width of its largest index, as writers choose it) + run headers
                auto bits = [](uint64_t v) { int b = 0; while (v) { b++; v >>= 1; } return b; };
                // hybrid worst case: bit-packed, FLAT_BLK * b / 8 bytes + headers; or RLE runs of
                // 8 repeats, a header byte + ceil(b / 8) value bytes per 8 entries (1-bit levels: 1 KiB)
                auto cap = [](int b, uint32_t most) {
                    const uint64_t bp = uint64_t(FLAT_BLK) * uint64_t(b) / 8;
                    const uint64_t rle = uint64_t(FLAT_BLK) / 8 * (1 + (uint64_t(b) + 7) / 8);
                    return uint32_t(std::min<uint64_t>(most, align_up(std::max(bp, rle) + NL_SLACK, 16)));
                };
                ctx->null_dcap = std::max(ctx->null_dcap, cap(bits(uint64_t(std::max(lc.max_def, 0))), NL_DST));
                if (lc.dict_page >= 0)
                    ctx->null_icap = std::max(ctx->null_icap, cap(bits(uint64_t(std::max<int64_t>(lc.dict_n, 1) - 1)), NL_IST));
            }
            if (pp.dbp_off != ~0ull) {
                pg.dbp = S + pp.dbp_off;
                pg.dbp_pub = reinterpret_cast<WinPub*>(S + ctx->off_npub + pp.dbp_pub_off);
                pg.dbp_nwin = pp.dbp_nwin;
                pg.dbp_bcap = pp.dbp_bcap;
                ctx->max_dbp_nwin = std::max(ctx->max_dbp_nwin, pp.dbp_nwin);
            }
            if (pp.seg_off != ~0ull) {
                pg.seg = S + pp.seg_off;
                pg.nseg = pp.nseg;
                pg.seg_len = pp.seg_len;
                pg.nwin = pp.nwin;
                pg.npub = reinterpret_cast<WinPub*>(S + ctx->off_npub + pp.pub_off);
                ctx->max_nwin = std::max(ctx->max_nwin, pp.nwin);
                ctx->l_nest.push_back(int(i));
                for (int k = 0; k < pp.nseg; k++) { ctx->l_nseg.push_back(int(i)); ctx->l_nseg.push_back(k); }
            }
            if (pp.dx_off != ~0ull) {
                pg.dx = reinterpret_cast<uint64_t*>(S + pp.dx_off);
                ctx->l_dlen.push_back(int(i));
                if (pg.encoding == PF_ENC_DELTA_BYTE_ARRAY) ctx->l_dba.push_back(int(i));
            }
            DevChunk& ck = ctx->chunks[pg.chunk];
            if (pp.is_dict) {
                ck.dict_data = pg.body;
                if (ck.ptype == PF_BYTE_ARRAY) {
                    ck.dict_pos = reinterpret_cast<uint32_t*>(S + pp.aux_off);
                    ck.dict_len = ck.dict_pos + (pg.num_values + 1);
                }
            }
        }
    }
    for (size_t b = 0; b < ctx->bajobs.size(); b++) {
        BaJob& J = ctx->bajobs[b];
        const size_t words = size_t(J.n_tiles) * (BA_TILE_BYTES / 32);
        J.cand = reinterpret_cast<uint32_t*>(S + ba_bm[b]);
        J.link1 = J.cand + words;
        J.link2 = J.link1 + words;
        J.tile_cnt = J.link2 + words;
        const DevPage& pg = ctx->pages[J.page];
        if (int(b) < ctx->n_ba_dict) {
            const DevChunk& ck = ctx->chunks[J.chunk];
            J.p = pg.body;
            J.n = pg.body_len;
            J.count = ck.dict_n;
            J.pos = ck.dict_pos;
            J.len = ck.dict_len;
            J.state = ck.dict_n > 0 ? BA_OK : BA_SKIP;
        } else {
            J.pos = pg.aux;   // p, n, count, state: k_count
        }
    }
    for (int c = 0; c < n_chunks; c++) {
        DevChunk& ck = ctx->chunks[c];
        const OutPlan& op = oplan[c];
        auto at = [](uint8_t* base, size_t off) { return off == ~size_t(0) ? nullptr : base + off; };
        ck.values = at(O, op.values);
        ck.validity = at(B, op.validity);
        ck.offsets = reinterpret_cast<int32_t*>(at(O, op.offsets));
        ck.list_offsets = reinterpret_cast<int32_t*>(at(O, op.list_offsets));
        ck.list_validity = at(B, op.list_validity);
        ck.def_levels = at(O, op.def);
        ck.rep_levels = at(O, op.rep);
        if (ctx->host_status[c] == 0) {
            if (ck.needs_count) ctx->l_scan.push_back(c);
        }
    }
    // (page, block) pairs of the flat kernels. A chunk with a large dictionary keeps all its blocks on
    // one blockIdx % 8 label (the dispatcher's XCD group, MI355X_MICROARCH.md), so the dictionary is
    // gathered through one XCD's L2 instead of all eight (config 4: 400 KB dictionaries); such chunks
    // go to the least loaded label, all other blocks then fill the labels evenly. Labels are
    // interleaved into the grid; short ones are padded with (-1, 0).
    // Four such grids, one after the other in l_flat: fixed-width pages (k_flat_fixed), the other flat
    // pages (k_flat_all), then the blocks of nullable 4- and 8-byte pages (k_flat_null<4> / <8>);
    // k_flat_fixed and k_flat_null queue what they do not take for k_flat_all's last workgroups.
    constexpr uint32_t STICKY_DICT = 64u << 10;
    std::vector<int> spread[4];
    std::vector<std::vector<int>> sticky[4];
    for (auto& v : sticky) v.resize(static_cast<size_t>(n_chunks));
    std::vector<int> decode_first, count_rest;
    for (size_t i = 0; i < ctx->pages.size(); i++) {
        const DevPage& pg = ctx->pages[i];
        if (pg.flags & PG_DICT) continue;
        const DevChunk& ck = ctx->chunks[pg.chunk];
        if (pg.encoding == PF_ENC_DELTA_BINARY_PACKED && pg.aux && ck.ptype != PF_BYTE_ARRAY) ctx->l_delta.push_back(int(i));
        if (ck.needs_count) (ck.ptype == PF_BYTE_ARRAY && ck.max_rep == 0 ? ctx->l_count : count_rest).push_back(int(i));
        if (ck.ptype == PF_BYTE_ARRAY && ck.max_rep == 0 && pg.runtab != nullptr &&
            (pg.encoding == PF_ENC_PLAIN_DICTIONARY || pg.encoding == PF_ENC_RLE_DICTIONARY)) {
            const int nb = std::max(1, int((int64_t(pg.num_values) + FLAT_BLK - 1) / FLAT_BLK));
            for (int b = 0; b < nb; b++) { ctx->l_cdict.push_back(int(i)); ctx->l_cdict.push_back(b); }
        }
        if (ck.max_rep == 0) {   // (page, block) pairs
            // fixed-width pages without a level table (no nulls) take blocks of FLAT_BLK << fix_shift
            // entries (the block index carries the shift in bits 28..31): a block's metadata chain and
            // run-table load are paid once per 8192 entries instead of per 4096 (PF_FIX_BLK=4096|8192|16384)
            const int fix_shift = ctx->opts.fix_shift;
            const int sh = (ck.ptype != PF_BYTE_ARRAY && pg.lvltab == nullptr) ? fix_shift : 0;
            const int64_t bsz = FLAT_BLK << sh;
            const int nb = std::max(1, int((int64_t(pg.num_values) + bsz - 1) / bsz));
            const bool dict_enc = pg.encoding == PF_ENC_PLAIN_DICTIONARY || pg.encoding == PF_ENC_RLE_DICTIONARY;
            const bool big_dict = ck.dict_page >= 0 && ctx->pages[size_t(ck.dict_page)].body_len > STICKY_DICT && dict_enc;
            const int grid = (pg.lvltab != nullptr && ck.ptype != PF_BYTE_ARRAY && (dict_enc || pg.encoding == PF_ENC_PLAIN))
                                 ? (ck.width == 4 ? 2 : (ck.width == 8 ? 3 : 1))
                                 : (ck.ptype != PF_BYTE_ARRAY ? 0 : 1);
            std::vector<int>& q = big_dict ? sticky[grid][size_t(pg.chunk)] : spread[grid];
            for (int b = 0; b < nb; b++) { q.push_back(int(i)); q.push_back(b | (sh << 28)); }
        }
        // k_decode does the pages the flat kernels do not take: nested pages and encodings other than
        // PLAIN / dictionary / DELTA_BINARY_PACKED go first (one block each), the rest are only checked
        const int e = pg.encoding;
        if (ck.max_rep > 0 || !(e == PF_ENC_PLAIN || e == PF_ENC_PLAIN_DICTIONARY || e == PF_ENC_RLE_DICTIONARY ||
                                e == PF_ENC_DELTA_BINARY_PACKED) || ck.ptype == PF_BOOLEAN)
            decode_first.push_back(int(i));
        else
            ctx->l_decode.push_back(int(i));
    }
    ctx->n_decode_first = int(decode_first.size());
    ctx->n_count_flat = int(ctx->l_count.size());
    ctx->l_count.insert(ctx->l_count.end(), count_rest.begin(), count_rest.end());
    ctx->l_decode.insert(ctx->l_decode.begin(), decode_first.begin(), decode_first.end());
    int n_grid[4] = {};
    for (int gi = 0; gi < 4; gi++) {
        std::vector<int> xq[8];
        size_t load[8] = {};
        std::vector<int> order(static_cast<size_t>(n_chunks));
        for (int c = 0; c < n_chunks; c++) order[size_t(c)] = c;
        const auto& sk = sticky[gi];
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return sk[size_t(a)].size() > sk[size_t(b)].size(); });
        for (int c : order) {
            if (sk[size_t(c)].empty()) continue;
            const int x = int(std::min_element(load, load + 8) - load);
            xq[x].insert(xq[x].end(), sk[size_t(c)].begin(), sk[size_t(c)].end());
            load[x] += sk[size_t(c)].size() / 2;
        }
        const std::vector<int>& sp = spread[gi];
        for (size_t k = 0; k + 1 < sp.size(); k += 2) {
            const int x = int(std::min_element(load, load + 8) - load);
            xq[x].push_back(sp[k]);
            xq[x].push_back(sp[k + 1]);
            load[x]++;
        }
        const size_t longest = *std::max_element(load, load + 8);
        for (size_t k = 0; k < longest; k++)
            for (int x = 0; x < 8; x++) {
                const bool have = k < load[x];
                ctx->l_flat.push_back(have ? xq[x][2 * k] : -1);
                ctx->l_flat.push_back(have ? xq[x][2 * k + 1] : 0);
            }
        n_grid[gi] = int(8 * longest);
    }
    ctx->n_flat_fixed = n_grid[0];
    ctx->n_flat_all = n_grid[1];
    ctx->n_null4 = n_grid[2];
    ctx->n_null8 = n_grid[3];
    mark();
    // k_snappy_litcopy candidates (k_snappy_head decides): dictionary pages, and data pages that did
    // not compress (a stream of literals only; one literal is read in place instead)
    for (size_t j = 0; j < ctx->jobs.size(); j++) {
        SnappyJob& jb = ctx->jobs[j];
        if ((ctx->pages[size_t(jb.page)].flags & PG_DICT) || jb.src_len >= jb.dst_len) {
            jb.dflags |= 2u;
            ctx->l_djobs.push_back(int(j));
        }
    }
    // ---- Snappy tables: 8 KiB index windows, 64 KiB pieces ----
    {
        int rc = plan_snappy(ctx);
        if (rc) return rc;
    }
    mark();
    // ---- metadata upload ----
    size_t m = 0;
    ctx->off_chunks = take(m, sizeof(DevChunk) * n_chunks);
    ctx->off_pages = take(m, sizeof(DevPage) * ctx->pages.size());
    ctx->off_jobs = take(m, sizeof(SnappyJob) * ctx->jobs.size());
    ctx->off_lists = take(m, sizeof(int) * (ctx->l_dictbin.size() + ctx->l_delta.size() + ctx->l_count.size() +
                                            ctx->l_scan.size() + ctx->l_flat.size() + ctx->l_decode.size() + ctx->l_runs.size() +
                                            ctx->l_dlen.size() + ctx->l_dba.size() + ctx->l_lvl.size() + ctx->l_djobs.size() +
                                            ctx->l_nest.size() + ctx->l_nseg.size() + ctx->l_cdict.size()));
    ctx->off_res = take(m, sizeof(DevChunkResult) * n_chunks);
    ctx->off_pieces = take(m, sizeof(int2) * ctx->pieces.size());
    ctx->off_splits = take(m, sizeof(uint32_t) * ctx->n_splits);
    ctx->off_fallback = take(m, sizeof(int) * ctx->jobs.size());
    ctx->off_wins = take(m, sizeof(int2) * ctx->wins.size());
    ctx->off_bajobs = take(m, sizeof(BaJob) * ctx->bajobs.size());
    ctx->off_batiles = take(m, sizeof(int2) * ctx->ba_tiles.size());
    ctx->off_nfbq = take(m, 16 + sizeof(int2) * size_t(ctx->n_flat_fixed + ctx->n_null4 + ctx->n_null8), 16);   // fallback queue
    m = take(m, 256) + 256;   // arena counter lives in the last 256 bytes
    ctx->meta_bytes = m;
    HIPCHK(ctx, ctx->d_meta.ensure(m));
    HIPCHK(ctx, ctx->h_meta.ensure(m));
    {   // each Snappy data page reads its job's fallback flag (k_flat_fixed: were the values written direct?)
        const int* d_fb = reinterpret_cast<const int*>(static_cast<uint8_t*>(ctx->d_meta.p) + ctx->off_fallback);
        for (size_t j = 0; j < ctx->jobs.size(); j++) ctx->pages[size_t(ctx->jobs[j].page)].jfb = d_fb + j;
    }
    HIPCHK(ctx, ctx->h_res.ensure(align_up(sizeof(DevChunkResult) * n_chunks, 256) + sizeof(DevChunk) * n_chunks + 256));
    if (!input_h2d) EVREC(ctx, ctx->ev[0], st);
    int rc = upload_meta(ctx);
    if (rc) return rc;
    mark();
    rc = enqueue_kernels(ctx);
    if (rc) return rc;
    mark();
    if (dbg_plan) {
        auto us = [&](int a, int b) { return long(std::chrono::duration_cast<std::chrono::microseconds>(tp[b] - tp[a]).count()); };
        std::fprintf(stderr, "[pf plan] chunks %d pages %zu jobs %zu wins %zu | pages %ld ba %ld alloc+lists %ld snappy %ld meta %ld launch %ld us\n",
                     n_chunks, ctx->pages.size(), ctx->jobs.size(), ctx->wins.size(), us(0, 1), us(1, 2), us(2, 3), us(3, 4),
                     us(4, 5), us(5, 6));
    }
    ctx->pending = true;
    ctx->tables_from_decode = true;
    return PF_OK;
}

int pf_wait(pf_ctx* ctx) {
    if (!ctx) return fail(nullptr, PF_ERR_INVALID_ARG, "null ctx");
    if (!ctx->pending) return fail(ctx, PF_ERR_STATE, "nothing to wait for");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    for (;;) {
        hipError_t e = hipEventSynchronize(ctx->ev_done);
        if (e != hipSuccess) { ctx->pending = false; return fail(ctx, PF_ERR_HIP, std::string("decode: ") + hipGetErrorString(e)); }
        const DevChunkResult* r = static_cast<const DevChunkResult*>(ctx->h_res.p);
        const DevChunk* dc = reinterpret_cast<const DevChunk*>(static_cast<uint8_t*>(ctx->h_res.p) +
                                                               align_up(sizeof(DevChunkResult) * ctx->n_chunks, 256));
        // chars arena overflow: grow to the exact need and run the batch once more
        uint64_t need = 0;
        bool overflow = false;
        for (int c = 0; c < ctx->n_chunks; c++) {
            if (ctx->chunks[c].ptype == PF_BYTE_ARRAY) need += align_up(uint64_t(std::max<int64_t>(r[c].num_chars, 0)), 256);
            if (r[c].status == PF_ERR_CAPACITY && ctx->chunks[c].ptype == PF_BYTE_ARRAY && r[c].num_chars <= 0x7fffffff)
                overflow = true;
        }
        if (overflow && ctx->reruns == 0) {
            ctx->reruns++;
            ctx->chars_need = size_t(need) + (1u << 20);
            HIPCHK(ctx, ctx->d_chars.ensure(ctx->chars_need));
            int rc = upload_meta(ctx);
            if (rc) { ctx->pending = false; return rc; }
            rc = enqueue_kernels(ctx);
            if (rc) { ctx->pending = false; return rc; }
            continue;
        }
        int first_err = PF_OK;
        for (int c = 0; c < ctx->n_chunks; c++) {
            pf_column_info& ci = ctx->info[c];
            const DevChunk& ck = ctx->chunks[c];
            ci.num_entries = ck.num_entries;
            ci.num_slots = r[c].num_slots;
            ci.num_values = r[c].num_values;
            ci.num_rows = r[c].num_rows;
            ci.num_chars = ck.ptype == PF_BYTE_ARRAY ? r[c].num_chars : 0;
            ci.width = ck.width;
            ci.status = r[c].status;
            ci.d_values = ck.values;
            ci.d_validity = ck.validity;
            ci.d_offsets = ck.offsets;
            ci.d_chars = dc[c].chars;
            ci.d_list_offsets = ck.list_offsets;
            ci.d_list_validity = ck.list_validity;
            ci.d_def_levels = ck.def_levels;
            ci.d_rep_levels = ck.rep_levels;
            if (ci.status != 0 && first_err == PF_OK) {
                first_err = ci.status;
                char buf[160];
                std::snprintf(buf, sizeof buf, "chunk %d: decode failed (status %d, page %d)", c, ci.status, r[c].err_page);
                fail(ctx, first_err, buf);
            }
        }
        ctx->pending = false;
        ctx->timing_valid = true;
        return first_err;
    }
}

int pf_column_info_get(pf_ctx* ctx, int chunk, pf_column_info* out) {
    if (!ctx || !out) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    if (chunk < 0 || chunk >= ctx->n_chunks) return fail(ctx, PF_ERR_INVALID_ARG, "chunk index out of range");
    *out = ctx->info[chunk];
    return PF_OK;
}

namespace {
// Enqueue the D2H copies of chunk i's arrays on the context stream (no synchronisation).
int enqueue_copy(pf_ctx* ctx, int chunk, const pf_column_out* o) {
    if (!ctx || !o) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    if (chunk < 0 || chunk >= ctx->n_chunks) return fail(ctx, PF_ERR_INVALID_ARG, "chunk index out of range");
    const pf_column_info& ci = ctx->info[chunk];
    if (ci.status != 0) return fail(ctx, ci.status, "chunk failed to decode");
    struct Item { void* dst; size_t cap; const void* src; size_t n; };
    Item items[8] = {
        {o->values, o->values_cap, ci.d_values, size_t(ci.num_slots) * size_t(ci.width)},
        {o->validity, o->validity_cap, ci.d_validity, size_t((ci.num_slots + 7) / 8)},
        {o->offsets, o->offsets_cap, ci.d_offsets, ci.d_offsets ? 4 * size_t(ci.num_slots + 1) : 0},
        {o->chars, o->chars_cap, ci.d_chars, size_t(ci.num_chars)},
        {o->list_offsets, o->list_offsets_cap, ci.d_list_offsets, ci.d_list_offsets ? 4 * size_t(ci.num_rows + 1) : 0},
        {o->list_validity, o->list_validity_cap, ci.d_list_validity, size_t((ci.num_rows + 7) / 8)},
        {o->def_levels, o->def_levels_cap, ci.d_def_levels, size_t(ci.num_entries)},
        {o->rep_levels, o->rep_levels_cap, ci.d_rep_levels, size_t(ci.num_entries)},
    };
    for (const Item& it : items)
        if (it.dst && it.src && it.n > it.cap) return fail(ctx, PF_ERR_CAPACITY, "output buffer too small");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    for (const Item& it : items)
        if (it.dst && it.src && it.n) HIPCHK(ctx, hipMemcpyAsync(it.dst, it.src, it.n, hipMemcpyDeviceToHost, ctx->stream));
    return PF_OK;
}
}  // namespace

int pf_copy_column(pf_ctx* ctx, int chunk, const pf_column_out* o) {
    const int rc = enqueue_copy(ctx, chunk, o);
    if (rc) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev_copy, ctx->stream));
    HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));
    return PF_OK;
}

int pf_copy_columns_async(pf_ctx* ctx, int n, const int* chunks, const pf_column_out* outs) {
    if (!ctx || n < 0 || (n > 0 && (!chunks || !outs))) return fail(ctx, PF_ERR_INVALID_ARG, "bad arguments");
    for (int i = 0; i < n; i++) {   // capacities first: nothing is enqueued if any buffer is too small
        if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
        const int c = chunks[i];
        if (c < 0 || c >= ctx->n_chunks) return fail(ctx, PF_ERR_INVALID_ARG, "chunk index out of range");
        const pf_column_info& ci = ctx->info[c];
        if (ci.status != 0) return fail(ctx, ci.status, "chunk failed to decode");
        const pf_column_out& o = outs[i];
        const size_t need[8] = {size_t(ci.num_slots) * size_t(ci.width), size_t((ci.num_slots + 7) / 8),
                                ci.d_offsets ? 4 * size_t(ci.num_slots + 1) : 0, size_t(ci.num_chars),
                                ci.d_list_offsets ? 4 * size_t(ci.num_rows + 1) : 0, size_t((ci.num_rows + 7) / 8),
                                size_t(ci.num_entries), size_t(ci.num_entries)};
        const void* dst[8] = {o.values, o.validity, o.offsets, o.chars, o.list_offsets, o.list_validity, o.def_levels,
                              o.rep_levels};
        const void* src[8] = {ci.d_values, ci.d_validity, ci.d_offsets, ci.d_chars, ci.d_list_offsets, ci.d_list_validity,
                              ci.d_def_levels, ci.d_rep_levels};
        const size_t cap[8] = {o.values_cap, o.validity_cap, o.offsets_cap, o.chars_cap, o.list_offsets_cap,
                               o.list_validity_cap, o.def_levels_cap, o.rep_levels_cap};
        for (int k = 0; k < 8; k++)
            if (dst[k] && src[k] && need[k] > cap[k]) return fail(ctx, PF_ERR_CAPACITY, "output buffer too small");
    }
    for (int i = 0; i < n; i++) {
        const int rc = enqueue_copy(ctx, chunks[i], &outs[i]);
        if (rc) return rc;
    }
    if (n > 0) {
        HIPCHK(ctx, hipEventRecord(ctx->ev_copy, ctx->stream));
        ctx->copies_pending = true;
    }
    return PF_OK;
}

namespace {
// Host layout of pf_copy_batch_async: [out arena | bits arena | chars arena], each 256-B aligned.
struct BatchLayout { size_t out, bits_off, bits, chars_off, chars, total; };
BatchLayout batch_layout(const pf_ctx* ctx) {
    BatchLayout b{};
    b.out = ctx->out_bytes;
    b.bits_off = align_up(b.out, 256);
    b.bits = ctx->bits_bytes;
    b.chars_off = align_up(b.bits_off + b.bits, 256);
    const uint8_t* c0 = static_cast<const uint8_t*>(ctx->d_chars.p);
    size_t hi = 0, bound = 0;
    for (int c = 0; c < ctx->n_chunks && c < int(ctx->info.size()); c++) {
        const pf_column_info& ci = ctx->info[c];
        if (ci.d_chars && ci.num_chars > 0) {
            hi = std::max(hi, size_t(static_cast<const uint8_t*>(ci.d_chars) - c0) + size_t(ci.num_chars));
            bound += align_up(size_t(ci.num_chars), 256);
        }
    }
    b.chars = hi;   // bytes copied: the arena's used extent (depends on the order k_scan placed the chunks)
    // buffer size: an order-independent bound, so equal batches always need equal buffers
    b.total = b.chars_off + std::max(hi, bound);
    return b;
}
}  // namespace

int pf_batch_bytes(pf_ctx* ctx, size_t* bytes) {
    if (!ctx || !bytes) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    if (!ctx->tables_from_decode) return fail(ctx, PF_ERR_STATE, "no finished decode");
    *bytes = batch_layout(ctx).total;
    return PF_OK;
}

int pf_copy_batch_async(pf_ctx* ctx, void* host, size_t cap) {
    if (!ctx || (!host && cap)) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    if (!ctx->tables_from_decode) return fail(ctx, PF_ERR_STATE, "no finished decode");
    const BatchLayout b = batch_layout(ctx);
    if (b.total > cap) return fail(ctx, PF_ERR_CAPACITY, "batch buffer too small (pf_batch_bytes)");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    uint8_t* h = static_cast<uint8_t*>(host);
    // pinned pages with a device address: k_download; otherwise (or PF_DL_KERNEL=0) SDMA copies
    void* hd = nullptr;
    if (ctx->opts.dl_kernel && (b.out || b.bits || b.chars)) {
        if (hipHostGetDevicePointer(&hd, host, 0) != hipSuccess || !hd || (reinterpret_cast<uintptr_t>(hd) & 15u) != 0) {
            (void)hipGetLastError();   // (not a mapped pinned buffer: the copy path)
            hd = nullptr;
        }
    }
    hipStream_t cs = ctx->stream;
    if (ctx->opts.dl_stream) {   // the download on the copy stream, after this context's decode
        {
            std::lock_guard<std::mutex> lk(ctx->streams->mu);
            if (!ctx->streams->copy_stream) {
                int least = 0, greatest = 0;
                if (ctx->opts.dl_prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
                    HIPCHK(ctx, hipStreamCreateWithPriority(&ctx->streams->copy_stream, hipStreamNonBlocking, greatest));
                else
                    HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->streams->copy_stream, hipStreamNonBlocking));
            }
        }
        cs = ctx->streams->copy_stream;
        HIPCHK(ctx, hipEventRecord(ctx->ev_dl, ctx->stream));
        HIPCHK(ctx, hipStreamWaitEvent(cs, ctx->ev_dl, 0));
    }
    if (hd) {
        uint8_t* hdev = static_cast<uint8_t*>(hd);
        const DlRange r0{hdev, static_cast<const uint8_t*>(ctx->d_out.p), b.out};
        const DlRange r1{hdev + b.bits_off, static_cast<const uint8_t*>(ctx->d_bits.p), b.bits};
        const DlRange r2{hdev + b.chars_off, static_cast<const uint8_t*>(ctx->d_chars.p), b.chars};
        hipLaunchKernelGGL(k_download, dim3(256), dim3(256), 0, cs, r0, r1, r2);
        HIPCHK(ctx, hipGetLastError());
    } else {
        if (b.out) HIPCHK(ctx, hipMemcpyAsync(h, ctx->d_out.p, b.out, hipMemcpyDeviceToHost, cs));
        if (b.bits) HIPCHK(ctx, hipMemcpyAsync(h + b.bits_off, ctx->d_bits.p, b.bits, hipMemcpyDeviceToHost, cs));
        if (b.chars) HIPCHK(ctx, hipMemcpyAsync(h + b.chars_off, ctx->d_chars.p, b.chars, hipMemcpyDeviceToHost, cs));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev_copy, cs));
    ctx->copies_pending = true;
    return PF_OK;
}

int pf_column_info_host(pf_ctx* ctx, int chunk, const void* host, pf_column_info* out) {
    if (!ctx || !out || !host) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    if (chunk < 0 || chunk >= ctx->n_chunks) return fail(ctx, PF_ERR_INVALID_ARG, "chunk index out of range");
    const BatchLayout b = batch_layout(ctx);
    const uint8_t* h = static_cast<const uint8_t*>(host);
    auto rebase = [&](const void* p) -> const void* {
        if (!p) return nullptr;
        const uint8_t* q = static_cast<const uint8_t*>(p);
        const uint8_t* o = static_cast<const uint8_t*>(ctx->d_out.p);
        const uint8_t* v = static_cast<const uint8_t*>(ctx->d_bits.p);
        const uint8_t* c = static_cast<const uint8_t*>(ctx->d_chars.p);
        if (q >= o && q <= o + b.out) return h + (q - o);
        if (q >= v && q <= v + b.bits) return h + b.bits_off + (q - v);
        if (q >= c && q <= c + b.chars) return h + b.chars_off + (q - c);
        return nullptr;
    };
    pf_column_info ci = ctx->info[chunk];
    ci.d_values = rebase(ci.d_values);
    ci.d_validity = static_cast<const uint8_t*>(rebase(ci.d_validity));
    ci.d_offsets = static_cast<const int32_t*>(rebase(ci.d_offsets));
    ci.d_chars = static_cast<const uint8_t*>(rebase(ci.d_chars));
    ci.d_list_offsets = static_cast<const int32_t*>(rebase(ci.d_list_offsets));
    ci.d_list_validity = static_cast<const uint8_t*>(rebase(ci.d_list_validity));
    ci.d_def_levels = static_cast<const uint8_t*>(rebase(ci.d_def_levels));
    ci.d_rep_levels = static_cast<const uint8_t*>(rebase(ci.d_rep_levels));
    *out = ci;
    return PF_OK;
}

int pf_sync(pf_ctx* ctx) {
    if (!ctx) return fail(nullptr, PF_ERR_INVALID_ARG, "null ctx");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (ctx->copies_pending) HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));   // this context's copies only
    ctx->copies_pending = false;
    return PF_OK;
}

int pf_snappy_decompress(pf_ctx* ctx, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    if (!ctx || (!src && n) || !out_len) return fail(ctx, PF_ERR_INVALID_ARG, "null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "previous decode not waited for");
    uint64_t ulen = 0;
    size_t p = 0;
    for (int sh = 0;; sh += 7) {
        if (p >= n || sh > 28) return fail(ctx, PF_ERR_CORRUPT_PAGE, "snappy: bad length preamble");
        uint8_t c = src[p++];
        ulen |= uint64_t(c & 0x7f) << sh;
        if (!(c & 0x80)) break;
    }
    *out_len = size_t(ulen);
    if (ulen > cap) return fail(ctx, PF_ERR_CAPACITY, "snappy: destination too small");
    if (n > 0xffffffffull || ulen > 0xffffffffull) return fail(ctx, PF_ERR_INVALID_ARG, "snappy: buffer too large");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (ctx->copies_pending) HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));   // arenas may be reallocated below
    ctx->copies_pending = false;
    ctx->n_chunks = 0;
    ctx->info.clear();
    ctx->tables_from_decode = false;   // d_meta now holds this call's layout
    HIPCHK(ctx, ctx->d_in.ensure(std::max<size_t>(n, 1)));
    HIPCHK(ctx, ctx->d_scratch.ensure(std::max<size_t>(ulen, 1) + 16));
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_in.p, src, n, hipMemcpyHostToDevice, st));
    SnappyJob job{};
    job.src = static_cast<const uint8_t*>(ctx->d_in.p);
    job.dst = static_cast<uint8_t*>(ctx->d_scratch.p);
    job.src_len = uint32_t(n);
    job.dst_len = uint32_t(ulen);
    ctx->jobs.assign(1, job);
    ctx->chunks.clear();
    ctx->pages.clear();
    int rc = plan_snappy(ctx);
    if (rc) return rc;
    size_t m = 0;
    auto take = [](size_t& cursor, size_t sz) { size_t o = align_up(cursor, 256); cursor = o + sz; return o; };
    size_t o_job = take(m, sizeof(SnappyJob)), o_pc = take(m, sizeof(int2) * ctx->pieces.size());
    size_t o_sp = take(m, 4 * ctx->pieces.size()), o_fb = take(m, 4), o_wn = take(m, sizeof(int2) * ctx->wins.size());
    size_t o_res = take(m, sizeof(DevChunkResult));
    m = align_up(m, 256);
    HIPCHK(ctx, ctx->d_meta.ensure(m));
    HIPCHK(ctx, ctx->h_meta.ensure(m));
    uint8_t* h = static_cast<uint8_t*>(ctx->h_meta.p);
    std::memset(h, 0, m);
    std::memcpy(h + o_job, ctx->jobs.data(), sizeof(SnappyJob));
    std::memcpy(h + o_pc, ctx->pieces.data(), sizeof(int2) * ctx->pieces.size());
    std::memset(h + o_sp, 0xff, 4 * ctx->pieces.size());
    std::memcpy(h + o_wn, ctx->wins.data(), sizeof(int2) * ctx->wins.size());
    uint8_t* d = static_cast<uint8_t*>(ctx->d_meta.p);
    HIPCHK(ctx, hipMemcpyAsync(d, h, m, hipMemcpyHostToDevice, st));
    ctx->d_last_splits = reinterpret_cast<const uint32_t*>(d + o_sp);
    launch_snappy(reinterpret_cast<const SnappyJob*>(d + o_job), 1, reinterpret_cast<const int2*>(d + o_wn),
                  int(ctx->wins.size()), ctx->d_win, ctx->d_ent, ctx->d_lane_out, reinterpret_cast<const int2*>(d + o_pc),
                  int(ctx->pieces.size()), reinterpret_cast<uint32_t*>(d + o_sp), reinterpret_cast<int*>(d + o_fb),
                  reinterpret_cast<DevChunkResult*>(d + o_res), int(ctx->jobs.empty() ? 1 : ctx->jobs[0].n_win),
                  ctx->opts.exec, st);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, ctx->h_res.ensure(512));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_res.p, d + o_res, sizeof(DevChunkResult), hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(static_cast<uint8_t*>(ctx->h_res.p) + 256, d + o_fb, 4, hipMemcpyDeviceToHost, st));
    if (ulen) HIPCHK(ctx, hipMemcpyAsync(dst, ctx->d_scratch.p, ulen, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    const DevChunkResult* r = static_cast<const DevChunkResult*>(ctx->h_res.p);
    if (r->status != 0) return fail(ctx, r->status, "snappy: corrupt input");
    return PF_OK;
}

// GPU page-header scan (pfloor.h): k_page_scan per chunk, then k_page_crc over the pages found.
int pf_scan_pages(pf_ctx* ctx, const pf_scan_chunk* chunks, int n_chunks, const uint8_t* bytes, size_t n_bytes,
                  int bytes_on_device, int verify_crc, pf_page_desc* pages_out, pf_scan_result* results) {
    if (!ctx || n_chunks < 0 || (n_chunks && (!chunks || !results || !pages_out)) || (!bytes && n_bytes))
        return fail(ctx, PF_ERR_INVALID_ARG, "scan: null arg");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "previous decode not waited for");
    if (n_chunks == 0) return PF_OK;
    int64_t slots = 0;
    for (int c = 0; c < n_chunks; c++) {
        const pf_scan_chunk& k = chunks[c];
        if (k.page_base < 0 || k.page_cap < 0 || k.chunk_offset > n_bytes || k.chunk_size > n_bytes - k.chunk_offset)
            return fail(ctx, PF_ERR_INVALID_ARG, "scan: chunk " + std::to_string(c) + " outside the buffer / bad slots");
        slots = std::max<int64_t>(slots, int64_t(k.page_base) + k.page_cap);
    }
    if (slots > (int64_t(1) << 30)) return fail(ctx, PF_ERR_INVALID_ARG, "scan: too many page slots");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (ctx->copies_pending) HIPCHK(ctx, hipEventSynchronize(ctx->ev_copy));
    ctx->copies_pending = false;
    const uint8_t* d_bytes = bytes;
    if (!bytes_on_device && n_bytes) {
        HIPCHK(ctx, ctx->d_scan_in.ensure(n_bytes));
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_scan_in.p, bytes, n_bytes, hipMemcpyHostToDevice, st));
        d_bytes = static_cast<const uint8_t*>(ctx->d_scan_in.p);
    }
    size_t m = 0;
    auto take = [](size_t& cursor, size_t sz) { size_t o = align_up(cursor, 256); cursor = o + sz; return o; };
    const size_t ns = size_t(std::max<int64_t>(slots, 1));
    const size_t o_ck = take(m, sizeof(ScanChunk) * n_chunks), o_pg = take(m, sizeof(pf_page_desc) * ns);
    const size_t o_crc = take(m, sizeof(ScanCrc) * ns), o_res = take(m, sizeof(ScanResult) * n_chunks);
    const size_t o_bad = take(m, 4 * size_t(n_chunks)), o_list = take(m, 4 * ns);
    m = align_up(m, 256);
    HIPCHK(ctx, ctx->d_scan.ensure(m));
    HIPCHK(ctx, ctx->h_meta.ensure(m));
    uint8_t* h = static_cast<uint8_t*>(ctx->h_meta.p);
    uint8_t* d = static_cast<uint8_t*>(ctx->d_scan.p);
    ScanChunk* hc = reinterpret_cast<ScanChunk*>(h + o_ck);
    for (int c = 0; c < n_chunks; c++)
        hc[c] = ScanChunk{d_bytes + chunks[c].chunk_offset, chunks[c].chunk_size, chunks[c].num_values, chunks[c].page_base,
                          chunks[c].page_cap};
    int32_t* hbad = reinterpret_cast<int32_t*>(h + o_bad);
    for (int c = 0; c < n_chunks; c++) hbad[c] = INT32_MAX;
    HIPCHK(ctx, hipMemcpyAsync(d + o_ck, h + o_ck, o_list - o_ck, hipMemcpyHostToDevice, st));
    ScanResult* d_res = reinterpret_cast<ScanResult*>(d + o_res);
    ScanCrc* d_crc = reinterpret_cast<ScanCrc*>(d + o_crc);
    launch_page_scan(reinterpret_cast<const ScanChunk*>(d + o_ck), n_chunks, reinterpret_cast<pf_page_desc*>(d + o_pg),
                     d_crc, d_res, st);
    HIPCHK(ctx, hipGetLastError());
    ScanResult* hr = reinterpret_cast<ScanResult*>(h + o_res);
    HIPCHK(ctx, hipMemcpyAsync(hr, d_res, sizeof(ScanResult) * n_chunks, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    if (verify_crc) {
        int32_t* hl = reinterpret_cast<int32_t*>(h + o_list);
        int n = 0;
        for (int c = 0; c < n_chunks; c++)
            for (int i = 0; i < hr[c].n_pages; i++) hl[n++] = chunks[c].page_base + i;
        if (n) {
            HIPCHK(ctx, hipMemcpyAsync(d + o_list, hl, 4 * size_t(n), hipMemcpyHostToDevice, st));
            launch_page_crc(d_crc, reinterpret_cast<const int*>(d + o_list), n, d_res, reinterpret_cast<int32_t*>(d + o_bad), st);
            HIPCHK(ctx, hipGetLastError());
            HIPCHK(ctx, hipMemcpyAsync(hr, d_res, sizeof(ScanResult) * n_chunks, hipMemcpyDeviceToHost, st));
            HIPCHK(ctx, hipMemcpyAsync(hbad, d + o_bad, 4 * size_t(n_chunks), hipMemcpyDeviceToHost, st));
        }
    }
    HIPCHK(ctx, hipMemcpyAsync(pages_out, d + o_pg, sizeof(pf_page_desc) * size_t(slots), hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    int rc = PF_OK;
    for (int c = 0; c < n_chunks; c++) {
        pf_scan_result& r = results[c];
        r.n_pages = hr[c].n_pages;
        r.status = hr[c].status;
        r.err_page = hr[c].err_page;
        r.crc_pages = hr[c].crc_pages;
        if (r.status == PF_OK && verify_crc && hbad[c] != INT32_MAX) {
            r.status = PF_ERR_CORRUPT_PAGE;
            r.err_page = hbad[c] - chunks[c].page_base;
        }
        if (r.status != PF_OK && rc == PF_OK) {
            rc = r.status;
            fail(ctx, rc, "scan: chunk " + std::to_string(c) + " page " + std::to_string(r.err_page) +
                              (hbad[c] != INT32_MAX && verify_crc ? ": CRC checksum verification failed" : ": corrupt page header"));
        }
    }
    return rc;
}

// Test hook: which path decoded the last pf_snappy_decompress (1 = serial fallback).
int pf_snappy_last_fallback(pf_ctx* ctx) {
    return ctx && ctx->h_res.p ? *reinterpret_cast<const int*>(static_cast<uint8_t*>(ctx->h_res.p) + 256) : -1;
}

// Diagnostics (not part of pfloor.h): the index tables of the last pf_snappy_decompress.
int pf_debug_snappy_tables(pf_ctx* ctx, uint32_t* splits, int n_splits, uint32_t* wins, int n_wins, uint32_t* lane_out,
                           uint32_t* tokmap) {
    if (!ctx || !ctx->d_last_splits) return fail(ctx, PF_ERR_STATE, "no snappy tables");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (splits) HIPCHK(ctx, hipMemcpy(splits, ctx->d_last_splits, 4 * size_t(n_splits), hipMemcpyDeviceToHost));
    if (wins) HIPCHK(ctx, hipMemcpy(wins, ctx->d_win, sizeof(SnapWin) * size_t(n_wins), hipMemcpyDeviceToHost));
    if (lane_out) HIPCHK(ctx, hipMemcpy(lane_out, ctx->d_lane_out, 256 * size_t(n_wins), hipMemcpyDeviceToHost));
    if (tokmap) HIPCHK(ctx, hipMemcpy(tokmap, ctx->d_tokmap.p, 1024 * size_t(n_wins), hipMemcpyDeviceToHost));
    return PF_OK;
}

// Diagnostics (not part of pfloor.h): per Snappy job of the last finished pf_decode_row_group,
// {fallback flag (FB_*), compressed length, decompressed length, chunk, page}. Returns the job count.
int pf_debug_snappy_fallback(pf_ctx* ctx, int* out, int n_jobs) {
    if (!ctx || !ctx->d_meta.p || !ctx->tables_from_decode) return fail(ctx, PF_ERR_STATE, "no finished decode");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int nj = int(ctx->jobs.size());
    const int m = n_jobs < nj ? n_jobs : nj;
    if (out && m > 0) {
        std::vector<int> fb(size_t(m), 0);
        HIPCHK(ctx, hipMemcpy(fb.data(), static_cast<uint8_t*>(ctx->d_meta.p) + ctx->off_fallback, 4 * size_t(m),
                              hipMemcpyDeviceToHost));
        for (int i = 0; i < m; i++) {
            const SnappyJob& jb = ctx->jobs[size_t(i)];
            const int rec[5] = {fb[size_t(i)], int(jb.src_len), int(jb.dst_len), jb.chunk, jb.page};
            for (int q = 0; q < 5; q++) out[5 * i + q] = rec[q];
        }
    }
    return nj;
}

// Diagnostics (not part of pfloor.h): per page of the last finished pf_decode_row_group, what
// k_snappy_head decided (DIRECT_NONE / DIRECT_VALUES / DIRECT_INPLACE). Returns the page count.
int pf_debug_page_direct(pf_ctx* ctx, int* out, int n_pages) {
    if (!ctx || !ctx->d_meta.p || !ctx->tables_from_decode) return fail(ctx, PF_ERR_STATE, "no finished decode");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int np = int(ctx->pages.size());
    const int m = n_pages < np ? n_pages : np;
    if (out && m > 0) {
        std::vector<DevPage> pg(static_cast<size_t>(m));
        HIPCHK(ctx, hipMemcpy(pg.data(), static_cast<uint8_t*>(ctx->d_meta.p) + ctx->off_pages, sizeof(DevPage) * size_t(m),
                              hipMemcpyDeviceToHost));
        for (int i = 0; i < m; i++) out[i] = pg[size_t(i)].direct;
    }
    return np;
}

// Diagnostics (not part of pfloor.h): per page of the last finished pf_decode_row_group, which
// parallel paths took it: {direct (DIRECT_*), dbp_ok (1 = k_dbp_* decoded it, 2 = handed back to
// k_delta), seg_ok (1 = nested segment kernels, 2 = hand-over failed, decoded whole)}. Returns the
// page count; out holds 3 ints per page.
int pf_debug_page_paths(pf_ctx* ctx, int* out, int n_pages) {
    if (!ctx || !ctx->d_meta.p || !ctx->tables_from_decode) return fail(ctx, PF_ERR_STATE, "no finished decode");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int np = int(ctx->pages.size());
    const int m = n_pages < np ? n_pages : np;
    if (out && m > 0) {
        std::vector<DevPage> pg(static_cast<size_t>(m));
        HIPCHK(ctx, hipMemcpy(pg.data(), static_cast<uint8_t*>(ctx->d_meta.p) + ctx->off_pages, sizeof(DevPage) * size_t(m),
                              hipMemcpyDeviceToHost));
        for (int i = 0; i < m; i++) {
            out[3 * i] = pg[size_t(i)].direct;
            out[3 * i + 1] = pg[size_t(i)].dbp_ok;
            out[3 * i + 2] = pg[size_t(i)].seg_ok;
        }
    }
    return np;
}

// Diagnostics (tests): the done flags of the last decode's pages (DONE_FIXED 1 / DONE_FLAT 2 /
// DONE_NULL 4: which kernel took the page; k_page_null and k_flat_null both set DONE_NULL, and only
// k_page_null's pages keep no level table (lvl = 0 in out[2 * i + 1])).
extern "C" int pf_debug_page_done(pf_ctx* ctx, int* out, int n_pages) {
    if (!ctx || !ctx->d_meta.p || !ctx->tables_from_decode) return fail(ctx, PF_ERR_STATE, "no finished decode");
    if (ctx->pending) return fail(ctx, PF_ERR_STATE, "call pf_wait first");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int np = int(ctx->pages.size());
    const int m = n_pages < np ? n_pages : np;
    if (out && m > 0) {
        std::vector<DevPage> pg(static_cast<size_t>(m));
        HIPCHK(ctx, hipMemcpy(pg.data(), static_cast<uint8_t*>(ctx->d_meta.p) + ctx->off_pages, sizeof(DevPage) * size_t(m),
                              hipMemcpyDeviceToHost));
        for (int i = 0; i < m; i++) {
            out[2 * i] = pg[size_t(i)].done;
            uint32_t lt1 = 0;   // k_lvl's "block table fits" word (k_flat_null ran on the page)
            if (pg[size_t(i)].lvltab) HIPCHK(ctx, hipMemcpy(&lt1, pg[size_t(i)].lvltab + 1, 4, hipMemcpyDeviceToHost));
            out[2 * i + 1] = int(lt1);
        }
    }
    return np;
}

int pf_last_timing(pf_ctx* ctx, float* stage_ms, int n_stages, int* n_written) {
    if (!ctx || !stage_ms || n_stages < 0) return fail(ctx, PF_ERR_INVALID_ARG, "bad arg");
    if (!ctx->timing) return fail(ctx, PF_ERR_STATE, "stage timing is off (pf_ctx_set_timing)");
    if (!ctx->timing_valid) return fail(ctx, PF_ERR_STATE, "no finished decode");
    int k = 0;
    for (int i = 0; i + 1 < N_EVENTS && k < n_stages; i++, k++) {
        float ms = 0;
        HIPCHK(ctx, hipEventElapsedTime(&ms, ctx->ev[i], ctx->ev[i + 1]));
        stage_ms[k] = ms;
    }
    if (n_written) *n_written = k;
    return PF_OK;
}

}  // extern "C"
