// pf_internal.h — device-side work descriptors shared by the HIP kernels and the host
// runtime (pf_runtime.hip). Not part of the C ABI.
//
// HBM layout of one decode batch (one pf_decode_row_group call):
//   in      : the caller's chunk bytes (resident, or one H2D copy of the pinned buffer)
//   scratch : decompressed page bodies, 16-B aligned, in page order (k_snappy writes,
//             the page kernels read); per-page BYTE_ARRAY value positions / dict ids
//   out     : per chunk: values | validity | offsets | chars | list offsets | levels,
//             each array 256-B aligned inside one arena
//   meta    : DevChunk[], DevPage[], DevChunkResult[] (small)
#pragma once
#include <stdint.h>

namespace pf {

// Decoder options. The product library (libpfloor.so) always runs these defaults and reads no
// environment. The diagnostics build (-DPF_DIAG, diag/libpfloor_diag.so) takes them from PF_*
// environment variables once per context, at pf_ctx_create: A/B selectors for the tools and the
// switches tests use to force rare paths (forced fallbacks, segment lengths, skipped stages).
struct PfOpts {
    int exec = 5;             // PF_EXEC: block-parallel Snappy executor: 5 producer / consumer | 2 one wave
    bool ba_fused = true;     // PF_BA_FUSED=0: the round-3 PLAIN BYTE_ARRAY walk kernels
    bool page_null = false;   // PF_PAGE_NULL=1: k_page_null before k_lvl
    bool null_dict_lds = true;   // PF_NULL_DICT_LDS=0: k_flat_null never stages its dictionary
    int null_stagger = 0;     // PF_DEBUG_NULL_STAGGER=k: k_flat_null's blocks > 0 wait k rounds (race tests)
    bool nest_timeout = false;   // PF_DEBUG_NEST_TIMEOUT=1: every k_nest_lvl hand-over times out (whole-page path; tests)
    uint32_t null_dcap = 0;   // PF_NULL_DCAP=b: k_flat_null's level-byte stage instead of the batch's (16: blocks with
                              // level bytes do not fit, so k_lvl refuses the page and the fallback queue decodes it; tests)
    bool piece_order = true;  // PF_PIECE_ORDER=0: Snappy pieces in page order
    unsigned debug_skip = 0;  // PF_DEBUG_SKIP=parse,exec,ba,levels,count,flat,decode (results are wrong)
    int force_serial = 0;     // PF_DEBUG_FORCE_SERIAL=k: every k-th Snappy job to the serial kernel
    int force_redo = 0;       // PF_DEBUG_FORCE_REDO=k: every k-th Snappy job rejected by the block executor
    bool exec_stream = false; // PF_EXEC_STREAM=1: the executor on a low-priority stream of its own
    bool zc = true;           // PF_ZC=0: SDMA copies for the batch tables instead of k_copy_words
    bool dl_kernel = true;    // PF_DL_KERNEL=0: pf_copy_batch_async by SDMA copies instead of k_download
    bool h2d_kernel = false;  // PF_H2D_KERNEL=1: pinned chunk bytes to the device by a kernel instead of SDMA (E2E: no gain, r06)
    int h2d_grid = 256;       // PF_H2D_GRID: that kernel's workgroups (fewer: a slower upload beside the downloads)
    bool dl_stream = true;    // PF_DL_STREAM=0: pf_copy_batch_async on the decode stream instead of the copy stream
    bool dl_prio = false;     // PF_DL_PRIO=1: the copy stream at the device's highest stream priority
    bool debug_plan = false;  // PF_DEBUG_PLAN=1: host planning phase times on stderr
    int64_t nest_seg = 0;     // PF_NEST_SEG=n: nested segment length, forced (0: default, not forced)
    bool nest_seg_set = false;
    bool dbp_par = true;      // PF_DBP_PAR=0: every DELTA_BINARY_PACKED page on k_delta
    int fix_shift = 1;        // PF_FIX_BLK=4096|8192|16384: fixed-width flat blocks (log2 of the multiple of 4096)
    int decode_grid = 32;     // PF_DECODE_GRID: k_decode blocks when no page is known to need it (grid-stride check)
    int count_grid = 64;      // PF_COUNT_GRID: k_count blocks (grid-stride; nearly every page is counted by k_count_flat)
};

enum : int32_t {
    PG_V2 = 1,            // DATA_PAGE_V2
    PG_COMPRESSED = 2,    // body lives in scratch after k_snappy
    PG_DICT = 4,          // dictionary page
};

// One decompression job (Snappy raw stream -> dst).
struct SnappyJob {
    const uint8_t* src;
    uint8_t* dst;
    uint32_t src_len;
    uint32_t dst_len;
    int32_t page;         // global page index (for error attribution)
    int32_t chunk;
    uint32_t split_base;  // first entry of this job's 64 KiB split table
    uint32_t n_pieces;    // ceil(dst_len / 65536), >= 1
    uint32_t* tokmap;     // bit i = a token starts at input byte i (n_win * 256 words, index pass)
    uint32_t win_base;    // first entry of this job's 8 KiB index windows (SnapWin / lane outs)
    uint32_t n_win;       // ceil(src_len / 8192), >= 1
    // direct pages (k_snappy_head): output bytes [dlo, dst_len) go to ddst + offset (the column's
    // values) instead of dst + offset; bytes below dlo (the v1 level section) still go to dst.
    // dgran: the store width (4, 8 or 16 bytes) ddst's alignment allows (flush chunks sit at 16-byte
    // aligned output offsets). Only the
    // block-parallel executor writes direct; the whole-page redo and the serial kernel write dst.
    uint8_t* ddst;
    uint32_t dlo;
    uint32_t dgran;
    uint32_t dflags;      // bit 0 (diagnostics) = the block-parallel executor rejects the job (PF_DEBUG_FORCE_REDO);
                          // bit 1 = k_snappy_litcopy candidate (dictionary page, or a data page that did not compress)
    uint32_t lit;         // FB_LITCOPY: the page's literal count (their table is in tokmap)
};

// DONE_PAGE: k_page_null decoded the whole page (with DONE_NULL); k_lvl and k_flat_null skip only
// such pages -- never DONE_NULL itself, which k_flat_null's own finished blocks of the page set.
enum : int32_t { DONE_FIXED = 1, DONE_FLAT = 2, DONE_NULL = 4, DONE_PAGE = 8 };

// DevPage.direct (k_snappy_head): how the page's decompressed body reaches the decoders
enum : int32_t { DIRECT_NONE = 0, DIRECT_VALUES = 1, DIRECT_INPLACE = 2 };

struct DevPage {
    const uint8_t* body;      // v1: [rep][def][values] uncompressed; v2: values section
    const uint8_t* lvl;       // v2: [rep][def] raw levels (never compressed); v1: null
    uint32_t body_len;
    uint32_t rep_len;         // v2 byte lengths
    uint32_t def_len;
    int32_t chunk;
    int32_t flags;
    int32_t encoding;
    int32_t def_enc;
    int32_t rep_enc;
    int32_t num_values;       // level entries
    int32_t done;             // DONE_FIXED | DONE_FLAT: k_flat_fixed / k_flat decoded (or failed) the page; k_decode skips it
    int64_t entry_start;      // first level entry of this page within its chunk (host prefix sum)
    // written by k_count, consumed by k_scan
    int64_t n_slots;
    int64_t n_values;
    int64_t n_rows;
    int64_t n_chars;
    // written by k_scan (or host for flat fixed-width chunks)
    int64_t slot_start;
    int64_t value_start;
    int64_t row_start;
    int64_t char_start;
    // per-page scratch: BYTE_ARRAY value positions (PLAIN) or dictionary ids
    uint32_t* aux;
    int64_t aux_cap;          // entries
    int32_t ba_job;           // PLAIN BYTE_ARRAY data page: its BaJob (k_count fills it), else -1
    int32_t counted;          // 1: k_count_flat counted the page (k_count skips it)
    uint32_t* runtab;         // dictionary data page of a flat chunk: id run table (k_runs), else null
    uint32_t* lvltab;         // nullable fixed-width page of a flat chunk: definition-level run table (k_lvl), else null
    uint32_t lvl_cap;         // runs the level table can hold
    // DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY page (k_dlen, pf_delta.hip): {cpos[aux_cap + 1],
    // lenA[aux_cap], lenB[aux_cap]} (u64), values in the length streams, first bad value, and
    // where the chars / suffixes start in the values section; else null
    uint64_t* dx;
    int64_t dx_total;
    int64_t dx_bad;
    uint32_t dx_data;
    uint32_t dx_pad;
    // Snappy data pages: the job's fallback flag (FB_*, read after the executor), and what
    // k_snappy_head decided (DIRECT_*): VALUES = a PLAIN fixed-width page with every level present
    // whose values the executor wrote straight into the column (k_flat_fixed then only sets the
    // validity bits, unless the job fell back to the redo / serial path, which writes the body);
    // INPLACE = the stream is one literal: body points at it in the compressed input, no executor.
    const int* jfb;
    int32_t direct;
    int32_t direct_pad;
    // nested data pages split into segments of seg_len entries (k_nest_*, pf_pages.hip), else null:
    // {RleState ck[3][nseg] (rep, def, value stream state at each segment's start), SegRec rec[nseg]}
    uint8_t* seg;
    int32_t nseg;
    int32_t seg_len;
    int32_t seg_ok;           // k_nest_lvl: 1 = the segment kernels decode the page (k_count / k_decode skip it)
    int32_t nwin;             // k_nest_lvl windows per level stream (the page's bytes / NEST_WIN, rounded up)
    struct WinPub* npub;      // [2][nwin]: what each window of the rep / def stream passes to the next (zeroed per batch)
    // large DELTA_BINARY_PACKED INT32 / INT64 pages decoded block-parallel (k_dbp_*, pf_delta.hip), else null:
    // {uint32_t pos[dbp_bcap] (block header positions), uint64_t sum[dbp_bcap] (block delta sums, then bases)}
    uint8_t* dbp;
    struct WinPub* dbp_pub;   // [dbp_nwin] window hand-overs of the block chain (zeroed per batch)
    int32_t dbp_nwin;
    int32_t dbp_ok;           // 1: k_dbp_* decoded the page; 0 / 2 (not taken / failed): k_delta decodes it
    uint32_t dbp_bcap;        // blocks the tables hold
    uint32_t dbp_pad;
};

// k_nest_lvl / k_dbp_pos: a window's hand-over to the next window of its stream -- the position of
// the first run header (block header) at or past the window's end, the entries (blocks) before it,
// whether the chain ended (st = 1) -- packed in one 64-bit word (0 until published) that is stored and
// polled with relaxed agent-scope atomics (round 5: three stores and a release flag made every
// hand-over write back the XCD's L2 and every acquire invalidate the reader's).
struct WinPub {
    uint64_t w;
};
#ifdef __HIPCC__
__device__ __forceinline__ void winpub_put(WinPub& me, uint64_t p, uint64_t e, uint32_t st) {
    // st + 1 in the low two bits (never 0); a position or count past 31 bits publishes 3 (overflow)
    const bool ovf = p > 0x7fffffffull || e > 0x7fffffffull || st > 1u;
    const uint64_t w = (uint64_t(p & 0x7fffffffu) << 33) | (uint64_t(e & 0x7fffffffu) << 2) | uint64_t(ovf ? 3u : st + 1u);
    __hip_atomic_store(&me.w, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Waits up to spin_cap polls; false: no hand-over came (or it overflowed), the caller gives the page up.
__device__ __forceinline__ bool winpub_get(const WinPub& pv, uint32_t spin_cap, uint64_t& p, uint64_t& e, uint32_t& st) {
    if (spin_cap == 0) return false;   // (diagnostics: every hand-over times out)
    uint64_t w;
    uint32_t spins = 0;
    while ((w = __hip_atomic_load(&pv.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 && ++spins < spin_cap)
        __builtin_amdgcn_s_sleep(2);
    if (w == 0 || (w & 3u) == 3u) return false;
    p = w >> 33;
    e = (w >> 2) & 0x7fffffffull;
    st = uint32_t(w & 3u) - 1u;
    return true;
}
#endif
#ifndef PF_NEST_WIN
#define PF_NEST_WIN 2048
#endif
constexpr uint32_t NEST_WIN = PF_NEST_WIN;  // k_nest_lvl window bytes (power of two)
#ifndef PF_DBP_WIN
#define PF_DBP_WIN 4096
#endif
constexpr uint32_t DBP_WIN = PF_DBP_WIN;    // k_dbp_pos window bytes (power of two)
constexpr int32_t DBP_PAR_MIN = 16384;      // DELTA_BINARY_PACKED pages with at least this many entries go block-parallel

// One segment of a nested page: its level counts (k_count_seg), their exclusive prefixes over the
// page (k_nest_scan), the chars of its values and their prefix (k_nest_ids / k_nest_chars).
struct SegRec {
    uint32_t ns, nv, nr, pad;
    uint64_t chars;
    uint32_t sb, vb, rb, pad2;
    uint64_t cb;
};
constexpr uint32_t NEST_CK_BYTES = 40;      // sizeof(RleState) (pf_device.h)
constexpr uint32_t NEST_SEG = 2048;         // default entries per segment
constexpr uint32_t NEST_MAX_SEGS = 1024;    // segments per page (k_nest_scan keeps their targets in LDS)
__host__ __device__ inline uint64_t nest_seg_bytes(int32_t nseg) {
    return uint64_t(nseg) * (3ull * NEST_CK_BYTES + sizeof(SegRec));
}

// k_runs run table of a page: {nruns, values covered, all levels present, valid}, then nruns
// entries {first | packed << 31, RLE value or bit offset}; a run's count is the next first - first.
constexpr uint32_t RT_CAP = 1024;
constexpr uint32_t RT_BYTES = 16 + 8 * RT_CAP;

// k_lvl definition-level run table of a nullable flat page: {nruns, valid, present values, -}, then
// nruns entries {first entry, RLE value or bit offset, count | packed << 31, present values before},
// then LT_BT_WORDS words per 4096-entry block (k_flat_null): {first run, end run, first value index,
// end value index, level bytes [d0, d1), dictionary-id bytes [i0, i1)} of the block.
constexpr uint32_t LT_BLOCK_RUNS = 512;    // most runs one k_flat_null block may overlap (its LDS table)
constexpr uint32_t LT_BT_WORDS = 8;
constexpr uint32_t NL_DST = 4096;          // most level bytes one k_flat_null block stages in LDS
constexpr uint32_t NULL_DICT_LDS = 16384;   // k_flat_null stages dictionaries up to this many bytes in LDS
constexpr uint32_t NL_IST = 12288;         // most dictionary-id bytes one k_flat_null block stages in LDS
constexpr uint32_t NL_SLACK = 256;         // run-header bytes a block's level / id byte range may add
// k_flat_null's dynamic LDS, per batch: level bytes (dcap), dictionary-id bytes (icap) a block may
// stage -- from the batch's widest level / id bit width (host-known: max definition level, dictionary
// size), FBLK values of it + NL_SLACK, at most NL_DST / NL_IST; k_lvl's block table is checked against
// the same caps -- and the dictionary bytes it stages (dlds, 0: none). Multiples of 16.
struct NullCaps {
    uint32_t dcap, icap, dlds;
};
__host__ __device__ inline uint32_t lvl_table_cap(int32_t num_values) {
    // RLE runs are >= 8 repeats and bit-packed groups 8 values for the writers we know (parquet-mr,
    // Arrow): <= 2 runs per 16 entries; a page needing more is left to k_flat / k_decode
    return uint32_t(num_values) / 8u + 64u;
}

// One PLAIN BYTE_ARRAY length walk (a BYTE_ARRAY dictionary page, or the values section of a
// PLAIN BYTE_ARRAY data page), done tile-parallel by the k_ba_* kernels (pf_pages.hip).
// BA_RELINK: the fused tile pass (k_ba_tile) rejected the job -- a value longer than its halo, or
// filters it could not separate -- and k_ba_fallback re-links it over the whole job before any walk
enum : int32_t { BA_OK = 0, BA_FALLBACK = 1, BA_SKIP = 2, BA_RELINK = 3 };
struct BaJob {
    const uint8_t* p;         // stream (data pages: set by k_count)
    uint32_t* pos;            // out: chars start of value k
    uint32_t* len;            // out (optional): length of value k
    int64_t* chars_out;       // out (optional): total chars
    uint32_t* cand;           // bitmaps over the stream, n_cap / 32 + 1 words each
    uint32_t* link1;
    uint32_t* link2;
    uint32_t* tile_cnt;       // per tile: accepted positions, then their exclusive scan
    int64_t count;            // values to read (data pages: set by k_count)
    uint32_t n;               // stream bytes (data pages: set by k_count; <= n_cap)
    uint32_t n_cap;           // host bound: tiles and bitmaps are sized for it
    uint32_t n_tiles;
    int32_t chunk, page;
    int32_t state;            // BA_* (data pages: BA_SKIP until k_count fills the job)
};

struct DevChunk {
    int32_t ptype, type_length, width, max_def, max_rep, repeated_def, list_null_def, codec;
    int32_t dict_page;        // global page index of the dictionary page, -1 if none
    int32_t first_page;       // first data page (global index)
    int32_t n_pages;          // data pages
    int32_t needs_count;      // 1: BYTE_ARRAY or nested -> k_count + k_scan
    int64_t num_entries;
    // dictionary (k_dict): fixed width -> dict_data is the decoded PLAIN page;
    // BYTE_ARRAY -> dict_pos[i] = byte offset of entry i's length prefix in dict_data
    const uint8_t* dict_data;
    uint32_t* dict_pos;       // n+1 entries: start of chars of entry i (after the prefix), end at [n] sentinel
    uint32_t* dict_len;
    int64_t dict_n;
    // outputs
    uint8_t* values;
    uint8_t* validity;
    int32_t* offsets;
    uint8_t* chars;
    int32_t* list_offsets;
    uint8_t* list_validity;
    uint8_t* def_levels;
    uint8_t* rep_levels;
    int64_t values_cap, chars_cap, slots_cap, rows_cap;   // capacities (bytes / elements)
};

struct DevChunkResult {
    int64_t num_slots, num_values, num_rows, num_chars;
    int32_t status;           // pf_status (first error wins, atomicMin on negative codes)
    int32_t err_page;
};

// GPU page-header scan (pf_scan.hip, pf_scan_pages)
struct ScanChunk {            // device copy of pf_scan_chunk
    const uint8_t* base;      // chunk's first byte
    uint64_t size;
    int64_t num_values;
    int32_t page_base;
    int32_t page_cap;
};

struct ScanCrc {              // per page slot: header crc and the page bytes it covers
    const uint8_t* body;
    uint32_t len;
    uint32_t crc;
    int32_t has_crc;
    int32_t chunk;
};

struct ScanResult {           // mirrors pf_scan_result
    int32_t n_pages;
    int32_t status;
    int32_t err_page;
    int32_t crc_pages;
};

}  // namespace pf
