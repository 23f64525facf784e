// sidx_common.hpp -- shared host/device definitions of the MI355X record indexer.
//
// Layout of one index build (one "slab" = a contiguous byte range of a node's file that
// lives in HBM on one GPU; a single-GPU build is one slab covering the whole file):
//   * the slab is cut into TILE-byte tiles, one 256-thread workgroup per tile;
//   * every tile's monoid aggregate of its bytes is folded by a device-wide exclusive scan
//     (k_scan_excl, decoupled look-back over blocks of tiles) into the state before it;
//   * records are owned by the tile holding the delimiter that starts them and are written
//     as 16-byte rows {u64 offset, u64 length} straight to the row table in HBM.
// See DESIGN.md for the per-format monoids and the reference citations.
#pragma once
#include <stdint.h>

namespace sidx {

typedef unsigned long long u64;
typedef long long i64;
typedef unsigned int u32;

#ifndef SIDX_TILE
#define SIDX_TILE 16384
#endif
#ifndef SIDX_NTHREADS
#define SIDX_NTHREADS (SIDX_TILE / 128)
#endif
constexpr int TILE = SIDX_TILE;           // bytes per workgroup tile
constexpr int NTHREADS = SIDX_NTHREADS;   // 128 contiguous bytes per thread
constexpr int NWAVES = NTHREADS / 64;
constexpr int CHUNK = 16;                 // bytes per lane load (global_load_dwordx4)
constexpr int NCHUNKS = TILE / CHUNK;     // 2048
constexpr int CPT = NCHUNKS / NTHREADS;   // chunks per thread = 8
constexpr int REGION = TILE / NTHREADS;   // contiguous bytes owned by a thread = 128
constexpr int MAX_DEFER = 16;             // deferred (tile-crossing) records per tile
constexpr int FQ_TILE_WORDS = 2 * MAX_DEFER;  // FASTQ tile pass: a tile's deferred records (u32 words)
#ifndef SIDX_HALO
#define SIDX_HALO 1024
#endif
constexpr int HALO = SIDX_HALO;           // bytes past the tile staged with it (records that
                                          // cross the tile end resolve in LDS)
constexpr int HALO_CHUNKS = HALO / CHUNK; // loaded by the first threads as an extra chunk
static_assert(HALO_CHUNKS < NTHREADS, "one more thread loads the front pad");

// Formats (values shared with include/shockidx.h).
enum Fmt : int { F_NONE = 0, F_FASTA = 1, F_FASTQ = 2, F_SAM = 3, F_LINE = 4 };

// Record status codes (4 bits, low bits of the first-bad key).
enum Status : u32 {
  ST_OK = 0,
  ST_END = 1,            // FASTQ: clean end of records (not an error)
  ST_FQ_TRUNC = 2,       // fastq.go:156,175,187 "truncated fastq record"
  ST_FQ_EMPTYLINES = 3,  // fastq.go:162
  ST_FQ_NOAT = 4,        // fastq.go:165
  ST_FQ_NOID = 5,        // fastq.go:168
  ST_FQ_EMPTYSEQ = 6,    // fastq.go:180
  ST_FQ_NOPLUS = 7,      // fastq.go:192
  ST_FQ_IDMISMATCH = 8,  // fastq.go:197
  ST_FQ_LENMISMATCH = 9, // fastq.go:207
  ST_FA_INVALID = 10,    // fasta.go:120 "Invalid fasta entry: <piece[:50]>"
  ST_DONTCARE = 11,      // FASTQ: a blank group right after another blank group
  ST_NEEDMORE = 12,      // slab halo exhausted before the record could be closed
  ST_ABSENT = 13,        // record would start at EOF: does not exist (not an error)
  ST_DEFER = 14,         // internal: leave the tile -> wave-cooperative global path
  ST_SLOW = 15,          // internal: take the general (searching) validator
};

// Look-back status word: [63:62] flag, [61:48] build epoch (never 0), [47:0] payload.
// Words of an older build carry another epoch and read as "not published", so the status
// array needs no memset per build (it is cleared only when the 14-bit epoch wraps).
constexpr u64 FLAG_AGG = 1ull << 62;
constexpr u64 FLAG_INC = 2ull << 62;
constexpr int EPOCH_SHIFT = 48;
constexpr u32 EPOCH_MASK = 0x3FFF;
constexpr u64 PAYLOAD_MASK = (1ull << EPOCH_SHIFT) - 1;

// First-bad key: record index << 28 | tile << 4 | status (min over the slab).
constexpr int KEY_TILE_BITS = 24;
constexpr int KEY_REC_SHIFT = 4 + KEY_TILE_BITS;
constexpr u64 KEY_NONE = ~0ull;
constexpr int NCOUNTERS = 8;  // u32 counters per build slot

// Kernel parameters for one slab.
struct SlabParams {
  const uint8_t *data;   // slab bytes (16-byte aligned), readable up to data[end)
  u64 n;                 // bytes owned by this slab (tiles cover [0, n))
  u64 end;               // readable end (n + halo); EOF at `end` iff eof != 0
  u64 base;              // file offset of data[0]
  u64 state_in;          // monoid state before data[0] (format-specific packing)
  u64 row_base;          // record index stored at rows[0]
  u64 row_cap;           // capacity of rows (in 16-byte rows)
  u64 *rows;             // out: {offset, length} little-endian pairs
  u64 *status;           // status[ntiles - 1]: the slab aggregate (INC word) for k_finalize
  u64 *badkey;           // min first-bad key (KEY_NONE before launch)
  u64 *detail;           // per-tile {pos, len} of the tile's first bad record (FASTA msg)
  u32 *counters;         // [0] unused, [1] defer overflow, [2] k_fixup items, [3] k_fixup overflow,
                         // [4] [5] scan tickets, [6] unused, [7] k_fixup finish ticket (NCOUNTERS, reset by the previous finalize)
  u64 *badkey_next;      // the other build's first-bad slot (reset by finalize)
  u32 *counters_next;    // the other build's counters (reset by finalize)
  u32 ntiles;
  u32 epoch;             // 1..EPOCH_MASK, distinct for consecutive builds on a status array
  int eof;               // 1 iff `end` is the end of the file
  int file_start;        // 1 iff data[0] is file offset 0 (owns record 0)
  u64 *timing;           // diagnostic: per-workgroup phase cycle sums (null in production)
  u64 *summary;          // multi-GPU: 64-byte slab summary written by finalize (or null)
  u64 front;             // readable bytes before data[0] (slabs after the first)
  u32 debug;             // ablation knobs of the SIDX_DIAG variant (two-pass kernels): bit0
                         // skip emission, bit2 skip deferred records
  // line tile pass: per tile the last '\n' + 1 (0: none) and its exclusive max scan
  u64 *pcnt;
  u64 *ppre;
  // look-back words of the tile-aggregate scans (k_scan_excl), one array per scan of a build;
  // each word FLAG | epoch tag | payload; the scans' tickets are counters[4 + which]
  u64 *scan_look[2];
  u32 pgrid;             // persistent grid of the tile passes
  u32 seq;               // multi-GPU: the caller's build tag, stamped into the slab summary
  u64 *fix;              // k_fixup queue (32-byte items); counters[2] = items, counters[3] = overflow
  u32 fixcap;
  // exclusive monoid prefix of every tile's aggregate (k_scan_excl): k_index1's incoming
  // states, the tile passes' record / row bases
  const u64 *tile_excl;
  // per-tile monoid aggregates (two-pass and tile passes); FASTQ tile pass provisional rows
  // (RCAP u32 per tile: start | length << 16) and per-tile results (FQ_TILE_WORDS u32)
  u64 *fq_agg;
  u32 *fq_stage;
  u32 *fq_tiles;
  // format speculation (single builds with auto-detection): every kernel of the pipeline exits
  // at once unless k_detect's result *gate equals gate_fmt; k_finalize then reports flag 16 and
  // the detected format, and the host re-runs with it.  Null: no gate.
  const int *gate;
  int gate_fmt;
  u32 inject;            // test hooks (shockidx_debug_inject): bit0 finalize reports one record short
  // download filters over FASTQ (k_fq_tiles<true>): per record its three inner line ends
  // (3 u16 per record, RCAP records per tile; sidx_filter.hip's spans come from them)
  uint16_t *fq_lines;
};
__device__ __forceinline__ bool gated_off(const SlabParams &p) { return p.gate && *p.gate != p.gate_fmt; }

// Multi-GPU slab summary (mirrors shockidx_slab_summary in include/shockidx.h).
// `seq` is the tag the caller gave the slab's build (shockidx_slab.seq): the fold refuses a
// summary whose tag is not the one the caller expects (a stale summary, e.g. an exchange whose
// copy had not landed).
struct SlabSummary {
  u64 agg, state_in, key, natural, row_base, err_pos, err_len;
  uint16_t fmt, flags;
  u32 seq;
};
static_assert(sizeof(SlabSummary) == 64, "summary is exchanged as 64 bytes");

// Fold of all slab summaries for one rank (mirrors shockidx_slab_plan).
struct SlabPlan {
  u64 state_in, first_record, count, err_pos, err_len;
  u32 code;
  int err_rank;
  u32 inconsistent, flags;
};

// Device result of finalize (mirrored by shockidx_result in include/shockidx.h).
struct DevResult {
  u64 count;       // records (rows) produced, Go's `count`
  u64 state_out;   // monoid state after the slab
  u64 slab_agg;    // monoid aggregate of the slab bytes (independent of state_in)
  u64 key;         // first-bad key (record index << 28 | tile << 4 | status) or KEY_NONE
  u64 natural;     // count if no record terminated the sequence inside the slab
  u64 err_pos;     // FASTA error piece position (file offset)
  u64 err_len;     // FASTA error piece length
  u32 code;        // ST_* of the terminating record (0 / END / ABSENT = success)
  u32 flags;       // bit0 capacity overflow, bit1 internal error, bit2 needmore
  u32 path;        // set by the host: 1 tile pass, 2 two-pass build
  u32 fmt;         // format actually indexed
  u32 fixups;      // records / tiles queued for k_fixup (diagnostic)
  u32 fix_tiles;   // of which whole tiles (diagnostic)
  u32 detected;    // gated builds: k_detect's format (SHOCKIDX_FMT_*)
  u32 pad;
};

}  // namespace sidx
