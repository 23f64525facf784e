// sidx_capi.cpp -- host side of libshockidx: the C ABI declared in include/shockidx.h.
//
// Owns HIP streams, device workspaces and pinned staging; stages host bytes to HBM, runs
// the gfx950 kernels (sidx_kernels.hip), turns the device result into Go's (count, err),
// and writes the .idx file with the reference's temp-file + rename protocol
// (shock-server/node/file/index/record.go:35-41,65-87).  No index computation happens on
// the host: without a usable GPU every entry point fails with SHOCKIDX_EHIP.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>
#include <string>

#include <rccl/rccl.h>

#include "../../include/shockidx.h"
#include "sidx_common.hpp"
#include "sidx_subset.hpp"
#include "sidx_host.hpp"

using namespace sidx;

extern "C" hipError_t sidx_launch_detect(const uint8_t *d, u64 n, int *d_out, hipStream_t s);
extern "C" hipError_t sidx_launch_index(int fmt, const SlabParams *p, DevResult *d_res, hipStream_t s,
                                        hipEvent_t ek0, hipEvent_t ek1);
extern "C" hipError_t sidx_launch_chunkrecord(const uint8_t *d, u64 n, int fasta, long long chunk, u64 *rows,
                                              u64 row_cap, u64 *out, long long curr0, u64 cnt0, u64 max_steps,
                                              hipStream_t s);
extern "C" hipError_t sidx_cr_gpos_count(const uint8_t *d, u64 n, u64 *tcnt, u64 *toff, uint16_t *slot,
                                         void *scan_tmp, size_t *scan_bytes, hipStream_t s);
extern "C" hipError_t sidx_cr_gpos_write(const uint8_t *d, u64 n, const u64 *tcnt, const u64 *toff,
                                         const uint16_t *slot, u64 *G, hipStream_t s);
extern "C" u32 sidx_cr_gslot();
extern "C" hipError_t sidx_cr_graph(const uint8_t *d, u64 n, int fasta, u64 chunk, const u64 *base, u64 stride,
                                    u64 count, u64 *ft, u32 *J1, u32 *Ja, u32 *Jb, int levels, const u32 **JL,
                                    hipStream_t s);
extern "C" hipError_t sidx_cr_round(const uint8_t *d, u64 n, int fasta, u64 chunk, const u64 *base, u64 stride,
                                    u64 count, const u64 *ft, const u32 *JL, const u32 *J1, u32 L, u64 y, u64 k0,
                                    u64 cap, u32 *heads, u64 *pos, i64 *mres, u64 *ctl, u64 *rows, u64 row_cap,
                                    u32 verify_grid, hipStream_t s);
extern "C" int sidx_cr_verify_blocks_per_cu();
extern "C" u32 sidx_fa_slot();
extern "C" hipError_t sidx_fa_bnd_count(const uint8_t *d, u64 n, u64 *lnl, u64 *lgt, u64 *cnl, u64 *cgt, u64 *tcnt,
                                        u64 *toff, uint16_t *slot, void *tmp, size_t *tmp_bytes, hipStream_t s);
extern "C" hipError_t sidx_fa_bnd_write(const uint8_t *d, u64 n, const u64 *cnl, const u64 *cgt, const u64 *tcnt,
                                        const u64 *toff, const uint16_t *slot, u64 *B, hipStream_t s);
extern "C" hipError_t sidx_fa_anon_spans(const uint8_t *d, u64 n, const u64 *B, u64 bstride, u64 m, u64 *bspan, u64 *outlen,
                                         u64 *firstbad, hipStream_t s);
extern "C" hipError_t sidx_fa_anon_write(const uint8_t *d, u64 n, const u64 *bspan, const u64 *outoff, u64 K,
                                         uint8_t *out, hipStream_t s);
extern "C" hipError_t sidx_sam_anon_spans(const uint8_t *d, u64 n, const u64 *rows, u64 K, u64 *span, u64 *outlen,
                                          u64 *firstbad, u64 *firsteof, hipStream_t s);
extern "C" hipError_t sidx_sam_anon_write(const uint8_t *d, const u64 *span, const u64 *outlen, const u64 *outoff,
                                          u64 K, uint8_t *out, u64 *count, hipStream_t s);
extern "C" hipError_t sidx_crs_scan(const u64 *ri, u64 R, u64 *len, u64 *P, void *tmp, size_t *scan_bytes,
                                    hipStream_t s);
extern "C" hipError_t sidx_crs_build(const u64 *P, u64 R, u32 *J1, u32 *Ja, u32 *Jb, int levels, u32 *heads, u64 *rows,
                                     u64 row_cap, u64 *ctl, hipStream_t s);
extern "C" int sidx_tiles_blocks_per_cu();
extern "C" hipError_t sidx_launch_slab_guess(const uint8_t *d, u64 n, u64 front, int fmt, u64 *d_out,
                                             hipStream_t s);
extern "C" hipError_t sidx_launch_verify_rows(const u64 *rows, u64 row_base, u64 row_cap, DevResult *d_res, hipStream_t s);
extern "C" hipError_t sidx_launch_slab_combine(const void *d_all, int world, int rank, int fmt, const uint32_t *expect, void *d_plan,
                                               hipStream_t s);
extern "C" hipError_t sidx_id_lines(const uint8_t *text, u64 n, u32 *cnt, u64 *base, u64 *ends, void *tmp,
                                    size_t *tmp_bytes, hipStream_t s);
extern "C" hipError_t sidx_subset_parse(const uint8_t *text, const u64 *ends, u64 m, u32 *keep, i64 *val, u32 *st,
                                        hipStream_t s);
extern "C" hipError_t sidx_scan_flags(const u32 *in, u64 *out, u64 n, void *tmp, size_t *tmp_bytes, hipStream_t s);
extern "C" hipError_t sidx_scan_u64(const u64 *in, u64 *out, u64 n, void *tmp, size_t *tmp_bytes, hipStream_t s);
extern "C" hipError_t sidx_subset_compact(const u32 *keep, const u64 *rank, const i64 *val, const u32 *st, u64 m,
                                          i64 *cval, u32 *cst, u64 *cline, u64 *ctl, hipStream_t s);
extern "C" hipError_t sidx_subset_init(u64 *ctl, u64 nruns, hipStream_t s);
extern "C" hipError_t sidx_subset_check(const i64 *cval, const u32 *cst, u64 m, u64 *ctl, const u64 *parent,
                                        u64 parent_count, i64 ilength, u64 *rows, u64 rows_cap, u32 *startf,
                                        hipStream_t s);
extern "C" hipError_t sidx_subset_runs(const u64 *rows, const u32 *startf, const u64 *runid, u64 m, u64 *ctl,
                                       u64 *runs, u64 rows_cap, u64 runs_cap, hipStream_t s);
extern "C" hipError_t sidx_launch_fq_spans_place(const SlabParams *pp, u32 *spans, u64 *outlen, u64 K, int kind,
                                                hipStream_t s);
extern "C" hipError_t sidx_launch_fq_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                           hipEvent_t ek1);
extern "C" hipError_t sidx_launch_fa_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                           hipEvent_t ek1);
extern "C" int sidx_fa_tiles();
extern "C" hipError_t sidx_launch_line_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                             hipEvent_t ek1);
extern "C" int sidx_line_tiles();
extern "C" hipError_t sidx_launch_sam_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                            hipEvent_t ek1);
extern "C" int sidx_sam_tiles();
extern "C" hipError_t sidx_filter_spans(const uint8_t *data, u64 n, const u64 *rows, u64 K, int kind, u32 *spans,
                                        u64 *outlen, u64 *firstbad, hipStream_t s);
extern "C" hipError_t sidx_filter_write(const uint8_t *data, u64 n, const u64 *rows, const u32 *spans, const u64 *outlen,
                                        const u64 *outoff, u64 K, u64 total, int kind, u64 *wfirst, uint8_t *out,
                                        hipStream_t s);
extern "C" u64 sidx_filter_block();
extern "C" hipError_t sidx_filter_read_status(const uint8_t *data, u64 n, u64 start, u32 *out, hipStream_t s);
extern "C" hipError_t sidx_range_flags(const u64 *rows, u64 nrows, u64 a0, u64 nr, u32 *flags, hipStream_t s);
extern "C" hipError_t sidx_range_emit(const u64 *rows, u64 nrows, u64 a0, u64 nr, const u32 *flags, const u64 *id,
                                      u64 *recs, hipStream_t s);
extern "C" hipError_t sidx_gather(const uint8_t *data, u64 data_len, const u64 *runs, u64 bound, u64 *ctl, u64 *lens,
                                  u64 *outoff, void *tmp, size_t *tmp_bytes, u64 *wfirst, uint8_t *out, u64 out_cap,
                                  hipEvent_t e0, hipEvent_t e1, hipStream_t s);

namespace {

constexpr size_t STAGE_BYTES = 64ull << 20;  // pinned staging chunk
constexpr int NSTAGE = 2;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// Host copies between the caller's memory and the pinned staging buffers, split over a
// small persistent thread pool (one memcpy thread tops out near 25 GB/s, below PCIe Gen5).
class CopyPool {
 public:
  explicit CopyPool(int n) : nt_(n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this, i] { run(i); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  void copy(void *dst, const void *src, size_t n) {
    uint8_t *d = (uint8_t *)dst;
    const uint8_t *sp = (const uint8_t *)src;
    parallel(n, [d, sp](size_t a, size_t b) { memcpy(d + a, sp + a, b - a); });
  }
  // f(a, b) over disjoint 4 KiB-aligned slices of [0, n), one per thread (small n: inline)
  void parallel(size_t n, const std::function<void(size_t, size_t)> &f) {
    if (n < (4u << 20) || nt_ < 2) {
      if (n) f(0, n);
      return;
    }
    std::unique_lock<std::mutex> lk(m_);
    fn_ = &f;
    n_ = n;
    pending_ = nt_;
    ++gen_;
    cv_.notify_all();
    done_.wait(lk, [this] { return pending_ == 0; });
  }

 private:
  void run(int i) {
    unsigned long long seen = 0;
    for (;;) {
      const std::function<void(size_t, size_t)> *f;
      size_t n;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        f = fn_;
        n = n_;
      }
      const size_t per = ((n + nt_ - 1) / nt_ + 4095) & ~(size_t)4095;
      const size_t a = (size_t)i * per < n ? (size_t)i * per : n, b = a + per < n ? a + per : n;
      if (b > a) (*f)(a, b);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  const int nt_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t)> *fn_ = nullptr;
  size_t n_ = 0;
  int pending_ = 0;
  unsigned long long gen_ = 0;
  bool stop_ = false;
};

struct shockidx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ek0 = nullptr, ek1 = nullptr;
  hipEvent_t stage_ev[NSTAGE] = {nullptr, nullptr};
  uint8_t *d_in = nullptr;
  u64 d_in_cap = 0;
  u64 *d_rows = nullptr;
  u64 d_rows_cap = 0;  // rows
  u64 *d_status = nullptr;
  u64 *d_detail = nullptr;
  u64 *d_fix = nullptr;  // k_fixup queue (FixRec, 32 bytes each), tiles_cap items
  u64 tiles_cap = 0;
  uint8_t *d_small = nullptr;  // badkey[2] | counters[2][NCOUNTERS] | result | detect
  u32 epoch = 0;               // build epoch for the look-back words (1..EPOCH_MASK)
  bool slots_dirty = false;    // a build took an epoch and did not reach its finalize
  int spec_fmt = 0;            // the last detected format (speculated by the next AUTO build)
  u64 *d_timing = nullptr;     // diagnostic phase timing buffer (SHOCKIDX_TIMING)
  u32 tiles_grid = 0;               // persistent grid of the tile passes (CUs x co-resident)
  uint8_t *h_stage[NSTAGE] = {nullptr, nullptr};
  DevResult *h_res = nullptr;
  CopyPool *pool = nullptr;        // host memcpy threads for the host-memory entry points
  uint8_t *d_sub = nullptr;        // subset / gather workspace
  u64 d_sub_cap = 0;
  int *h_det = nullptr;
  u64 ws_cap = 0;                  // SHOCKIDX_WORKSPACE_CAP: trim the caches above this after a call
  u64 dev_cap = 0;                 // device bytes a build may hold (0: what the device has free;
                                   //   shockidx_ctx_set_dev_cap / SHOCKIDX_DEV_CAP)
  u32 *d_fqstage = nullptr;        // FASTQ tile pass: provisional rows (TILE / 64 per tile)
  u64 fqstage_cap = 0;             //   (u32 entries)
  u32 *d_fqtiles = nullptr;        //   per-tile results (FQ_TILE_WORDS per tile)
  u64 fqtiles_cap = 0;
  uint8_t *d_cra = nullptr;        // speculative chunkrecord: FASTQ record table / FASTA tile counts
  u64 cra_cap = 0;                 //   (bytes)
  uint8_t *d_crb = nullptr;        //   node positions, jump tables, path, results (bytes)
  uint8_t *d_slot[2] = {nullptr, nullptr};  // fd builds within the device cap: the two slab slots
  u64 slot_cap = 0;                //   (bytes each)
  u64 crb_cap = 0;
  u32 cr_grid = 0;                 //   k_cr_verify persistent grid
  hipStream_t s_copy = nullptr;    // slab-pipelined host builds: the H2D stream
  uint8_t *h_rows[2] = {nullptr, nullptr};  // slab-pipelined fd builds: pinned row staging (D2H)
  // download filters over FASTQ: the tile pass keeps each record's line ends (k_fq_tiles<true>)
  bool want_spans = false;
  uint16_t *d_fqlines = nullptr;
  u64 fqlines_cap = 0;             //   (u16 entries)
  SlabParams last_p;               // the last FASTQ tile pass's parameters (k_fq_spans_place)
  bool last_spans = false;         //   its line ends are in d_fqlines
  // test hooks (shockidx_debug_inject, not in the public header): bit0 a freshly grown status
  // array is filled with published words of the next build's epoch before it is zeroed, bit1
  // after it is zeroed (what a zeroing that lost a race with the build would leave), bit2 the
  // finalize reports one record short
  u32 inject = 0;
};

namespace {

constexpr u64 SPEC_MIN_BYTES = 1ull << 20;  // smaller AUTO builds detect first (a re-run costs little)
constexpr size_t SMALL_BADKEY = 0, SMALL_COUNTERS = 64, SMALL_RESULT = 128, SMALL_DETECT = 320, SMALL_CHUNK = 384,
                 SMALL_SLABSUM = 448, SMALL_BYTES = 512;  // badkey slots at +0/+8, counter slots at +64/+80

int set_hip(shockidx_result *r, hipError_t e, const char *what) {
  if (r) {
    snprintf(r->err, sizeof r->err, "%s: %s", what, hipGetErrorString(e));
    r->err_len = strlen(r->err);
    r->status = SHOCKIDX_EHIP;
  }
  return SHOCKIDX_EHIP;
}

int set_msg(shockidx_result *r, int code, const char *msg) {
  if (r) {
    snprintf(r->err, sizeof r->err, "%s", msg);
    r->err_len = strlen(r->err);
    r->status = code;
  }
  return code;
}

#define HIPCHK(expr, what)                      \
  do {                                          \
    hipError_t _e = (expr);                     \
    if (_e != hipSuccess) return set_hip(res, _e, what); \
  } while (0)

void reset_result(shockidx_result *r) {
  if (!r) return;
  memset(r, 0, sizeof *r);
}

// dev knob (placement probes): SHOCKIDX_CONTIG_WS bit 1 = the tile status words, bit 2 = the tile
// pass's record-start slots in contiguous memory
bool verify_rows() {
  const char *v = getenv("SHOCKIDX_VERIFY");
  return v && *v && strcmp(v, "0") != 0;
}

// "2147483648", "2G", "512M", "64K" (binary units); anything unparsable is 0 (no cap)
u64 parse_bytes(const char *v) {
  char *end = nullptr;
  const double x = strtod(v, &end);
  if (!(x > 0) || end == v) return 0;
  const double m = (*end == 'G' || *end == 'g') ? 1073741824.0 : (*end == 'M' || *end == 'm') ? 1048576.0
                   : (*end == 'K' || *end == 'k') ? 1024.0 : 1.0;
  return x * m < 1.8e19 ? (u64)(x * m) : ~0ull;
}

bool ws_contig(int bit) {
  const char *e = getenv("SHOCKIDX_CONTIG_WS");
  return e && (atoi(e) & bit);
}
int ensure_dev(shockidx_ctx *c, void **p, u64 *cap, u64 need, size_t elem, shockidx_result *res,
               bool node = false) {
  if (*cap >= need && *p) return 0;
  if (*p) { (void)hipFree(*p); *p = nullptr; *cap = 0; }
  u64 want = need + need / 8 + 64;
  HIPCHK(sidx_host::dev_malloc(p, want * elem + 64, node), "hipMalloc");
  *cap = want;
  (void)c;
  return 0;
}

// device bytes held by the context's grow-only caches (input staging, rows, tile status,
// scan and subset workspaces)
u64 workspace_bytes(const shockidx_ctx *c) {
  return c->d_in_cap + 16 * c->d_rows_cap + 13 * 8 * c->tiles_cap + c->d_sub_cap +
         4 * (c->fqstage_cap + c->fqtiles_cap) + 2 * c->fqlines_cap + c->cra_cap + c->crb_cap + 2 * c->slot_cap;
}

// free the large caches (they regrow on demand); the tile status words go only with keep = 0
void trim_workspace(shockidx_ctx *c, u64 keep) {
  if (workspace_bytes(c) <= keep) return;
  (void)hipStreamSynchronize(c->stream);
  auto drop = [](void *&p, auto &cap) {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  };
  drop((void *&)c->d_in, c->d_in_cap);
  drop((void *&)c->d_rows, c->d_rows_cap);
  drop((void *&)c->d_sub, c->d_sub_cap);
  drop((void *&)c->d_fqstage, c->fqstage_cap);
  drop((void *&)c->d_fqtiles, c->fqtiles_cap);
  drop((void *&)c->d_fqlines, c->fqlines_cap);
  c->last_spans = false;
  drop((void *&)c->d_cra, c->cra_cap);
  drop((void *&)c->d_crb, c->crb_cap);
  for (int i = 0; i < 2; ++i) {
    if (c->d_slot[i]) (void)hipFree(c->d_slot[i]);
    c->d_slot[i] = nullptr;
  }
  c->slot_cap = 0;
  if (keep == 0 || workspace_bytes(c) > keep) {
    (void)hipFree(c->d_status);
    (void)hipFree(c->d_detail);
    (void)hipFree(c->d_fix);
    c->d_status = c->d_detail = c->d_fix = nullptr;
    c->tiles_cap = 0;  // a fresh (zeroed) status array comes back with the next build
  }
}

// trims the caches to the context's cap when a host-facing call returns
struct TrimGuard {
  shockidx_ctx *c;
  ~TrimGuard() {
    if (c && c->ws_cap) trim_workspace(c, c->ws_cap);
  }
};

// test hook: every status word published (INC) with the next build's epoch and payload 0, on
// the build stream -- the stale look-back words a recycled allocation could hold
hipError_t poison_status(shockidx_ctx *c, u64 words) {
  const u64 w = FLAG_INC | ((u64)((c->epoch + 1) & EPOCH_MASK) << EPOCH_SHIFT);
  std::vector<u64> h(words, w);
  hipError_t e = hipMemcpyAsync(c->d_status, h.data(), words * sizeof(u64), hipMemcpyHostToDevice, c->stream);
  return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
}

int ensure_tiles(shockidx_ctx *c, u64 ntiles, shockidx_result *res) {
  if (c->tiles_cap >= ntiles && c->d_status) return 0;
  // the fresh array is zeroed, so any epoch >= 1 is unpublished; the epoch keeps counting so
  // the first-bad / counter slots keep alternating (finalize resets the next build's slot)
  if (c->d_status) (void)hipFree(c->d_status);
  if (c->d_detail) (void)hipFree(c->d_detail);
  if (c->d_fix) (void)hipFree(c->d_fix);
  c->d_fix = nullptr;
  c->d_status = nullptr;
  c->d_detail = nullptr;
  u64 want = ntiles + ntiles / 8 + 64;
  // status words: slab aggregate (last tile's word) | line: last '\n' per tile | its max scan |
  // scan look-back words (two scans) | tile aggregates | their exclusive prefixes
  HIPCHK(sidx_host::dev_malloc((void **)&c->d_status, 7 * want * sizeof(u64), ws_contig(1)), "hipMalloc(status)");
  // detail slots: one per tile (+1) and one per k_fixup queue item (the FASTA tile pass)
  HIPCHK(hipMalloc((void **)&c->d_detail, 4 * want * sizeof(u64)), "hipMalloc(detail)");
  HIPCHK(hipMalloc((void **)&c->d_fix, 4 * want * sizeof(u64)), "hipMalloc(fix)");
  // on the build stream and waited for: a null-stream memset is not ordered with the
  // non-blocking context stream, and a reused allocation's old look-back words could be read
  if (c->inject & 1) HIPCHK(poison_status(c, 7 * want), "poison");
  HIPCHK(hipMemsetAsync(c->d_status, 0, 7 * want * sizeof(u64), c->stream), "hipMemset(status)");
  if (c->inject & 2) HIPCHK(poison_status(c, 7 * want), "poison");
  HIPCHK(hipStreamSynchronize(c->stream), "hipMemset(status) sync");
  c->tiles_cap = want;
  return 0;
}

// resolve kind/fmt into the kernel format (device detection when AUTO).  With `gate`, an AUTO
// record build of a context whose last detection found FASTQ or FASTA speculates that format:
// k_detect is launched without waiting for it, *gate points at its result and the pipeline's
// kernels run only if it matches (SlabParams::gate); one host round trip per build instead of two.
int resolve_format(shockidx_ctx *c, const uint8_t *d_data, u64 n, int kind, int fmt, hipStream_t s,
                   int *kfmt, shockidx_result *res, const int **gate = nullptr) {
  if (gate) *gate = nullptr;
  if (kind == SHOCKIDX_LINE) { *kfmt = F_LINE; return 0; }
  if (kind != SHOCKIDX_RECORD) return set_msg(res, SHOCKIDX_EINVAL, "invalid index kind");
  if (fmt == SHOCKIDX_FMT_AUTO) {
    int *d_det = (int *)(c->d_small + SMALL_DETECT);
    HIPCHK(sidx_launch_detect(d_data, n, d_det, s), "detect launch");
    if (gate && n >= SPEC_MIN_BYTES && (c->spec_fmt == SHOCKIDX_FMT_FASTQ || c->spec_fmt == SHOCKIDX_FMT_FASTA)) {
      *gate = d_det;
      *kfmt = c->spec_fmt;
      return 0;
    }
    HIPCHK(hipMemcpyAsync(c->h_det, d_det, 2 * sizeof(int), hipMemcpyDeviceToHost, s), "detect copy");
    HIPCHK(hipStreamSynchronize(s), "detect sync");
    fmt = c->h_det[0];
    c->spec_fmt = fmt;
    if (fmt == SHOCKIDX_FMT_NONE) {
      // errors.go:20 via multi.go:61
      return set_msg(res, SHOCKIDX_EFORMAT, "Invalid file type for filter");
    }
  }
  if (fmt != SHOCKIDX_FMT_FASTA && fmt != SHOCKIDX_FMT_FASTQ && fmt != SHOCKIDX_FMT_SAM && fmt != SHOCKIDX_FMT_LINE)
    return set_msg(res, SHOCKIDX_EINVAL, "invalid format");
  *kfmt = fmt;
  return 0;
}

// After a gated build: the speculation was wrong (flag 16) -> the detected format, or Go's
// error for none.  Returns 2 when the caller must re-run with *kfmt (0: the speculation held).
int respeculate(shockidx_ctx *c, const DevResult &dr, int *kfmt, shockidx_result *res) {
  if (!(dr.flags & 16)) return 0;
  const int det = (int)dr.detected;
  c->spec_fmt = det;
  res->format = SHOCKIDX_FMT_NONE;
  if (det == SHOCKIDX_FMT_NONE) return set_msg(res, SHOCKIDX_EFORMAT, "Invalid file type for filter");
  if (det != SHOCKIDX_FMT_FASTA && det != SHOCKIDX_FMT_FASTQ && det != SHOCKIDX_FMT_SAM)
    return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: detected format");
  *kfmt = det;
  res->format = det;
  return 2;
}

const char *status_message(u32 code) {
  switch (code) {
    case ST_FQ_TRUNC: return "Invalid format: truncated fastq record";
    case ST_FQ_EMPTYLINES: return "Invalid format: empty line(s) between records";
    case ST_FQ_NOAT: return "Invalid format: id line does not start with @";
    case ST_FQ_NOID: return "Invalid format: missing sequence ID";
    case ST_FQ_EMPTYSEQ: return "Invalid format: empty sequence";
    case ST_FQ_NOPLUS: return "Invalid format: plus line does not start with +";
    case ST_FQ_IDMISMATCH: return "Invalid format: quality ID does not match sequence ID";
    case ST_FQ_LENMISMATCH: return "Invalid format: length of sequence and quality lines do not match";
    default: return nullptr;
  }
}

std::mutex &device_mutex(int device) {
  static std::mutex mu[64];
  return mu[device & 63];
}

// Slab geometry of one index pass (a single-GPU build is one slab = the whole file).
struct SlabGeom {
  u64 n, end, front, base, state_in, row_base;
  int eof, file_start;
  void *d_summary;
  u32 seq = 0;  // the summary's build tag (shockidx_slab.seq)
};

// One device-resident index pass.  Fills *dr (host copy of the device result).
int run_index(shockidx_ctx *c, const uint8_t *d_data, u64 n, int kfmt, u64 *d_rows, u64 row_cap,
              hipStream_t s, DevResult *dr, shockidx_result *res, const SlabGeom *geom = nullptr,
              bool general = false, const int *gate = nullptr) {
  const u64 ntiles = n ? (n + TILE - 1) / TILE : 1;
  if (ntiles >= (1ull << KEY_TILE_BITS)) return set_msg(res, SHOCKIDX_EINVAL, "input too large for one slab");
  if (int rc = ensure_tiles(c, ntiles, res)) return rc;
  const bool fq_tiles0 = !general && kfmt == F_FASTQ;
  const bool fa_tiles0 = !general && kfmt == F_FASTA && (!geom || n > 0) && sidx_fa_tiles() &&
                         2 * c->tiles_cap < (1ull << KEY_TILE_BITS);
  const bool ln_tiles0 = !general && kfmt == F_LINE && n > 0 && sidx_line_tiles();
  // SAM: single-slab builds (slabs keep the two-pass build and its halo handling)
  const bool sm_tiles0 = !general && kfmt == F_SAM && n > 0 && !geom && sidx_sam_tiles();
  if (fq_tiles0 || fa_tiles0 || ln_tiles0 || sm_tiles0) {  // provisional rows and per-tile results
    // (FASTQ: a 128-byte line + an overflow slot per tile, sidx_kernels.hip fq_start; 1 KiB per tile here)
    if (int rc = ensure_dev(c, (void **)&c->d_fqstage, &c->fqstage_cap,
                            (ln_tiles0 || sm_tiles0) ? ntiles * (TILE / 32) : (ntiles + c->tiles_grid + 16) * (TILE / 64), 4,
                            res, ws_contig(2)))
      return rc;
    if (int rc = ensure_dev(c, (void **)&c->d_fqtiles, &c->fqtiles_cap, ntiles * FQ_TILE_WORDS, 4, res)) return rc;
  }
  if (fq_tiles0 && c->want_spans) {
    if (int rc = ensure_dev(c, (void **)&c->d_fqlines, &c->fqlines_cap, ntiles * 3 * (TILE / 64), 2, res)) return rc;
  }
  if (getenv("SHOCKIDX_TIMING") && !c->d_timing) {
    HIPCHK(hipMalloc((void **)&c->d_timing, 9 * 8 * 65536), "hipMalloc(timing)");
  }
  // A build that stopped between taking its epoch and its finalize (a launch or sync error)
  // left its first-bad / counter slot, scan tickets included, unreset: reset both slots before
  // anything reads them (k_scan_excl would otherwise wait on look-back words nobody writes).
  if (c->slots_dirty) {
    HIPCHK(hipMemsetAsync(c->d_small + SMALL_BADKEY, 0xFF, 16, s), "slot reset");
    HIPCHK(hipMemsetAsync(c->d_small + SMALL_COUNTERS, 0, 2 * 4 * NCOUNTERS, s), "slot reset");
    c->slots_dirty = false;
  }
  // next epoch (taken only once every allocation above succeeded); when the 14-bit epoch wraps,
  // clear the status array so no stale word can carry the current epoch
  if (++c->epoch > EPOCH_MASK) {
    HIPCHK(hipMemsetAsync(c->d_status, 0, 7 * c->tiles_cap * sizeof(u64), s), "status clear");
    c->epoch = 2;  // keep the slot parity alternating across the wrap (EPOCH_MASK is odd)
  }
  c->slots_dirty = true;  // until this build's finalize has run (the sync below)
  const u32 slot = c->epoch & 1;
  SlabParams p;
  memset(&p, 0, sizeof p);
  p.data = d_data;
  p.n = n;
  p.end = geom ? geom->end : n;
  p.front = geom ? geom->front : 0;
  p.base = geom ? geom->base : 0;
  p.state_in = geom ? geom->state_in : 0;
  p.row_base = geom ? geom->row_base : 0;
  p.summary = geom ? (u64 *)geom->d_summary : nullptr;
  p.row_cap = row_cap;
  p.rows = d_rows;
  p.status = c->d_status;
  p.pcnt = c->d_status + c->tiles_cap;
  p.ppre = c->d_status + 2 * c->tiles_cap;
  p.scan_look[0] = c->d_status + 3 * c->tiles_cap;
  p.scan_look[1] = c->d_status + 4 * c->tiles_cap;
  p.fq_agg = c->d_status + 5 * c->tiles_cap;
  p.tile_excl = c->d_status + 6 * c->tiles_cap;
  p.pgrid = c->tiles_grid < ntiles ? c->tiles_grid : (u32)ntiles;
  p.fix = general ? nullptr : c->d_fix;  // null: the two-pass build (k_index1) for every format
  p.fixcap = (u32)c->tiles_cap;
  p.badkey = (u64 *)(c->d_small + SMALL_BADKEY + 8 * slot);
  p.badkey_next = (u64 *)(c->d_small + SMALL_BADKEY + 8 * (slot ^ 1));
  p.detail = c->d_detail;
  p.counters = (u32 *)(c->d_small + SMALL_COUNTERS + 4 * NCOUNTERS * slot);
  p.counters_next = (u32 *)(c->d_small + SMALL_COUNTERS + 4 * NCOUNTERS * (slot ^ 1));
  p.ntiles = (u32)ntiles;
  p.epoch = c->epoch;
  p.seq = geom ? geom->seq : 0;
  p.inject = (c->inject & 4) ? 1u : 0u;
  p.eof = geom ? geom->eof : 1;
  p.file_start = geom ? geom->file_start : 1;
  p.gate = gate;
  p.gate_fmt = kfmt;
  if (const char *dbg = getenv("SHOCKIDX_DEBUG")) p.debug = (u32)atoi(dbg);  // SIDX_DIAG variant ablations
  if (getenv("SHOCKIDX_TIMING")) {  // diagnostic phase timing: per-workgroup cycle sums
    HIPCHK(hipMemsetAsync(c->d_timing, 0, 9 * 8 * 65536, s), "timing clear");
    p.timing = c->d_timing;
  }
  DevResult *d_res = (DevResult *)(c->d_small + SMALL_RESULT);
  // tile passes (one read of the input): FASTQ, FASTA (detail slots of tiles + queue items
  // within the key) and line, single builds and slabs alike; SAM single builds.  Otherwise (SAM
  // slabs, the general re-run) the two-pass build (k_tile_agg + scan + k_index1).
  const bool tiles = !general && p.fix;
  const bool fq_tiles = tiles && fq_tiles0;
  const bool fa_tiles = tiles && fa_tiles0;
  const bool ln_tiles = tiles && ln_tiles0;
  const bool sm_tiles = tiles && sm_tiles0;
  if (fq_tiles || fa_tiles || ln_tiles || sm_tiles) {
    p.fq_stage = c->d_fqstage;
    p.fq_tiles = c->d_fqtiles;
  }
  p.fq_lines = (fq_tiles && c->want_spans) ? c->d_fqlines : nullptr;
  c->last_spans = false;
  // One build's device work at a time per GPU: each build alone saturates HBM, so builds
  // from different contexts (concurrent goroutines, §8(b) "Threading") run back to back
  // instead of splitting the CUs.  Host staging of other builds still overlaps.
  std::unique_lock<std::mutex> device_lock(device_mutex(c->device));
  // the build's device time runs from its first kernel's start to the end of its last one: a
  // tile pass records its start (and end) in its own dispatch packet (hipExtLaunchKernel), so
  // its start event is ev0; the two-pass build brackets its kernels with stream events
  const bool tile_pass = fq_tiles || fa_tiles || ln_tiles || sm_tiles;
  hipEvent_t k0 = tile_pass ? c->ev0 : c->ek0;
  if (!tile_pass) HIPCHK(hipEventRecord(c->ev0, s), "event");
  if (fq_tiles) HIPCHK(sidx_launch_fq_tiles(&p, d_res, s, k0, c->ek1), "tile pass launch");
  else if (fa_tiles) HIPCHK(sidx_launch_fa_tiles(&p, d_res, s, k0, c->ek1), "FASTA tile pass launch");
  else if (ln_tiles) HIPCHK(sidx_launch_line_tiles(&p, d_res, s, k0, c->ek1), "line tile pass launch");
  else if (sm_tiles) HIPCHK(sidx_launch_sam_tiles(&p, d_res, s, k0, c->ek1), "SAM tile pass launch");
  else HIPCHK(sidx_launch_index(kfmt, &p, d_res, s, k0, c->ek1), "index launch");
  if (res) res->path = (fq_tiles || fa_tiles || ln_tiles || sm_tiles) ? 1u : 2u;
  HIPCHK(hipEventRecord(c->ev1, s), "event");
  // SHOCKIDX_VERIFY (the GPU test suite): the whole table's contiguity, after the timed kernels
  if (d_rows && verify_rows()) HIPCHK(sidx_launch_verify_rows(d_rows, p.row_base, row_cap, d_res, s), "verify launch");
  HIPCHK(hipMemcpyAsync(c->h_res, d_res, sizeof(DevResult), hipMemcpyDeviceToHost, s), "result copy");
  HIPCHK(hipStreamSynchronize(s), "index sync");
  c->slots_dirty = false;
  if (p.fq_lines) {
    c->last_p = p;
    c->last_spans = true;
  }
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
  if (res) res->kernel_ms += ms;
  float kms = 0.f;
  (void)hipEventElapsedTime(&kms, k0, c->ek1);
  if (res) res->index_ms = kms;
  *dr = *c->h_res;
  device_lock.unlock();
  // the fix-up queue overflowed (pathological input): redo the build two-pass (the next epoch
  // uses the other first-bad / counter slots, already reset)
  if ((dr->flags & 8) && !general) {
    if (res) res->reruns++;
    return run_index(c, d_data, n, kfmt, d_rows, row_cap, s, dr, res, geom, true, gate);
  }
  return 0;
}

// Translate the device result into (count, status, err).  Returns SHOCKIDX_OK,
// SHOCKIDX_EFORMAT, or a negative code.  FASTA messages read the piece from d_data.
int translate(shockidx_ctx *c, const DevResult &dr, const uint8_t *d_data, hipStream_t s,
              shockidx_result *res) {
  res->count = dr.count;
  res->fixups = dr.fixups;
  res->fix_tiles = dr.fix_tiles;
  res->state_out = dr.state_out;
  res->term_code = dr.code;
  res->flags = dr.flags;
  if (dr.flags & 2) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: device invariant violated");
  if (dr.flags & 4) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: slab halo exhausted");
  if (dr.code == ST_OK || dr.code == ST_END || dr.code == ST_ABSENT) {
    res->status = SHOCKIDX_OK;
    return SHOCKIDX_OK;
  }
  if (dr.code == ST_FA_INVALID) {
    // fasta.go:115-121: fmt.Errorf("Invalid fasta entry: %s", read[0:min(50, len(read))])
    static const char pre[] = "Invalid fasta entry: ";
    const u64 show = dr.err_len < 50 ? dr.err_len : 50;
    memcpy(res->err, pre, sizeof pre - 1);
    if (show) {
      hipError_t e = hipMemcpyAsync(res->err + sizeof pre - 1, d_data + dr.err_pos, show,
                                    hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) return set_hip(res, e, "error text copy");
    }
    res->err_len = sizeof pre - 1 + show;
    res->err[res->err_len] = 0;
    res->status = SHOCKIDX_EFORMAT;
    return SHOCKIDX_EFORMAT;
  }
  const char *m = status_message(dr.code);
  if (!m) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: unknown device status");
  return set_msg(res, SHOCKIDX_EFORMAT, m);
}

// Index d_data (already in c->d_in or caller memory) into c->d_rows, growing on overflow.
int build_resident(shockidx_ctx *c, const uint8_t *d_data, u64 n, int kind, int fmt, hipStream_t s,
                   shockidx_result *res) {
  int kfmt = 0;
  const int *gate = nullptr;
  if (int rc = resolve_format(c, d_data, n, kind, fmt, s, &kfmt, res, &gate)) return rc;
  res->format = kfmt == F_LINE ? SHOCKIDX_FMT_LINE : kfmt;
  u64 cap = kfmt == F_LINE ? n / 16 + 4096 : n / 32 + 4096;
  for (int attempt = 0; attempt < 3; ++attempt) {
    if (int rc = ensure_dev(c, (void **)&c->d_rows, &c->d_rows_cap, cap, 16, res)) return rc;
    DevResult dr;
    if (int rc = run_index(c, d_data, n, kfmt, c->d_rows, c->d_rows_cap, s, &dr, res, nullptr, false, gate)) return rc;
    if (gate) {
      gate = nullptr;
      if (int rc = respeculate(c, dr, &kfmt, res)) {
        if (rc < 0 || rc == SHOCKIDX_EFORMAT) return rc;
        res->reruns++;
        continue;  // the detected format, ungated
      }
    }
    if (dr.flags & 1) {  // row capacity overflow: grow to the exact count and rerun
      cap = dr.count;
      res->reruns++;
      continue;
    }
    return translate(c, dr, d_data, s, res);
  }
  return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: row capacity");
}

// Copy `count` rows from c->d_rows into a malloc'ed host table via pinned staging: the DMA
// of chunk i+1 overlaps the (threaded) host copy of chunk i.
// The caller's table (free()-able, released by shockidx_free).  Large tables are 2 MiB aligned
// and advised for transparent huge pages: the threaded copy out of the staging buffers then
// faults the fresh memory in 2 MiB pages instead of 4 KiB ones.
uint64_t *alloc_rows_out(size_t bytes) {
  constexpr size_t HUGE = 2u << 20;
  if (bytes < 4 * HUGE) return (uint64_t *)malloc(bytes ? bytes : 16);
  void *p = nullptr;
  if (posix_memalign(&p, HUGE, (bytes + HUGE - 1) & ~(HUGE - 1))) return nullptr;
  (void)madvise(p, (bytes + HUGE - 1) & ~(HUGE - 1), MADV_HUGEPAGE);
  return (uint64_t *)p;
}

// Device rows -> host memory through the pinned staging: the DMA of chunk i + 1 overlaps the
// (threaded) host copy of chunk i.
int rows_to_host(shockidx_ctx *c, const u64 *d_src, size_t bytes, uint8_t *dst, hipStream_t s,
                 shockidx_result *res) {
  size_t issued = 0, done = 0;
  int i = 0;
  auto issue = [&](int b) -> hipError_t {
    const size_t k = bytes - issued < STAGE_BYTES ? bytes - issued : STAGE_BYTES;
    hipError_t e = hipMemcpyAsync(c->h_stage[b], (const uint8_t *)d_src + issued, k, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(c->stage_ev[b], s);
    issued += k;
    return e;
  };
  hipError_t e = bytes ? issue(0) : hipSuccess;
  while (e == hipSuccess && done < bytes) {
    const size_t k = bytes - done < STAGE_BYTES ? bytes - done : STAGE_BYTES;
    if (issued < bytes) e = issue(i ^ 1);
    if (e == hipSuccess) e = hipEventSynchronize(c->stage_ev[i]);
    if (e != hipSuccess) break;
    c->pool->copy(dst + done, c->h_stage[i], k);
    done += k;
    i ^= 1;
  }
  if (e != hipSuccess) return set_hip(res, e, "rows copy");
  return 0;
}

int fetch_rows(shockidx_ctx *c, u64 count, hipStream_t s, uint64_t **rows, shockidx_result *res) {
  const double t0 = now_ms();
  const size_t bytes = (size_t)count * 16;
  uint64_t *out = alloc_rows_out(bytes);
  if (!out) return set_msg(res, SHOCKIDX_ENOMEM, "out of host memory");
  if (int rc = rows_to_host(c, c->d_rows, bytes, (uint8_t *)out, s, res)) {
    free(out);
    return rc;
  }
  *rows = out;
  res->d2h_ms += now_ms() - t0;
  return 0;
}

// Stage n bytes into c->d_in (from byte `from` on).  `fill(dst, off, len)` produces host bytes
// (memcpy / pread).
template <class Fill>
int stage_in(shockidx_ctx *c, u64 n, hipStream_t s, Fill fill, shockidx_result *res, u64 from = 0) {
  const double t0 = now_ms();
  if (int rc = ensure_dev(c, (void **)&c->d_in, &c->d_in_cap, n + 64, 1, res, true)) return rc;
  u64 off = from;
  int i = 0;
  while (off < n) {
    const size_t k = n - off < STAGE_BYTES ? (size_t)(n - off) : STAGE_BYTES;
    HIPCHK(hipEventSynchronize(c->stage_ev[i]), "stage wait");  // buffer i free again
    if (int rc = fill(c->h_stage[i], off, k)) return rc;
    HIPCHK(hipMemcpyAsync(c->d_in + off, c->h_stage[i], k, hipMemcpyHostToDevice, s), "H2D");
    HIPCHK(hipEventRecord(c->stage_ev[i], s), "stage event");
    off += k;
    i ^= 1;
  }
  HIPCHK(hipStreamSynchronize(s), "H2D sync");
  res->h2d_ms += now_ms() - t0;
  return 0;
}

// Host memory the GPU can DMA from directly (hipHostRegister'ed or hipHostMalloc'ed)
bool host_pinned(const void *p, u64 n) {
  if (!p || !n) return false;
  hipPointerAttribute_t a0, a1;
  const hipError_t e0 = hipPointerGetAttributes(&a0, p);
  (void)hipGetLastError();  // a plain pageable pointer reports an error here
  if (e0 != hipSuccess || a0.type != hipMemoryTypeHost) return false;
  // the last byte too, in the same mapping: a buffer only partly registered (or two adjacent
  // registrations) takes the staging path instead of a DMA that would run past the pinning
  const hipError_t e1 = hipPointerGetAttributes(&a1, (const uint8_t *)p + (n - 1));
  (void)hipGetLastError();
  return e1 == hipSuccess && a1.type == hipMemoryTypeHost && a0.devicePointer && a1.devicePointer &&
         (const uint8_t *)a1.devicePointer - (const uint8_t *)a0.devicePointer == (ptrdiff_t)(n - 1);
}
constexpr u64 PIN_PIECE = 1ull << 30;

// Host bytes of a file for stage_in: pread until every byte of [off, off + k) has arrived
// (Linux returns at most 0x7ffff000 bytes per call; short reads and EINTR are retried).
struct PreadFill {
  int fd;
  shockidx_result *res;
  CopyPool *pool;  // slices of each staging chunk are read by the pool's threads in parallel
  int operator()(uint8_t *dst, u64 off, size_t k) const {
    std::atomic<int> bad{0};
    const int fdl = fd;
    pool->parallel(k, [&, fdl](size_t a, size_t b) {
      size_t got = a;
      while (got < b && !bad.load(std::memory_order_relaxed)) {
        ssize_t r = pread(fdl, dst + got, b - got, (off_t)(off + got));
        if (r < 0) {
          if (errno == EINTR) continue;
          bad.store(errno ? errno : EIO);
          return;
        }
        if (r == 0) { bad.store(-1); return; }
        got += (size_t)r;
      }
    });
    const int e = bad.load();
    if (e == -1) return set_msg(res, SHOCKIDX_EIO, "unexpected end of file");
    if (e) return set_msg(res, SHOCKIDX_EIO, strerror(e));
    return 0;
  }
};
PreadFill pread_fill(shockidx_ctx *c, int fd, shockidx_result *res) { return PreadFill{fd, res, c->pool}; }

// Stage the file bytes [off, off + n) into c->d_in.  A file that maps goes to HBM straight out of
// the page cache: mapped read-only, pinned 256 MiB at a time (hipHostRegister), each piece DMA'd
// as soon as it is pinned, everything unpinned once the stream drains (the bytes cross host
// memory once; the fd pipeline below does the same per slab).  A file that does not map, or pages
// that do not pin, go (from there on) through the copy threads into the pinned staging.
// The page-cache DMA pins a node file's pages until its copy drains.  Bytes a single call may
// keep pinned (several large builds at once could lock that much host RAM):
// SHOCKIDX_PIN_CAP_GIB, else a quarter of the host's memory; past it the rest of the file goes
// through the pinned staging buffers (pread by the copy threads).
u64 pin_cap() {
  if (const char *e = getenv("SHOCKIDX_PIN_CAP_GIB")) {  // (clamped: a negative or non-numeric value pins nothing)
    const double g = atof(e);
    return g > 0 ? (u64)((g < 1e6 ? g : 1e6) * (double)(1ull << 30)) : 0;
  }
  const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
  return pages > 0 && psz > 0 ? (u64)pages * (u64)psz / 4 : (64ull << 30);
}
// Process-wide pinned host bytes: every page-cache DMA reserves what it pins from one
// budget, pin_cap(), before hipHostRegister and gives it back after unregistering, so concurrent
// builds (a gpuPoolSize of contexts, a multi-GPU group) cannot pin more than the cap together.
// A reservation that fails sends the bytes through the pinned staging buffers instead.
std::atomic<u64> g_pinned{0};
bool pin_reserve(u64 b) {
  const u64 cap = pin_cap();
  u64 cur = g_pinned.load();
  do {
    if (cur + b > cap) return false;
  } while (!g_pinned.compare_exchange_weak(cur, cur + b));
  return true;
}
void pin_release(u64 b) { g_pinned.fetch_sub(b); }


int stage_fd(shockidx_ctx *c, int fd, u64 off, u64 n, hipStream_t s, shockidx_result *res) {
  u64 done = 0;
  if (n >= (64ull << 20) && !getenv("SHOCKIDX_NO_MMAP_DMA")) {
    if (int rc = ensure_dev(c, (void **)&c->d_in, &c->d_in_cap, n + 64, 1, res, true)) return rc;
    const double t0 = now_ms();
    const u64 a0 = off & ~4095ull, lead = off - a0;
    const size_t maplen = (size_t)(((off + n + 4095) & ~4095ull) - a0);
    void *mp = mmap(nullptr, maplen, PROT_READ, MAP_SHARED, fd, (off_t)a0);
    if (mp != MAP_FAILED) {
      uint8_t *map = (uint8_t *)mp;
      constexpr u64 CH = 256ull << 20;
      u64 reg = 0, held = 0;
      hipError_t e = hipSuccess;
      for (u64 mlo = 0; mlo < maplen; mlo += CH) {
        const u64 mhi = maplen - mlo < CH ? maplen : mlo + CH;
        if (!pin_reserve(mhi - mlo)) break;  // over the process-wide pin budget: the rest through the staging buffers
        if (hipHostRegister(map + mlo, (size_t)(mhi - mlo), 0) != hipSuccess) {
          (void)hipGetLastError();
          pin_release(mhi - mlo);
          break;
        }
        ++reg;
        held += mhi - mlo;
        const u64 blo = mlo > lead ? mlo - lead : 0, bhi = mhi - lead < n ? mhi - lead : n;  // file bytes - off
        if (bhi > blo && (e = hipMemcpyAsync(c->d_in + blo, map + lead + blo, bhi - blo, hipMemcpyHostToDevice, s)) != hipSuccess)
          break;
        done = bhi;
      }
      const hipError_t se = hipStreamSynchronize(s);
      for (u64 k = 0; k < reg; ++k) (void)hipHostUnregister(map + k * CH);
      pin_release(held);
      munmap(mp, maplen);
      if (e != hipSuccess) return set_hip(res, e, "page-cache DMA");
      if (se != hipSuccess) return set_hip(res, se, "H2D sync");
      res->h2d_ms += now_ms() - t0;
    }
  }
  if (done >= n) return 0;
  const PreadFill pf = pread_fill(c, fd, res);
  return stage_in(c, n, s, [&](uint8_t *dst, u64 o, size_t k) -> int { return pf(dst, off + o, k); }, res, done);
}

// Slab-pipelined FASTQ record build of a pinned host body: the body crosses PCIe in 1 GiB
// slabs on a copy stream while the compute stream indexes slab k as soon as its bytes and a
// 4 MiB halo have arrived, with slab k - 1's exact end state as its incoming state (the slab
// kernels of the multi-GPU protocol, with no guess), and the calling thread copies slab k's
// rows out while later slabs are still arriving -- so only the last slab's index and rows
// are left after the H2D.  Anything but a clean slab (an error, a blank group before the end,
// a record past the halo, any device flag) falls back to the one-pass build of the whole body,
// which is in HBM by then.  *done = 0: not applicable (the caller runs the plain path).
constexpr u64 PIPE_SLAB = 1ull << 30, PIPE_HALO = 4ull << 20;
// the slab builds' end-of-build invariants (never expected: a violation is an internal error,
// not a short table)
const char *const SLAB_SEAM_MSG = "internal error: a slab's first row does not start where the previous slab's rows end";
const char *const SLAB_END_MSG = "internal error: the rows do not end at the end of the file";
int build_host_pipelined(shockidx_ctx *c, const void *data, u64 n, int kind, int fmt, uint64_t **rows,
                         shockidx_result *res, bool *done) {
  *done = false;
  if (kind != SHOCKIDX_RECORD || n < 2 * PIPE_SLAB || !host_pinned(data, n) ||
      (fmt != SHOCKIDX_FMT_AUTO && fmt != SHOCKIDX_FMT_FASTQ) || getenv("SHOCKIDX_NO_HOST_PIPE"))
    return 0;
  const double t0 = now_ms();
  hipStream_t s = c->stream;
  if (!c->s_copy) HIPCHK(hipStreamCreateWithFlags(&c->s_copy, hipStreamNonBlocking), "copy stream");
  if (int rc = ensure_dev(c, (void **)&c->d_in, &c->d_in_cap, n + 64, 1, res, true)) return rc;
  const u64 K = (n + PIPE_SLAB - 1) / PIPE_SLAB;
  std::vector<hipEvent_t> ev(K, nullptr);
  struct EvGuard {
    std::vector<hipEvent_t> &v;
    hipStream_t cs;
    ~EvGuard() {
      (void)hipStreamSynchronize(cs);
      for (auto e : v) if (e) (void)hipEventDestroy(e);
    }
  } guard{ev, c->s_copy};
  for (u64 k = 0; k < K; ++k) {
    HIPCHK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "event");
    const u64 lo = k * PIPE_SLAB, len = n - lo < PIPE_SLAB ? n - lo : PIPE_SLAB;
    HIPCHK(hipMemcpyAsync(c->d_in + lo, (const uint8_t *)data + lo, len, hipMemcpyHostToDevice, c->s_copy), "H2D");
    HIPCHK(hipEventRecord(ev[k], c->s_copy), "event");
  }
  *done = true;
  auto plain = [&]() -> int {  // the whole body, one pass (after every slab has arrived)
    HIPCHK(hipStreamSynchronize(c->s_copy), "H2D sync");
    const double th = now_ms();
    reset_result(res);
    res->h2d_ms = th - t0;
    int rc = build_resident(c, c->d_in, n, kind, fmt, s, res);
    if (rc < 0) return rc;
    if (int rc2 = fetch_rows(c, res->count, s, rows, res)) return rc2;
    res->total_ms = now_ms() - t0;
    return rc;
  };
  HIPCHK(hipStreamWaitEvent(s, ev[0], 0), "wait slab 0");
  int kfmt = 0;
  if (int rc = resolve_format(c, c->d_in, n, kind, fmt, s, &kfmt, res)) {
    if (rc < 0) return rc;
    return plain();  // no format: the plain build reports it
  }
  if (kfmt != SHOCKIDX_FMT_FASTQ) return plain();
  const u64 rcap = n / 32 + 4096;
  if (int rc = ensure_dev(c, (void **)&c->d_rows, &c->d_rows_cap, rcap, 16, res)) return rc;
  size_t out_cap = (size_t)(n / 128 + 4096) * 16;
  struct FreeDel {
    void operator()(uint8_t *p) const { free(p); }
  };
  std::unique_ptr<uint8_t, FreeDel> out((uint8_t *)alloc_rows_out(out_cap));  // freed on every error return
  if (!out) return set_msg(res, SHOCKIDX_ENOMEM, "out of host memory");
  u64 total = 0, state = 0, next_off = 0;
  double d2h = 0;
  for (u64 k = 0; k < K; ++k) {
    const u64 lo = k * PIPE_SLAB, nk = n - lo < PIPE_SLAB ? n - lo : PIPE_SLAB;
    const u64 endk = n - lo < nk + PIPE_HALO ? n - lo : nk + PIPE_HALO;
    const u64 need = (lo + endk - 1) / PIPE_SLAB;
    HIPCHK(hipStreamWaitEvent(s, ev[need], 0), "wait slab");
    SlabGeom g;
    g.n = nk;
    g.end = endk;
    g.front = lo;
    g.base = lo;
    g.state_in = state & 3;
    g.row_base = k ? 1 : 0;
    g.eof = lo + endk == n;
    g.file_start = k == 0;
    g.d_summary = c->d_small + SMALL_SLABSUM;
    DevResult dr;
    shockidx_result r2;
    reset_result(&r2);
    int rc = run_index(c, c->d_in + lo, nk, F_FASTQ, c->d_rows + 2 * total, rcap - total, s, &dr, &r2, &g);
    if (rc < 0) return set_msg(res, rc, r2.err);
    res->kernel_ms += r2.kernel_ms;
    res->index_ms += r2.index_ms;
    const bool last = lo + nk == n;
    const bool clean = rc == 0 && dr.flags == 0 && dr.count >= g.row_base &&
                       (dr.code == ST_OK || (last && (dr.code == ST_END || dr.code == ST_ABSENT)));
    if (!clean) {
      out.reset();
      return plain();
    }
    const u64 owned = dr.count - g.row_base;
    if ((total + owned) * 16 > out_cap) {
      size_t nc = out_cap;
      while ((total + owned) * 16 > nc) nc *= 2;
      uint8_t *o2 = (uint8_t *)realloc(out.get(), nc);
      if (!o2) return set_msg(res, SHOCKIDX_ENOMEM, "out of host memory");
      (void)out.release();
      out.reset(o2);
      out_cap = nc;
    }
    const double td = now_ms();
    if (int rc2 = rows_to_host(c, c->d_rows + 2 * total, owned * 16, out.get() + total * 16, s, res)) return rc2;
    d2h += now_ms() - td;
    if (owned) {  // the slab continues the table (record.go:51-83)
      const u64 *hr = (const u64 *)(out.get() + total * 16);
      if (hr[0] != next_off) return set_msg(res, SHOCKIDX_EINTERNAL, SLAB_SEAM_MSG);
      next_off = hr[2 * (owned - 1)] + hr[2 * (owned - 1) + 1];
    }
    total += owned;
    state = dr.state_out;
  }
  {  // the table ends at the file end, or before trailing blank lines (fastq.go:141-156)
    const uint8_t *hb = (const uint8_t *)data;
    if (next_off > n || (next_off < n && (hb[next_off] != '\n' || hb[n - 1] != '\n')))
      return set_msg(res, SHOCKIDX_EINTERNAL, SLAB_END_MSG);
  }
  if (total * 16 < out_cap) {
    uint8_t *o2 = (uint8_t *)realloc(out.get(), total ? total * 16 : 16);
    if (o2) {
      (void)out.release();
      out.reset(o2);
    }
  }
  *rows = (uint64_t *)out.release();
  res->count = total;
  res->format = SHOCKIDX_FMT_FASTQ;
  res->status = SHOCKIDX_OK;
  res->path = 3;  // the slab pipeline (the plain fallback reports its device build's path)
  res->d2h_ms = d2h;
  res->total_ms = now_ms() - t0;
  res->h2d_ms = res->total_ms - d2h - res->kernel_ms;  // the rest is waiting for the PCIe stream
  return SHOCKIDX_OK;
}

// record.go:35 tmpFilePath := fmt.Sprintf("%s/temp/%d%d.idx", conf.PATH_DATA, rand.Int(), rand.Int())
// (the caller passes PATH_DATA/temp as tmpdir)
std::string temp_idx_path(const char *tmpdir) {
  static std::atomic<unsigned long long> salt{0};
  std::mt19937_64 rng((unsigned long long)now_ms() * 1000003ull ^ (unsigned long long)getpid() ^ (salt++ << 20));
  return std::string(tmpdir) + "/" + std::to_string(rng() >> 1) + std::to_string(rng() >> 1) + ".idx";
}

// Where the rows of a slab-pipelined fd build go, as each slab's rows arrive in pinned host
// memory (called from the pipeline's index thread, rows in file order): the caller's table
// (shockidx_build_fd) or the temp .idx file (shockidx_create, pwrite at 16 * first row).
struct RowSink {
  virtual ~RowSink() {}
  virtual int put(const uint8_t *src, u64 first, u64 nrows, shockidx_result *res) = 0;
};
struct TableSink : RowSink {  // a malloc'ed table, grown as rows arrive (the caller frees it)
  uint8_t *out = nullptr;
  size_t cap = 0;
  // sized up front for the file (16 bytes per 32 input bytes: only the pages the rows touch are
  // ever faulted in), so the usual table is never copied while it grows
  explicit TableSink(u64 n) {
    cap = (size_t)(n / 32 + 4096) * 16;
    out = (uint8_t *)alloc_rows_out(cap);
    if (!out) cap = 0;
  }
  ~TableSink() override { free(out); }
  int put(const uint8_t *src, u64 first, u64 nrows, shockidx_result *res) override {
    const size_t need = (size_t)(first + nrows) * 16;
    if (need > cap) {
      size_t nc = cap ? cap : (64u << 20);
      while (nc < need) nc *= 2;
      uint8_t *o2 = (uint8_t *)alloc_rows_out(nc);
      if (!o2) return set_msg(res, SHOCKIDX_ENOMEM, "out of host memory");
      if (out) memcpy(o2, out, (size_t)first * 16);
      free(out);
      out = o2;
      cap = nc;
    }
    memcpy(out + (size_t)first * 16, src, (size_t)nrows * 16);
    return 0;
  }
};
struct FileSink : RowSink {  // the .idx temp file: rows are {u64 off, u64 len} LE (record.go:74-75)
  int fd = -1;
  int put(const uint8_t *src, u64 first, u64 nrows, shockidx_result *res) override {
    size_t left = (size_t)nrows * 16;
    off_t at = (off_t)(first * 16);
    while (left) {
      const ssize_t w = pwrite(fd, src, left > (1u << 30) ? (1u << 30) : left, at);
      if (w < 0) {
        if (errno == EINTR) continue;
        return set_msg(res, SHOCKIDX_EIO, strerror(errno));
      }
      src += w;
      at += w;
      left -= (size_t)w;
    }
    return 0;
  }
};

// Device bytes a build may hold: the context's cap (shockidx_ctx_set_dev_cap / SHOCKIDX_DEV_CAP),
// and never more than the device has free plus what this context already holds (its caches are
// freed or reused first).
u64 dev_budget(shockidx_ctx *c) {
  size_t fr = 0, tot = 0;
  u64 avail = ~0ull;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
    const u64 held = workspace_bytes(c);
    avail = (u64)fr + held > (256ull << 20) ? (u64)fr + held - (256ull << 20) : 0;
  } else {
    (void)hipGetLastError();
  }
  return c->dev_cap && c->dev_cap < avail ? c->dev_cap : avail;
}
// what a one-pass build of an n-byte node holds at its peak: the node, its rows (ensure_dev's
// growth included) and the per-tile workspaces
u64 one_pass_bytes(u64 n) { return n + n / 8 + (n / 32) * 16 * 9 / 8 + n / 8 + (64ull << 20); }

// Slab-pipelined build over a file descriptor -- the drop-in path: node.AsyncIndexer opens the
// node file and hands it to Create (node/index.go:107-121).  The file is DMA'd to HBM on the copy
// stream (out of the page cache, or through the pinned staging buffers); an index thread runs
// each slab as soon as its bytes and a 4 MiB halo have arrived, with the previous slab's exact end
// state as its incoming state (the multi-GPU slab kernels, no guess), and hands the slab's rows to
// the sink while later slabs are still being read -- so after the last byte crosses PCIe only the
// last slab's index and rows are left.  FASTQ, FASTA and line.
//
// Two layouts in HBM (round 6):
//  - whole: the node in one buffer (n bytes), 1 GiB slabs -- when one_pass_bytes(n) fits the
//    device budget, so the rare fallback below can index the node in place;
//  - ring: two slot buffers of S + 64 KiB + 4 MiB (slab k goes to slot k mod 2 with the 64 KiB
//    before it and its halo; the halo and front bytes cross PCIe twice, 0.4 %), S sized to the
//    budget -- so the device footprint does not grow with the node, like record.go's 4 KiB
//    bufio.Reader (record.go:51-83, fastq.go:136).  The producer reuses a slot once the index
//    thread is done with the slab in it.
// Anything but a clean slab (a format error, a record past the halo, a device flag, SAM, no
// detectable format) ends the slab walk.  Whole layout: the one-pass build of the whole file,
// which is in HBM by then (*fell_back = true, nothing reported to the caller).  Ring layout: the
// rows of the clean slabs before it are final (exact incoming states), and the rest of the file,
// from the start r of the first record not yet emitted, is re-read and indexed in one pass as a
// node of its own -- a record boundary resets every reader (FASTQ's skip loop and `empty`,
// FASTA's piece after UnreadByte, a line), so its rows are the file's rows shifted by r; its
// count and error complete the table.  The rest is walked through the same slots again, its
// first slab starting at r (*restart = r: build_fd_pipelined below loops), so a record longer than
// the halo but not than a slab costs one re-read of that record; only a record the walk cannot
// close from its own start (longer than a slab) takes the one-pass build of the rest, which needs
// one_pass_bytes of it within the budget, or the build fails with SHOCKIDX_ENOMEM.
// base > 0: this walk is such a rest -- the file bytes [base, base + n) as a node of its own
// (rows at absolute file offsets, numbered from row0; always the ring layout).
// *done = false: not applicable (small file, other kind), nothing was read.
int build_fd_walk(shockidx_ctx *c, int fd, u64 n, int kind, int fmt, RowSink &sink, shockidx_result *res,
                  bool *done, bool *fell_back, u64 base, u64 row0, u64 *restart) {
  *done = false;
  *fell_back = false;
  *restart = 0;
  if ((kind != SHOCKIDX_RECORD && kind != SHOCKIDX_LINE) || getenv("SHOCKIDX_NO_FD_PIPE") ||
      (kind == SHOCKIDX_RECORD && fmt != SHOCKIDX_FMT_AUTO && fmt != SHOCKIDX_FMT_FASTQ && fmt != SHOCKIDX_FMT_FASTA))
    return 0;
  const u64 budget = dev_budget(c);
  const bool ring = base || one_pass_bytes(n) > budget || getenv("SHOCKIDX_FD_RING");
  // slab bytes: 1 GiB; in the ring, what two slots and one slab's workspaces leave of the budget
  // (rows 16 B per 32 input bytes, tile words and starts ~1/16, status ~1/40: ~0.6 S; 2.7 S in all)
  constexpr u64 RFRONT = 64ull << 10, MIB = 1ull << 20;
  u64 S = PIPE_SLAB;
  if (ring) {
    const u64 fixed = 2 * (RFRONT + PIPE_HALO + 64) + 96 * MIB;
    S = budget > fixed ? (budget - fixed) * 10 / 27 : 0;
    S = S > PIPE_SLAB ? PIPE_SLAB : S & ~(16 * MIB - 1);
    if (S < 64 * MIB) return set_msg(res, SHOCKIDX_ENOMEM, "device memory: the build needs at least 256 MiB of its budget");
  }
  if (!ring && n < 2 * S) return 0;  // (whole layout: under 2 GiB the plain staging + one pass is as fast)
  const double t0 = now_ms();
  hipStream_t s = c->stream;
  if (!c->s_copy) HIPCHK(hipStreamCreateWithFlags(&c->s_copy, hipStreamNonBlocking), "copy stream");
  for (int i = 0; i < 2; ++i)
    if (!c->h_rows[i]) HIPCHK(hipHostMalloc((void **)&c->h_rows[i], STAGE_BYTES, 0), "hipHostMalloc(rows)");
  const u64 SLOT = RFRONT + S + PIPE_HALO + 64;
  uint8_t **slot = c->d_slot;  // (kept by the context, like its other caches, until a trim)
  if (ring) {
    if (c->slot_cap != SLOT) {
      // the caches of earlier (larger) builds go first: the node buffer of a one-pass build, rows
      trim_workspace(c, 0);
      for (int i = 0; i < 2; ++i) HIPCHK(sidx_host::dev_malloc((void **)&c->d_slot[i], SLOT, true), "hipMalloc(slab slot)");
      c->slot_cap = SLOT;
    } else if (c->d_in) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(c->d_in);
      c->d_in = nullptr;
      c->d_in_cap = 0;
    }
  } else {
    if (c->slot_cap) {  // (slots of an earlier build within a cap: not needed by this one)
      (void)hipStreamSynchronize(s);
      for (int i = 0; i < 2; ++i) {
        (void)hipFree(c->d_slot[i]);
        c->d_slot[i] = nullptr;
      }
      c->slot_cap = 0;
    }
    if (int rc = ensure_dev(c, (void **)&c->d_in, &c->d_in_cap, n + 64, 1, res, true)) return rc;
  }
  const u64 K = (n + S - 1) / S;
  // per slab its rows' device capacity (reused slab after slab); a slab with more rows (records
  // or lines under 32 bytes on average) overflows it and the slab walk ends (the fallback below)
  const u64 rcap = S / 32 + 4096;
  if (int rc = ensure_dev(c, (void **)&c->d_rows, &c->d_rows_cap, rcap, 16, res)) return rc;
  std::vector<hipEvent_t> ev(K, nullptr);
  struct EvGuard {
    std::vector<hipEvent_t> &v;
    hipStream_t cs;
    ~EvGuard() {
      (void)hipStreamSynchronize(cs);
      for (auto e : v) if (e) (void)hipEventDestroy(e);
    }
  } guard{ev, c->s_copy};
  for (u64 k = 0; k < K; ++k) HIPCHK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "event");
  *done = true;
  // slab k: file bytes [lo, lo + nk) owned, [lo, lo + endk) readable from dk, fk bytes before it
  auto slab_lo = [&](u64 k) { return k * S; };
  auto slab_n = [&](u64 k) { return n - k * S < S ? n - k * S : S; };
  auto slab_end = [&](u64 k) { const u64 lo = k * S, nk = slab_n(k); return n - lo < nk + PIPE_HALO ? n - lo : nk + PIPE_HALO; };
  auto slab_front = [&](u64 k) { return ring ? (k * S < RFRONT ? k * S : RFRONT) : k * S; };
  auto slab_ptr = [&](u64 k) -> uint8_t * { return ring ? slot[k & 1] + slab_front(k) : c->d_in + k * S; };

  std::mutex mu;
  std::condition_variable cv;
  u64 recorded = 0;        // slabs whose arrival event is recorded on the copy stream
  u64 freed = 0;           // slabs the index thread is done with (their slot may be refilled)
  bool prod_failed = false, ix_over = false;
  // index thread: slab k after its bytes (+ halo) have arrived
  int crc = 0;             // its result: 0 clean, 1 fall back, 2 no format, 3 a Go error in a slab (err_dr), < 0 error (message in cres)
  DevResult err_dr{};
  shockidx_result cres;
  reset_result(&cres);
  u64 total = row0, next_off = base, last_len = 0;  // rows so far; where the next row must start; the last row's length
  int kfmt = 0;
  double t_d2h = 0;
  std::thread ix([&] {
    struct Over {  // wakes the producer whatever way the thread ends
      std::mutex &m;
      std::condition_variable &v;
      bool &f;
      ~Over() {
        { std::lock_guard<std::mutex> g(m); f = true; }
        v.notify_all();
      }
    } over{mu, cv, ix_over};
    if (hipSetDevice(c->device) != hipSuccess) { crc = set_msg(&cres, SHOCKIDX_EHIP, "hipSetDevice"); return; }
    u64 state = 0;
    for (u64 k = 0; k < K; ++k) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return recorded > k || prod_failed; });
        if (recorded <= k) { crc = 1; return; }
      }
      if (hipStreamWaitEvent(s, ev[k], 0) != hipSuccess) { crc = set_msg(&cres, SHOCKIDX_EHIP, "wait slab"); return; }
      const u64 lo = slab_lo(k), nk = slab_n(k), endk = slab_end(k);
      if (k == 0) {
        int rc = resolve_format(c, slab_ptr(0), ring ? endk : n, kind, fmt, s, &kfmt, &cres);
        if (rc < 0) { crc = rc; return; }
        if (rc) { crc = 2; return; }  // no format (multi.go:43-62 reads the first 32 KiB only): reported as is
        if (kfmt != F_FASTQ && kfmt != F_FASTA && kfmt != F_LINE) { crc = 1; return; }
      }
      SlabGeom g;
      g.n = nk;
      g.end = endk;
      g.front = slab_front(k);
      g.base = base + lo;  // (rows and FASTA error pieces at file offsets)
      g.state_in = kfmt == F_FASTQ ? (state & 3) : kfmt == F_FASTA ? (state & 1) : 0;
      g.row_base = k ? 1 : 0;  // the record open at a later slab's start is the previous slab's
      g.eof = lo + endk == n;
      g.file_start = k == 0;
      g.d_summary = c->d_small + SMALL_SLABSUM;
      DevResult dr;
      shockidx_result r2;
      reset_result(&r2);
      int rc = run_index(c, slab_ptr(k), nk, kfmt, c->d_rows, c->d_rows_cap, s, &dr, &r2, &g);
      if (rc == 0 && dr.flags == 1 && dr.count > g.row_base &&
          ensure_dev(c, (void **)&c->d_rows, &c->d_rows_cap, dr.count - g.row_base + 4096, 16, &r2) == 0)
        // more rows than the slab's share (records or lines under 32 bytes on average): the
        // slab again into rows grown to its count, while its bytes are still in the slot
        rc = run_index(c, slab_ptr(k), nk, kfmt, c->d_rows, c->d_rows_cap, s, &dr, &r2, &g);
      {  // (run_index waited for its kernels: the slot's bytes are no longer read)
        std::lock_guard<std::mutex> lg(mu);
        freed = k + 1;
      }
      cv.notify_all();
      if (rc < 0) { crc = set_msg(&cres, rc, r2.err); return; }
      cres.kernel_ms += r2.kernel_ms;
      cres.index_ms += r2.index_ms;
      const bool last = lo + nk == n;
      const bool ok = rc == 0 && dr.flags == 0 && dr.count >= g.row_base;
      const bool clean = ok && (dr.code == ST_OK || (last && (dr.code == ST_END || dr.code == ST_ABSENT)));
      // ring layout: a Go error inside a slab indexed with its exact incoming state is the
      // file's first (the slabs before it were clean) -- its rows before the error and its text
      // end the build, as the one-pass build ends them (record.go:51-83), without re-reading
      // the rest of the node.  (A blank group, a record past the halo, any flag: the fallback.)
      const bool slab_err = ring && ok && dr.code >= ST_FQ_TRUNC && dr.code <= ST_FA_INVALID &&
                            (dr.code != ST_FQ_TRUNC || last);
      // ring layout: a record the slab could not close through its halo (ST_NEEDMORE) or blank
      // lines running past it (ST_END before the file's end): the rows before it are final too,
      // and the walk restarts at it (build_fd_pipelined)
      const bool partial = ring && rc == 0 && dr.count >= g.row_base && !last &&
                           ((dr.flags == 4 && dr.code == ST_NEEDMORE) || (dr.flags == 0 && dr.code == ST_END));
      if (!clean && !slab_err && !partial) { crc = 1; return; }
      const u64 owned = dr.count - g.row_base;
      // rows D2H through the two pinned row buffers: chunk j + 1's DMA overlaps chunk j's sink
      const double td = now_ms();
      const u64 per = STAGE_BYTES / 16;
      u64 done_rows = 0;
      int b = 0;
      while (done_rows < owned) {
        const u64 m = owned - done_rows < per ? owned - done_rows : per;
        if (hipMemcpyAsync(c->h_rows[b], c->d_rows + 2 * done_rows, m * 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
          crc = set_msg(&cres, SHOCKIDX_EHIP, "rows copy");
          return;
        }
        // the slab's rows continue the table (record.go:51-83): its first row starts where the
        // previous slab's last row ended
        const u64 *hr = (const u64 *)c->h_rows[b];
        if (done_rows == 0 && hr[0] != next_off) { crc = set_msg(&cres, SHOCKIDX_EINTERNAL, SLAB_SEAM_MSG); return; }
        next_off = hr[2 * (m - 1)] + hr[2 * (m - 1) + 1];
        last_len = hr[2 * (m - 1) + 1];
        if (int r = sink.put(c->h_rows[b], total + done_rows, m, &cres)) { crc = r; return; }
        done_rows += m;
        b ^= 1;
      }
      t_d2h += now_ms() - td;
      total += owned;
      state = dr.state_out;
      if (slab_err) {
        err_dr = dr;
        crc = 3;
        return;
      }
      if (partial) { crc = 1; return; }
    }
  });
  // ---- producer --------------------------------------------------------------------------
  int prc = 0;
  // (a) DMA straight out of the page cache: the file mapped read-only and pinned 256 MiB at a time
  // (hipHostRegister of page-cached pages runs at ~160 GB/s, ahead of PCIe), so the bytes cross
  // the host's memory once instead of being copied into pinned staging first
  // (tools/probes/regprobe.cpp: register 6.7 ms + H2D 18.7 ms per GiB).  Chunks stay pinned until
  // the copy stream drains (unpinning behind the DMA cost a quarter of the rate,
  // profiles/r04/e2e_fd_page_cache_dma.txt) -- unless the process-wide pin budget runs out, when
  // the ring unpins the chunks behind its current slab.  (b) When the file does not map or its
  // pages do not pin: the copy threads pread it into the two pinned staging buffers.
  uint8_t *map = nullptr;  // the file from the page below base: node byte a is map[lead + a]
  const u64 a0 = base & ~4095ull, lead = base - a0, mn = lead + n;
  const size_t maplen = (size_t)((mn + 4095) & ~4095ull);
  if (!getenv("SHOCKIDX_NO_MMAP_DMA")) {
    void *mp = mmap(nullptr, maplen, PROT_READ, MAP_SHARED, fd, (off_t)a0);
    if (mp != MAP_FAILED) map = (uint8_t *)mp;
  }
  constexpr u64 CH = 256ull << 20;  // (chunks in map coordinates)
  const u64 nch = (mn + CH - 1) / CH;
  std::vector<u64> pinned(nch, 0);  // bytes registered (and reserved) per chunk
  bool pin_ok = map != nullptr;     // chunks still pin (else the staging path from here on)
  auto chunk_len = [&](u64 j) { return (size_t)((((j * CH + CH < mn ? j * CH + CH : mn) + 4095) & ~4095ull) - j * CH); };
  auto unpin = [&](u64 j) {
    if (!pinned[j]) return;
    (void)hipHostUnregister(map + j * CH);
    pin_release(pinned[j]);
    pinned[j] = 0;
  };
  // pin chunk j (reserving its bytes); false: it does not pin (the caller stages instead)
  auto pin = [&](u64 j, u64 keep_from) -> bool {
    if (pinned[j]) return true;
    if (!pin_ok) return false;
    const u64 len = chunk_len(j);
    if (!pin_reserve(len)) {
      // over the process-wide budget: unpin the chunks wholly before keep_from (their copies
      // must have landed first), then try once more
      bool any = false;
      for (u64 i = 0; i < j && (i + 1) * CH <= keep_from; ++i) any |= pinned[i] != 0;
      if (!any || hipStreamSynchronize(c->s_copy) != hipSuccess) return false;
      for (u64 i = 0; i < j && (i + 1) * CH <= keep_from; ++i) unpin(i);
      if (!pin_reserve(len)) return false;
    }
    if (hipHostRegister(map + j * CH, len, 0) != hipSuccess) {
      (void)hipGetLastError();
      pin_release(len);
      pin_ok = false;
      return false;
    }
    pinned[j] = len;
    return true;
  };
  // node bytes [a, b) to device address dst on the copy stream: pinned chunks, else staging
  int stage_i = 0;
  PreadFill fill = pread_fill(c, fd, res);
  auto copy_range = [&](uint8_t *dst, u64 a, u64 b, u64 keep_from) -> int {
    a += lead;  // (map coordinates from here: file offset a0 + x)
    b += lead;
    keep_from += lead;
    while (a < b) {
      const u64 j = a / CH, ce = (j + 1) * CH < b ? (j + 1) * CH : b;
      if (pin(j, keep_from)) {
        if (hipError_t e = hipMemcpyAsync(dst, map + a, ce - a, hipMemcpyHostToDevice, c->s_copy)) return set_hip(res, e, "page-cache DMA");
        dst += ce - a;
        a = ce;
        continue;
      }
      const size_t k = ce - a < STAGE_BYTES ? (size_t)(ce - a) : STAGE_BYTES;
      hipError_t e = hipEventSynchronize(c->stage_ev[stage_i]);  // buffer free again
      if (e != hipSuccess) return set_hip(res, e, "stage wait");
      if (int rc = fill(c->h_stage[stage_i], a0 + a, k)) return rc;
      if ((e = hipMemcpyAsync(dst, c->h_stage[stage_i], k, hipMemcpyHostToDevice, c->s_copy)) != hipSuccess ||
          (e = hipEventRecord(c->stage_ev[stage_i], c->s_copy)) != hipSuccess)
        return set_hip(res, e, "H2D");
      stage_i ^= 1;
      dst += k;
      a += k;
    }
    return 0;
  };
  auto publish = [&](u64 k) -> int {  // slab k's bytes are all issued: its event, then wake the index thread
    if (hipError_t e = hipEventRecord(ev[k], c->s_copy)) return set_hip(res, e, "event");
    {
      std::lock_guard<std::mutex> g(mu);
      recorded = k + 1;
    }
    cv.notify_all();
    return 0;
  };
  if (ring) {
    for (u64 k = 0; k < K && !prc; ++k) {
      {  // slot k mod 2 is free once the index thread is done with slab k - 2
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return freed + 2 > k || ix_over; });
        if (freed + 2 <= k) break;  // the index thread ended (fallback or error)
      }
      const u64 lo = slab_lo(k), fk = slab_front(k);
      prc = copy_range(slot[k & 1], lo - fk, lo + slab_end(k), lo - fk);
      if (!prc) prc = publish(k);
    }
  } else {
    u64 off = 0, ks = 0;
    while (off < n && !prc) {
      const u64 e = off + CH < n ? off + CH : n;
      prc = copy_range(c->d_in + off, off, e, 0);
      off = e;
      while (!prc && ks < K && slab_lo(ks) + slab_end(ks) <= off) prc = publish(ks++);
    }
  }
  {
    std::lock_guard<std::mutex> g(mu);
    if (prc) prod_failed = true;
  }
  cv.notify_all();
  ix.join();
  {  // before the pages are unpinned and unmapped
    const hipError_t se = hipStreamSynchronize(c->s_copy);
    if (se != hipSuccess && !prc) prc = set_hip(res, se, "H2D sync");
  }
  for (u64 j = 0; j < nch; ++j) unpin(j);
  if (map) munmap(map, maplen);
  if (prc) return prc;
  if (crc < 0) {
    memcpy(res->err, cres.err, sizeof res->err);
    res->err_len = cres.err_len;
    res->status = crc;
    return crc;
  }
  if (crc == 2) {  // the detection's error, as the one-pass build reports it (no rows)
    const int code = cres.status ? cres.status : SHOCKIDX_EFORMAT;
    memcpy(res->err, cres.err, sizeof res->err);
    res->err_len = cres.err_len;
    res->status = code;
    res->count = 0;
    res->total_ms = now_ms() - t0;
    return code;
  }
  if (crc == 3) {  // a Go error in a slab: the rows before it are in the sink
    res->count = total;
    res->format = kfmt == F_LINE ? SHOCKIDX_FMT_LINE : kfmt;
    res->path = 4;
    res->term_code = err_dr.code;
    res->kernel_ms = cres.kernel_ms;
    res->index_ms = cres.index_ms;
    res->d2h_ms = t_d2h;
    res->total_ms = now_ms() - t0;
    res->h2d_ms = res->total_ms - t_d2h - res->kernel_ms;
    if (err_dr.code == ST_FA_INVALID) {
      // fasta.go:115-121: "Invalid fasta entry: " + read[0:min(50, len(read))], the piece read
      // back from the file (it may begin before the slot holding the slab)
      static const char pre[] = "Invalid fasta entry: ";
      const u64 show = err_dr.err_len < 50 ? err_dr.err_len : 50;
      memcpy(res->err, pre, sizeof pre - 1);
      if (show && pread(fd, res->err + sizeof pre - 1, (size_t)show, (off_t)err_dr.err_pos) != (ssize_t)show)
        return set_msg(res, SHOCKIDX_EIO, "error text read");
      res->err_len = sizeof pre - 1 + show;
      res->err[res->err_len] = 0;
      res->status = SHOCKIDX_EFORMAT;
      return SHOCKIDX_EFORMAT;
    }
    const char *m = status_message(err_dr.code);
    if (!m) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: unknown device status");
    const u64 cnt = total;
    set_msg(res, SHOCKIDX_EFORMAT, m);
    res->count = cnt;
    return SHOCKIDX_EFORMAT;
  }
  if (crc == 1 && ring && next_off > base) {
    // the rest from r = next_off as a node of its own, through the same slots (the caller loops)
    *restart = next_off;
    res->count = total;
    res->format = kfmt == F_LINE ? SHOCKIDX_FMT_LINE : kfmt;
    res->path = 4;
    res->kernel_ms = cres.kernel_ms;
    res->index_ms = cres.index_ms;
    res->d2h_ms = t_d2h;
    res->total_ms = now_ms() - t0;
    res->h2d_ms = res->total_ms - t_d2h - res->kernel_ms;
    return 0;
  }
  if (crc == 1 && !ring) {  // the whole file, one pass (it is all in HBM once the copy stream drained)
    *fell_back = true;
    reset_result(res);
    res->h2d_ms = now_ms() - t0;
    return build_resident(c, c->d_in, n, kind, fmt, s, res);
  }
  if (crc == 1) {
    // ring, no progress (a record the walk cannot close from its own start): the rest of the file
    // from the first record not yet emitted, as a node of its own, in one pass
    const u64 r = next_off, end = base + n;
    for (int i = 0; i < 2; ++i) {
      (void)hipFree(c->d_slot[i]);
      c->d_slot[i] = nullptr;
    }
    c->slot_cap = 0;
    if (one_pass_bytes(end - r) > dev_budget(c))
      return set_msg(res, SHOCKIDX_ENOMEM, "device memory: the node's one-pass fallback does not fit the device budget");
    shockidx_result r3;
    reset_result(&r3);
    if (int rc = stage_fd(c, fd, r, end - r, s, &r3)) {
      memcpy(res->err, r3.err, sizeof res->err);
      res->err_len = r3.err_len;
      return res->status = rc;
    }
    const int sfmt = total ? (kfmt == F_LINE ? SHOCKIDX_FMT_AUTO : kfmt) : fmt;
    int rc = build_resident(c, c->d_in, end - r, kind, sfmt, s, &r3);
    if (rc < 0) {
      memcpy(res->err, r3.err, sizeof res->err);
      res->err_len = r3.err_len;
      return res->status = rc;
    }
    // its rows, shifted by r, continue the table
    const double td = now_ms();
    const u64 per = STAGE_BYTES / 16;
    for (u64 d = 0; d < r3.count;) {
      const u64 m = r3.count - d < per ? r3.count - d : per;
      HIPCHK(hipMemcpyAsync(c->h_rows[0], c->d_rows + 2 * d, m * 16, hipMemcpyDeviceToHost, s), "rows copy");
      HIPCHK(hipStreamSynchronize(s), "rows copy");
      u64 *hr = (u64 *)c->h_rows[0];
      for (u64 i = 0; i < m; ++i) hr[2 * i] += r;
      if (d == 0 && hr[0] != next_off) return set_msg(res, SHOCKIDX_EINTERNAL, SLAB_SEAM_MSG);
      if (int e = sink.put(c->h_rows[0], total + d, m, res)) return e;
      d += m;
    }
    res->count = total + r3.count;
    res->format = r3.format;
    res->status = r3.status;
    memcpy(res->err, r3.err, sizeof res->err);
    res->err_len = r3.err_len;
    res->path = 4;
    res->reruns = r3.reruns + 1;
    res->kernel_ms = cres.kernel_ms + r3.kernel_ms;
    res->index_ms = cres.index_ms + r3.index_ms;
    res->d2h_ms = t_d2h + (now_ms() - td);
    res->total_ms = now_ms() - t0;
    res->h2d_ms = res->total_ms - res->d2h_ms - res->kernel_ms;
    return rc;
  }
  // the table ends where the file does (FASTQ: or before trailing blank lines)
  {
    uint8_t a = '\n', z = '\n';
    const u64 end = base + n;
    bool bad = next_off > end;
    if (!bad && next_off < end) {
      if (kfmt != F_FASTQ || pread(fd, &a, 1, (off_t)next_off) != 1 || pread(fd, &z, 1, (off_t)(end - 1)) != 1) bad = true;
      bad |= a != '\n' || z != '\n';
    }
    if (!bad && kfmt == F_LINE && last_len)  // the line index's last row: the bytes after the last '\n'
      bad = pread(fd, &z, 1, (off_t)(end - 1)) != 1 || z == '\n';
    if (bad) return set_msg(res, SHOCKIDX_EINTERNAL, SLAB_END_MSG);
  }
  res->count = total;
  res->format = kfmt == F_LINE ? SHOCKIDX_FMT_LINE : kfmt;
  res->status = SHOCKIDX_OK;
  res->path = ring ? 4 : 3;  // the slab pipeline (4: through the two slots)
  res->kernel_ms = cres.kernel_ms;
  res->index_ms = cres.index_ms;
  res->d2h_ms = t_d2h;
  res->total_ms = now_ms() - t0;
  res->h2d_ms = res->total_ms - t_d2h - res->kernel_ms;
  return SHOCKIDX_OK;
}

// The fd build: build_fd_walk over the file, and again over the rest from each restart point
// (a record longer than the halo ended a walk through the slots), rows numbered on.
int build_fd_pipelined(shockidx_ctx *c, int fd, u64 n, int kind, int fmt, RowSink &sink, shockidx_result *res,
                       bool *done, bool *fell_back) {
  const double t0 = now_ms();
  u64 base = 0, row0 = 0;
  int f = fmt;
  double kms = 0, ims = 0, dms = 0;
  uint32_t reruns = 0;
  for (;;) {
    u64 restart = 0;
    const int rc = build_fd_walk(c, fd, n - base, kind, f, sink, res, done, fell_back, base, row0, &restart);
    if (rc || !restart) {
      if (base) {  // the walks before this one
        *done = true;
        res->kernel_ms += kms;
        res->index_ms += ims;
        res->d2h_ms += dms;
        res->reruns += reruns;
        res->path = 4;
        res->total_ms = now_ms() - t0;
        res->h2d_ms = res->total_ms - res->d2h_ms - res->kernel_ms;
      }
      return rc;
    }
    kms += res->kernel_ms;
    ims += res->index_ms;
    dms += res->d2h_ms;
    ++reruns;
    row0 = res->count;
    f = res->format == SHOCKIDX_FMT_LINE ? SHOCKIDX_FMT_AUTO : res->format;  // the format found at the file's start
    base = restart;
  }
}

}  // namespace

// ---- internal host API (sidx_host.hpp) for the other translation units ----------------------
namespace sidx_host {
double now_ms() { return ::now_ms(); }
int set_msg(shockidx_result *r, int code, const char *msg) { return ::set_msg(r, code, msg); }
int set_hip(shockidx_result *r, hipError_t e, const char *what) { return ::set_hip(r, e, what); }
const char *status_message(uint32_t code) { return ::status_message(code); }
int ctx_device(shockidx_ctx *c) { return c->device; }
hipStream_t ctx_stream(shockidx_ctx *c) { return c->stream; }
int ctx_stage(shockidx_ctx *c, const void *src, int fd, uint64_t off, uint64_t len, const uint8_t **d_out,
              shockidx_result *res) {
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int rc;
  if (src) {
    const uint8_t *base = (const uint8_t *)src + off;
    rc = stage_in(c, len, c->stream, [&](uint8_t *dst, u64 o, size_t k) -> int {
      c->pool->copy(dst, base + o, k);
      return 0;
    }, res);
  } else {
    rc = stage_fd(c, fd, off, len, c->stream, res);
  }
  if (rc) return rc;
  *d_out = c->d_in;
  return 0;
}
int ctx_to_host(shockidx_ctx *c, const void *d_src, uint64_t bytes, void *dst, shockidx_result *res) {
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  return rows_to_host(c, (const u64 *)d_src, bytes, (uint8_t *)dst, c->stream, res);
}
uint64_t *alloc_rows(uint64_t bytes) { return alloc_rows_out(bytes); }
hipError_t dev_malloc(void **p, size_t bytes, bool node) {
  if (node && bytes >= (64u << 20) && !getenv("SHOCKIDX_NO_CONTIG")) {
    if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();  // fragmented: plain memory below
  }
  return hipMalloc(p, bytes);
}
}  // namespace sidx_host

extern "C" {

int shockidx_abi_version(void) { return SHOCKIDX_ABI_VERSION; }

const char *shockidx_strerror(int code) {
  switch (code) {
    case SHOCKIDX_OK: return "ok";
    case SHOCKIDX_EFORMAT: return "format error";
    case SHOCKIDX_EINVAL: return "invalid argument";
    case SHOCKIDX_EHIP: return "HIP runtime error";
    case SHOCKIDX_ENOMEM: return "out of memory";
    case SHOCKIDX_EIO: return "I/O error";
    case SHOCKIDX_EINTERNAL: return "internal error";
    case SHOCKIDX_ESPACE: return "output capacity too small";
    default: return "unknown";
  }
}

void shockidx_free(void *p) { free(p); }

int shockidx_host_register(shockidx_ctx *c, void *p, uint64_t n) {
  shockidx_result tmp, *res = &tmp;
  if (!c || !p || !n) return SHOCKIDX_EINVAL;
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(hipHostRegister(p, n, hipHostRegisterDefault), "hipHostRegister");
  return SHOCKIDX_OK;
}

int shockidx_host_unregister(shockidx_ctx *c, void *p) {
  shockidx_result tmp, *res = &tmp;
  if (!c || !p) return SHOCKIDX_EINVAL;
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(hipHostUnregister(p), "hipHostUnregister");
  return SHOCKIDX_OK;
}

int shockidx_ctx_create(int device, shockidx_ctx **out) {
  shockidx_result tmp;
  shockidx_result *res = &tmp;
  reset_result(res);
  if (!out) return SHOCKIDX_EINVAL;
  *out = nullptr;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return SHOCKIDX_EINVAL;
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  shockidx_ctx *c = new shockidx_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e == hipSuccess) e = hipEventCreate(&c->ek0);
  if (e == hipSuccess) e = hipEventCreate(&c->ek1);
  for (int i = 0; i < NSTAGE && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc((void **)&c->d_small, SMALL_BYTES);
  if (e == hipSuccess) e = hipMemsetAsync(c->d_small, 0, SMALL_BYTES, c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(c->d_small + SMALL_BADKEY, 0xFF, 16, c->stream);  // both first-bad slots
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) {
    // persistent grids: one wave of co-resident workgroups over the CUs
    int cus = 0;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    int pp = sidx_tiles_blocks_per_cu();
    if (const char *w = getenv("SHOCKIDX_TILES_PER_CU")) pp = atoi(w) < pp ? atoi(w) : pp;  // tuning knob
    c->tiles_grid = (u32)(cus * (pp < 1 ? 1 : pp));
    const int vb = sidx_cr_verify_blocks_per_cu();
    c->cr_grid = (u32)(cus * (vb < 1 ? 1 : vb));
  }
  for (int i = 0; i < NSTAGE && e == hipSuccess; ++i) e = hipHostMalloc((void **)&c->h_stage[i], STAGE_BYTES, 0);
  if (e == hipSuccess) e = hipHostMalloc((void **)&c->h_res, sizeof(DevResult), 0);
  if (e == hipSuccess) e = hipHostMalloc((void **)&c->h_det, 64, 0);
  if (e == hipSuccess) {
    const unsigned hw = std::thread::hardware_concurrency();
    // 16 (a GPU's share of the host's cores on an 8-GPU MI355X node): the page-cached fd path
    // (pread into the pinned staging) ran 32.6 GiB/s with 8 threads, 38.2 with 16
    int nt = getenv("SHOCKIDX_COPY_THREADS") ? atoi(getenv("SHOCKIDX_COPY_THREADS")) : (int)(hw / 2 < 16 ? hw / 2 : 16);
    c->pool = new CopyPool(nt < 1 ? 1 : nt);
  }
  if (const char *cap = getenv("SHOCKIDX_WORKSPACE_CAP")) c->ws_cap = strtoull(cap, nullptr, 10);
  if (const char *cap = getenv("SHOCKIDX_DEV_CAP")) c->dev_cap = parse_bytes(cap);
  if (e != hipSuccess) {
    shockidx_ctx_destroy(c);
    return SHOCKIDX_EHIP;
  }
  *out = c;
  return SHOCKIDX_OK;
}

int shockidx_ctx_set_dev_cap(shockidx_ctx *c, uint64_t bytes) {
  if (!c) return SHOCKIDX_EINVAL;
  c->dev_cap = bytes;
  return SHOCKIDX_OK;
}

int shockidx_ctx_trim(shockidx_ctx *c, uint64_t keep_bytes) {
  if (!c) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  trim_workspace(c, keep_bytes);
  return SHOCKIDX_OK;
}

uint64_t shockidx_ctx_workspace_bytes(shockidx_ctx *c) { return c ? workspace_bytes(c) : 0; }

void shockidx_ctx_destroy(shockidx_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_in);
  (void)hipFree(c->d_rows);
  (void)hipFree(c->d_status);
  (void)hipFree(c->d_detail);
  (void)hipFree(c->d_fix);
  (void)hipFree(c->d_small);
  (void)hipFree(c->d_timing);
  for (int i = 0; i < NSTAGE; ++i) {
    if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
    if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
  }
  if (c->h_res) (void)hipHostFree(c->h_res);
  if (c->h_det) (void)hipHostFree(c->h_det);
  (void)hipFree(c->d_sub);
  (void)hipFree(c->d_fqstage);
  (void)hipFree(c->d_fqtiles);
  (void)hipFree(c->d_fqlines);
  (void)hipFree(c->d_cra);
  (void)hipFree(c->d_crb);
  for (int i = 0; i < 2; ++i) (void)hipFree(c->d_slot[i]);
  delete c->pool;
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ek0) (void)hipEventDestroy(c->ek0);
  if (c->ek1) (void)hipEventDestroy(c->ek1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->s_copy) (void)hipStreamDestroy(c->s_copy);
  for (int i = 0; i < 2; ++i)
    if (c->h_rows[i]) (void)hipHostFree(c->h_rows[i]);
  delete c;
}

int shockidx_build_device(shockidx_ctx *c, const void *d_data, uint64_t n, int kind, int fmt,
                          void *d_rows, uint64_t row_cap, void *stream, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  if (!c || (!d_data && n) || ((uintptr_t)d_data & 15)) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const uint8_t *dd = (const uint8_t *)d_data;
  int kfmt = 0;
  const int *gate = nullptr;
  if (int rc = resolve_format(c, dd, n, kind, fmt, s, &kfmt, res, &gate)) return rc;
  res->format = kfmt == F_LINE ? SHOCKIDX_FMT_LINE : kfmt;
  DevResult dr;
  if (int rc = run_index(c, dd, n, kfmt, (u64 *)d_rows, row_cap, s, &dr, res, nullptr, false, gate)) return rc;
  if (gate) {
    if (int rr = respeculate(c, dr, &kfmt, res)) {
      if (rr < 0 || rr == SHOCKIDX_EFORMAT) return rr;
      res->reruns++;
      if (int rc = run_index(c, dd, n, kfmt, (u64 *)d_rows, row_cap, s, &dr, res)) return rc;
    }
  }
  int rc = translate(c, dr, dd, s, res);
  if (rc >= 0 && (dr.flags & 1)) rc = set_msg(res, SHOCKIDX_ESPACE, "row capacity too small");
  res->count = dr.count;
  res->total_ms = now_ms() - t0;
  return rc;
}

// The serial walk from (curr, cnt) for at most `steps` chunks (UINT64_MAX: to the end)
int chunk_serial(shockidx_ctx *c, const uint8_t *dd, u64 n, int fasta, u64 chunk, u64 *rows, u64 row_cap,
                 u64 curr, u64 cnt, u64 steps, hipStream_t s, u64 out[3], shockidx_result *res) {
  u64 *d_out = (u64 *)(c->d_small + SMALL_CHUNK);
  HIPCHK(sidx_launch_chunkrecord(dd, n, fasta, (long long)chunk, rows, row_cap, d_out, (long long)curr, cnt, steps, s),
         "chunkrecord launch");
  HIPCHK(hipMemcpyAsync(c->h_det, d_out, 3 * sizeof(u64), hipMemcpyDeviceToHost, s), "chunkrecord copy");
  HIPCHK(hipStreamSynchronize(s), "chunkrecord sync");
  memcpy(out, c->h_det, 3 * sizeof(u64));
  return 0;
}

// Speculative chunkrecord (sidx_chunk.hip): predicted-successor graph over the node positions,
// its jump table, then rounds of path + exact evaluation of every chunk on the path; a chunk
// whose exact successor differs re-enters the path there (or a few serial steps first when
// that position is not a node).  *count = rows of the serial definition.
int chunk_spec(shockidx_ctx *c, const uint8_t *dd, u64 n, int kfmt, u64 chunk, u64 *rows, u64 row_cap,
               hipStream_t s, u64 *count, u64 *rounds, shockidx_result *res) {
  const int fasta = kfmt == SHOCKIDX_FMT_FASTA;
  constexpr u64 CT = 16384;
  // rows of the path per round: about the chunk count (chunks average between chunk - 32 KiB
  // and chunk bytes); a longer file takes further rounds
  const u64 ntile = n / CT + 1, est = n / chunk + 1, cap = 2 * est + 1024;
  u64 nb = 0, stride = 1;
  const u64 *base = nullptr;
  const u64 *toff_g = nullptr, *tcnt_g = nullptr;  // FASTA: per-tile node counts, their offsets
  const uint16_t *slot_g = nullptr;                 //   and the tiles' kept positions
  auto carve = [](uint8_t *&q, u64 bytes) { uint8_t *r = q; q += (bytes + 255) & ~255ull; return r; };
  if (!fasta) {  // the FASTQ record index (valid up to its first error) gives the node positions
    u64 rcap = n / 128 + 4096;
    for (int attempt = 0; attempt < 2; ++attempt) {
      if (int rc = ensure_dev(c, (void **)&c->d_cra, &c->cra_cap, rcap * 16, 1, res)) return rc;
      DevResult dr;
      shockidx_result r2;
      reset_result(&r2);
      if (int rc = run_index(c, dd, n, F_FASTQ, (u64 *)c->d_cra, rcap, s, &dr, &r2)) return set_msg(res, rc, r2.err);
      nb = dr.count;
      if (dr.flags & 1) { rcap = dr.count + 1; nb = 0; continue; }
      break;
    }
    base = (const u64 *)c->d_cra;
    stride = 2;
    if (nb && (3 * nb >= 0xFFFFFFF0ull)) nb = 0;
  } else {  // FASTA: every '>' preceded by '\n', plus position 0
    const u64 nt = (n + CT - 1) / CT;
    size_t sb = 0;
    HIPCHK(sidx_cr_gpos_count(dd, n, nullptr, nullptr, nullptr, nullptr, &sb, s), "scan size");
    const u64 slot_bytes = 2ull * sidx_cr_gslot() * nt;
    if (int rc = ensure_dev(c, (void **)&c->d_cra, &c->cra_cap, 16 * nt + slot_bytes + sb + 2048, 1, res)) return rc;
    uint8_t *q = c->d_cra;
    u64 *tcnt = (u64 *)carve(q, 8 * nt), *toff = (u64 *)carve(q, 8 * nt);
    uint16_t *slot = (uint16_t *)carve(q, slot_bytes);
    toff_g = toff;
    tcnt_g = tcnt;
    slot_g = slot;
    HIPCHK(sidx_cr_gpos_count(dd, n, tcnt, toff, slot, q, &sb, s), "node count");
    u64 last[2] = {0, 0};
    if (nt) {
      HIPCHK(hipMemcpyAsync(c->h_det, toff + nt - 1, 8, hipMemcpyDeviceToHost, s), "node count copy");
      HIPCHK(hipMemcpyAsync((u64 *)c->h_det + 1, tcnt + nt - 1, 8, hipMemcpyDeviceToHost, s), "node count copy");
      HIPCHK(hipStreamSynchronize(s), "node count sync");
      memcpy(last, c->h_det, 16);
    }
    nb = 1 + last[0] + last[1];
    if (nb >= 0xFFFFFFF0ull) nb = 0;
  }
  const u64 nn = fasta ? nb : 3 * nb;
  if (nb) {
    const u64 need = (fasta ? 8 * nb : 0) + 8 * (ntile + 2) + 12 * nn + 4 * cap + 16 * cap + 64 + 16 * 256;
    if (int rc = ensure_dev(c, (void **)&c->d_crb, &c->crb_cap, need, 1, res)) return rc;
    uint8_t *q = c->d_crb;
    if (fasta) {
      u64 *G = (u64 *)carve(q, 8 * nb);
      HIPCHK(hipMemsetAsync(G, 0, 8, s), "node 0");
      HIPCHK(sidx_cr_gpos_write(dd, n, tcnt_g, toff_g, slot_g, G, s), "node positions");
      base = G;
    }
    u64 *ft = (u64 *)carve(q, 8 * (ntile + 2));
    u32 *J1 = (u32 *)carve(q, 4 * nn), *Ja = (u32 *)carve(q, 4 * nn), *Jb = (u32 *)carve(q, 4 * nn);
    u32 *heads = (u32 *)carve(q, 4 * cap);
    u64 *pos = (u64 *)carve(q, 8 * cap);
    i64 *mres = (i64 *)carve(q, 8 * cap);
    u64 *ctl = (u64 *)carve(q, 64);
    int levels = 0;
    while (levels < 16 && (est >> levels) > 128) ++levels;
    const u32 *JL = J1;
    HIPCHK(sidx_cr_graph(dd, n, fasta, chunk, base, stride, nb, ft, J1, Ja, Jb, levels, &JL, s), "chunk graph");
    u64 y = 0, k0 = 0;
    for (u64 miss = 0; miss < 64;) {
      ++*rounds;
      HIPCHK(sidx_cr_round(dd, n, fasta, chunk, base, stride, nb, ft, JL, J1, 1u << levels, y, k0, cap, heads, pos,
                           mres, ctl, rows, row_cap, c->cr_grid, s),
             "chunk round");
      HIPCHK(hipMemcpyAsync(c->h_det, ctl, 5 * sizeof(u64), hipMemcpyDeviceToHost, s), "chunk round copy");
      HIPCHK(hipStreamSynchronize(s), "chunk round sync");
      u64 r[5];
      memcpy(r, c->h_det, sizeof r);
      if (r[1] == 0xFFFFFFFDull) {  // not a node: a few exact steps, then the path again
        u64 o[3];
        if (int rc = chunk_serial(c, dd, n, fasta, chunk, rows, row_cap, y, k0, 2, s, o, res)) return rc;
        if (o[2]) { *count = o[0]; return 0; }
        y = o[1];
        k0 = o[0];
        ++miss;
        continue;
      }
      if (r[2] == ~0ull) { *count = k0 + r[0]; return 0; }  // the whole path holds
      if ((i64)r[3] < 0) { *count = k0 + r[2] + 1; return 0; }  // that chunk is the last
      if (!(r[1] == 0xFFFFFFFCull && r[2] + 1 == r[0])) ++miss;  // not just the path's capacity
      y = r[4];
      k0 += r[2] + 1;
    }
    u64 o[3];  // still disagreeing: walk the rest
    if (int rc = chunk_serial(c, dd, n, fasta, chunk, rows, row_cap, y, k0, ~0ull, s, o, res)) return rc;
    *count = o[0];
    return 0;
  }
  u64 o[3];  // no nodes (e.g. the FASTQ record index fails at record 0): the serial walk
  if (int rc = chunk_serial(c, dd, n, fasta, chunk, rows, row_cap, 0, 0, ~0ull, s, o, res)) return rc;
  *count = o[0];
  return 0;
}

// chunkrecord (index/chunkrecord.go:41-99).  Default: the speculative build (chunk_spec);
// SHOCKIDX_CHUNK_MODE=serial: the serial walk alone (the definition, kept as a tested path).
int shockidx_chunkrecord_device(shockidx_ctx *c, const void *d_data, uint64_t n, int fmt, uint64_t chunk,
                                void *d_rows, uint64_t row_cap, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  if (!chunk) chunk = 1048576;  // conf.CHUNK_SIZE (conf/conf.go:138)
  if (!c || (!d_data && n) || (!d_rows && row_cap) || chunk < 32768 || chunk > (1ull << 40))
    return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  const uint8_t *dd = (const uint8_t *)d_data;
  int kfmt = 0;
  if (int rc = resolve_format(c, dd, n, SHOCKIDX_RECORD, fmt, s, &kfmt, res)) return rc;
  res->format = kfmt;
  if (kfmt == SHOCKIDX_FMT_SAM)  // sam.SeekChunk returns (0, nil): the Go driver never ends
    return set_msg(res, SHOCKIDX_EFORMAT, "chunkrecord: sam.SeekChunk never advances (reference loops forever)");
  if (kfmt != SHOCKIDX_FMT_FASTA && kfmt != SHOCKIDX_FMT_FASTQ) return set_msg(res, SHOCKIDX_EINVAL, "invalid format");
  const char *mode = getenv("SHOCKIDX_CHUNK_MODE");
  const bool serial = mode && !strcmp(mode, "serial");
  HIPCHK(hipEventRecord(c->ek0, s), "event");
  u64 cnt = 0, rounds = 0;
  if (serial) {
    u64 o[3];
    if (int rc = chunk_serial(c, dd, n, kfmt == SHOCKIDX_FMT_FASTA, chunk, (u64 *)d_rows, row_cap, 0, 0, ~0ull, s, o,
                              res))
      return rc;
    cnt = o[0];
  } else if (int rc = chunk_spec(c, dd, n, kfmt, chunk, (u64 *)d_rows, row_cap, s, &cnt, &rounds, res)) {
    return rc;
  }
  HIPCHK(hipEventRecord(c->ek1, s), "event");
  HIPCHK(hipEventSynchronize(c->ek1), "event sync");
  float kms = 0.f;
  (void)hipEventElapsedTime(&kms, c->ek0, c->ek1);
  res->kernel_ms = res->index_ms = kms;
  res->reruns = rounds;
  res->count = cnt;
  res->total_ms = now_ms() - t0;
  if (cnt > row_cap) return set_msg(res, SHOCKIDX_ESPACE, "row capacity too small");
  return SHOCKIDX_OK;
}

// chunkrecord of a subset node (index/chunkrecord.go:100-228): its record index rows (device,
// R rows) grouped into chunks of rows (sidx_chunk.hip): prefix sums of the lengths, every fresh
// start's successor, the jump table, the path from row 0.  Rows (16 * first row, 16 * rows).
int shockidx_chunkrecord_subset_device(shockidx_ctx *c, const void *d_ri, uint64_t nrows, void *d_rows,
                                       uint64_t row_cap, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  if (!c || (!d_ri && nrows) || (!d_rows && row_cap)) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  if (nrows >= 0xFFFFFFF0ull) return set_msg(res, SHOCKIDX_EINVAL, "record index too large");
  const double t0 = now_ms();
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  const u64 R = nrows;
  size_t sb = 0;
  HIPCHK(sidx_crs_scan(nullptr, R, nullptr, nullptr, nullptr, &sb, s), "scan size");
  auto r256 = [](u64 b) { return (b + 255) & ~255ull; };
  const u64 need = r256(8 * R + 8) + r256(8 * (R + 1)) + 3 * r256(4 * (R + 1)) + r256(4 * (R + 2)) + 256 + r256(sb);
  if (int rc = ensure_dev(c, (void **)&c->d_crb, &c->crb_cap, need, 1, res)) return rc;
  uint8_t *q = c->d_crb;
  auto carve = [&](u64 bytes) { uint8_t *r = q; q += r256(bytes); return r; };
  u64 *len = (u64 *)carve(8 * R + 8), *P = (u64 *)carve(8 * (R + 1));
  u32 *J1 = (u32 *)carve(4 * (R + 1)), *Ja = (u32 *)carve(4 * (R + 1)), *Jb = (u32 *)carve(4 * (R + 1));
  u32 *heads = (u32 *)carve(4 * (R + 2));
  u64 *ctl = (u64 *)carve(256);
  void *scan_tmp = carve(sb);
  HIPCHK(hipEventRecord(c->ek0, s), "event");
  HIPCHK(sidx_crs_scan((const u64 *)d_ri, R, len, P, scan_tmp, &sb, s), "prefix sums");
  HIPCHK(hipMemcpyAsync(c->h_det, P + R, 8, hipMemcpyDeviceToHost, s), "total copy");
  HIPCHK(hipStreamSynchronize(s), "total sync");
  u64 total = 0;
  memcpy(&total, c->h_det, 8);
  // chunks <= 2 * total / 1 MiB + 2 (a chunk and the row that closes it reach 1 MiB together)
  const u64 est = 2 * (total / 1048576) + 2;
  int levels = 0;
  while (levels < 16 && (est >> levels) > 128) ++levels;
  HIPCHK(sidx_crs_build(P, R, J1, Ja, Jb, levels, heads, (u64 *)d_rows, row_cap, ctl, s), "chunk build");
  HIPCHK(hipEventRecord(c->ek1, s), "event");
  HIPCHK(hipMemcpyAsync(c->h_det, ctl, 8, hipMemcpyDeviceToHost, s), "count copy");
  HIPCHK(hipStreamSynchronize(s), "count sync");
  u64 cnt = 0;
  memcpy(&cnt, c->h_det, 8);
  float kms = 0.f;
  (void)hipEventElapsedTime(&kms, c->ek0, c->ek1);
  res->kernel_ms = res->index_ms = kms;
  res->count = cnt;
  res->total_ms = now_ms() - t0;
  if (cnt > row_cap) return set_msg(res, SHOCKIDX_ESPACE, "row capacity too small");
  return SHOCKIDX_OK;
}

// chunkrecord over an open file: every byte to HBM through the pinned pread staging (the
// speculative device walk may inspect any window), the table back to a malloc'ed array
int shockidx_chunkrecord_fd(shockidx_ctx *c, int fd, uint64_t n, int fmt, uint64_t chunk, uint64_t **rows,
                            shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  if (!c || !rows || fd < 0) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  *rows = nullptr;
  if (!chunk) chunk = 1048576;
  TrimGuard trim{c};
  if (chunk < 32768 || chunk > (1ull << 40)) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  if (int rc = stage_fd(c, fd, 0, n, c->stream, res)) return rc;
  const u64 cap = n / (chunk - 32767) + 2;
  if (int rc = ensure_dev(c, (void **)&c->d_rows, &c->d_rows_cap, cap, 16, res)) return rc;
  const double h2d = res->h2d_ms;
  int rc = shockidx_chunkrecord_device(c, c->d_in, n, fmt, chunk, c->d_rows, c->d_rows_cap, res);
  res->h2d_ms = h2d;
  if (rc != SHOCKIDX_OK) return rc;
  if (int rc2 = fetch_rows(c, res->count, c->stream, rows, res)) return rc2;
  res->total_ms = now_ms() - t0;
  return SHOCKIDX_OK;
}

int shockidx_build_host(shockidx_ctx *c, const void *data, uint64_t n, int kind, int fmt,
                        uint64_t **rows, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  if (!c || !rows || (!data && n)) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  *rows = nullptr;
  const double t0 = now_ms();
  TrimGuard trim{c};
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  bool piped = false;
  if (int rc = build_host_pipelined(c, data, n, kind, fmt, rows, res, &piped); piped) return rc;
  if (host_pinned(data, n)) {  // registered / hipHostMalloc'ed: DMA straight from the caller's pages
    const double th = now_ms();
    if (int rc = ensure_dev(c, (void **)&c->d_in, &c->d_in_cap, n + 64, 1, res, true)) return rc;
    for (u64 off = 0; off < n; off += PIN_PIECE) {
      const u64 k = n - off < PIN_PIECE ? n - off : PIN_PIECE;
      HIPCHK(hipMemcpyAsync(c->d_in + off, (const uint8_t *)data + off, k, hipMemcpyHostToDevice, s), "H2D");
    }
    HIPCHK(hipStreamSynchronize(s), "H2D sync");
    res->h2d_ms += now_ms() - th;
  } else {
    auto fill = [&](uint8_t *dst, u64 off, size_t k) -> int {
      c->pool->copy(dst, (const uint8_t *)data + off, k);
      return 0;
    };
    if (int rc = stage_in(c, n, s, fill, res)) return rc;
  }
  int rc = build_resident(c, c->d_in, n, kind, fmt, s, res);
  if (rc < 0) return rc;
  if (int rc2 = fetch_rows(c, res->count, s, rows, res)) return rc2;
  res->total_ms = now_ms() - t0;
  return rc;
}

int shockidx_build_fd(shockidx_ctx *c, int fd, uint64_t n, int kind, int fmt, uint64_t **rows,
                      shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  if (!c || !rows || fd < 0) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  *rows = nullptr;
  const double t0 = now_ms();
  TrimGuard trim{c};
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  {
    TableSink sink(n);
    bool piped = false, fell = false;
    int rc = build_fd_pipelined(c, fd, n, kind, fmt, sink, res, &piped, &fell);
    if (piped) {
      if (rc < 0) return rc;
      if (!fell) {  // the table as it arrived (trimmed to the rows)
        uint8_t *t = sink.out;
        sink.out = nullptr;
        if (!t) t = (uint8_t *)malloc(16);
        *rows = (uint64_t *)t;
        if (!*rows) return set_msg(res, SHOCKIDX_ENOMEM, "out of host memory");
        res->total_ms = now_ms() - t0;
        return rc;
      }
      if (int rc2 = fetch_rows(c, res->count, s, rows, res)) return rc2;
      res->total_ms = now_ms() - t0;
      return rc;
    }
  }
  if (int rc = stage_fd(c, fd, 0, n, s, res)) return rc;
  int rc = build_resident(c, c->d_in, n, kind, fmt, s, res);
  if (rc < 0) return rc;
  if (int rc2 = fetch_rows(c, res->count, s, rows, res)) return rc2;
  res->total_ms = now_ms() - t0;
  return rc;
}

int shockidx_write_idx(const uint64_t *rows, uint64_t count, const char *tmpdir, const char *outpath,
                       char *err, size_t errlen) {
  auto fail = [&](const char *what) {
    if (err && errlen) snprintf(err, errlen, "%s: %s", what, strerror(errno));
    return SHOCKIDX_EIO;
  };
  if (!tmpdir || !outpath || (!rows && count)) return SHOCKIDX_EINVAL;
  std::string tmp = temp_idx_path(tmpdir);
  int fd = open(tmp.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0666);
  if (fd < 0) return fail("create");
  const uint8_t *p = (const uint8_t *)rows;
  size_t left = (size_t)count * 16;
  while (left) {  // rows are {u64 off, u64 len} little-endian in memory (record.go:74-75)
    ssize_t w = write(fd, p, left > (1u << 30) ? (1u << 30) : left);
    if (w < 0) {
      if (errno == EINTR) continue;
      int e = errno;
      close(fd);
      unlink(tmp.c_str());
      errno = e;
      return fail("write");
    }
    p += w;
    left -= (size_t)w;
  }
  if (close(fd) != 0) { unlink(tmp.c_str()); return fail("close"); }
  if (rename(tmp.c_str(), outpath) != 0) {  // record.go:87
    int e = errno;
    unlink(tmp.c_str());
    errno = e;
    return fail("rename");
  }
  return SHOCKIDX_OK;
}

int shockidx_create(shockidx_ctx *c, int fd, uint64_t n, int kind, const char *tmpdir, const char *outpath,
                    shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  if (c && fd >= 0 && tmpdir && outpath && n >= 2 * PIPE_SLAB) {
    // the slab pipeline writes each slab's rows into the temp file while later slabs are read
    reset_result(res);
    const double t0 = now_ms();
    TrimGuard trim{c};
    HIPCHK(hipSetDevice(c->device), "hipSetDevice");
    FileSink sink;
    const std::string tpath = temp_idx_path(tmpdir);
    sink.fd = open(tpath.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0666);
    if (sink.fd < 0) {
      snprintf(res->err, sizeof res->err, "create: %s", strerror(errno));
      res->err_len = strlen(res->err);
      res->status = SHOCKIDX_EIO;
      return SHOCKIDX_EIO;
    }
    bool piped = false, fell = false;
    int rc = build_fd_pipelined(c, fd, n, kind, SHOCKIDX_FMT_AUTO, sink, res, &piped, &fell);
    if (piped && !fell && rc == SHOCKIDX_OK) {
      const int ce = close(sink.fd);
      if (ce != 0 || rename(tpath.c_str(), outpath) != 0) {  // record.go:87
        const int e = errno;
        unlink(tpath.c_str());
        snprintf(res->err, sizeof res->err, "%s: %s", ce != 0 ? "close" : "rename", strerror(e));
        res->err_len = strlen(res->err);
        res->status = SHOCKIDX_EIO;
        return SHOCKIDX_EIO;
      }
      res->total_ms = now_ms() - t0;
      return SHOCKIDX_OK;
    }
    close(sink.fd);
    unlink(tpath.c_str());
    if (piped) {  // fell back (or failed): the one-pass result, written like the plain path
      if (rc != SHOCKIDX_OK) return rc;
      uint64_t *rows = nullptr;
      if (int rc2 = fetch_rows(c, res->count, c->stream, &rows, res)) return rc2;
      int w = shockidx_write_idx(rows, res->count, tmpdir, outpath, res->err, sizeof res->err);
      free(rows);
      if (w != SHOCKIDX_OK) {
        res->err_len = strlen(res->err);
        res->status = w;
        return w;
      }
      res->total_ms = now_ms() - t0;
      return SHOCKIDX_OK;
    }
  }
  uint64_t *rows = nullptr;
  int rc = shockidx_build_fd(c, fd, n, kind, SHOCKIDX_FMT_AUTO, &rows, res);
  if (rc != SHOCKIDX_OK) {
    free(rows);
    return rc;
  }
  const double t0 = now_ms();
  int w = shockidx_write_idx(rows, res->count, tmpdir, outpath, res->err, sizeof res->err);
  free(rows);
  if (w != SHOCKIDX_OK) {
    res->err_len = strlen(res->err);
    res->status = w;
    return w;
  }
  res->total_ms += now_ms() - t0;
  return SHOCKIDX_OK;
}

int shockidx_dev_alloc(shockidx_ctx *c, uint64_t bytes, void **d_ptr) {
  if (!c || !d_ptr) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  return sidx_host::dev_malloc(d_ptr, bytes ? bytes : 16, false) == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_ENOMEM;
}

int shockidx_dev_alloc_node(shockidx_ctx *c, uint64_t bytes, void **d_ptr) {
  if (!c || !d_ptr) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  return sidx_host::dev_malloc(d_ptr, bytes ? bytes : 16, true) == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_ENOMEM;
}

int shockidx_dev_free(shockidx_ctx *c, void *d_ptr) {
  if (!c) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  return hipFree(d_ptr) == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_EHIP;
}

// Both copies run on the context's stream and are waited for: the context streams are
// non-blocking, so a null-stream hipMemcpy is not ordered with their kernels, and a pageable
// host-to-device hipMemcpy may return before its DMA has landed -- a build launched right after
// on another context's stream could read the old bytes.
int shockidx_memcpy_h2d(shockidx_ctx *c, void *d_dst, const void *src, uint64_t bytes) {
  if (!c) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  if (hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return SHOCKIDX_EHIP;
  return hipStreamSynchronize(c->stream) == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_EHIP;
}

int shockidx_memcpy_d2h(shockidx_ctx *c, void *dst, const void *d_src, uint64_t bytes) {
  if (!c) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  if (hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return SHOCKIDX_EHIP;
  return hipStreamSynchronize(c->stream) == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_EHIP;
}

int shockidx_memset(shockidx_ctx *c, void *d_dst, int value, uint64_t bytes) {
  if (!c) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  if (hipMemsetAsync(d_dst, value, bytes, c->stream) != hipSuccess) return SHOCKIDX_EHIP;
  return hipStreamSynchronize(c->stream) == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_EHIP;
}

int shockidx_sync(shockidx_ctx *c) {
  if (!c) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  return hipDeviceSynchronize() == hipSuccess ? SHOCKIDX_OK : SHOCKIDX_EHIP;
}

void *shockidx_stream(shockidx_ctx *c) { return c ? (void *)c->stream : nullptr; }

// Diagnostic (not in the public header): copy the per-workgroup phase cycle sums of the
// last build made with SHOCKIDX_TIMING set into out[9 * nwg].
int shockidx_debug_timing(shockidx_ctx *c, uint64_t *out, uint32_t nwg) {
  if (!c || !c->d_timing || !out || nwg > 65536) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  if (hipDeviceSynchronize() != hipSuccess) return SHOCKIDX_EHIP;
  return hipMemcpy(out, c->d_timing, 9 * 8 * (size_t)nwg, hipMemcpyDeviceToHost) == hipSuccess ? SHOCKIDX_OK
                                                                                              : SHOCKIDX_EHIP;
}

int shockidx_debug_tiles_grid(shockidx_ctx *c) { return c ? (int)c->tiles_grid : 0; }

// Diagnostic (not in the public header): test hooks of the context (shockidx_ctx::inject);
// returns the previous flags.  The next build that grows the status arrays takes bits 0-1.
int shockidx_debug_inject(shockidx_ctx *c, uint32_t flags) {
  if (!c) return SHOCKIDX_EINVAL;
  const int old = (int)c->inject;
  c->inject = flags;
  return old;
}

int shockidx_slab_guess(shockidx_ctx *c, const shockidx_slab *sl, int fmt, uint64_t *guess) {
  shockidx_result tmp;
  shockidx_result *res = &tmp;
  reset_result(res);
  if (!c || !sl || !guess) return SHOCKIDX_EINVAL;
  if (sl->is_first) { *guess = 0; return SHOCKIDX_OK; }
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  u64 *d_out = (u64 *)(c->d_small + SMALL_DETECT + 32);
  HIPCHK(sidx_launch_slab_guess((const uint8_t *)sl->d_data, sl->n, sl->front, fmt, d_out, s), "guess launch");
  HIPCHK(hipMemcpyAsync(c->h_det + 2, d_out, 8, hipMemcpyDeviceToHost, s), "guess copy");
  HIPCHK(hipStreamSynchronize(s), "guess sync");
  memcpy(guess, c->h_det + 2, 8);
  return SHOCKIDX_OK;
}

int shockidx_slab_index(shockidx_ctx *c, const shockidx_slab *sl, int fmt, uint64_t state_in, void *d_rows,
                        uint64_t row_cap, void *d_summary, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  reset_result(res);
  // an empty slab owns no bytes: its pointer may sit at an unaligned file end (tiny files
  // cut into more slabs than 16-byte chunks); nothing is loaded through it
  const bool empty = sl && sl->n == 0 && !sl->is_first;
  if (!c || !sl || !d_summary || (!empty && ((uintptr_t)sl->d_data & 15)) || sl->end < sl->n ||
      (!sl->is_first && sl->n > 0 && sl->front < 16))
    return set_msg(res, SHOCKIDX_EINVAL, "invalid slab");
  if (fmt < SHOCKIDX_FMT_FASTA || fmt > SHOCKIDX_FMT_LINE) return set_msg(res, SHOCKIDX_EINVAL, "invalid format");
  const double t0 = now_ms();
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  SlabGeom g;
  g.n = sl->n;
  g.end = empty ? 0 : sl->end;
  g.front = (sl->is_first || empty) ? 0 : sl->front;
  g.base = sl->base;
  g.state_in = state_in;
  g.row_base = sl->is_first ? 0 : 1;  // record 0 belongs to the first slab
  g.eof = sl->is_last;
  g.file_start = sl->is_first;
  g.d_summary = d_summary;
  g.seq = sl->seq;
  res->format = fmt;
  DevResult dr;
  if (int rc = run_index(c, (const uint8_t *)sl->d_data, sl->n, fmt, (u64 *)d_rows, row_cap, c->stream, &dr, res, &g))
    return rc;
  res->count = dr.count;
  res->state_out = dr.state_out;
  res->term_code = dr.code;
  res->flags = dr.flags;
  res->fixups = dr.fixups;
  res->total_ms = now_ms() - t0;
  if (dr.flags & 2) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: device invariant violated");
  return SHOCKIDX_OK;
}

int shockidx_slab_combine(shockidx_ctx *c, const void *d_all, int world, int rank, int fmt,
                          const uint32_t *expect_seq, shockidx_slab_plan *plan) {
  shockidx_result tmp;
  shockidx_result *res = &tmp;
  reset_result(res);
  if (!c || !d_all || !plan || world < 1 || world > 32 || rank < 0 || rank >= world) return SHOCKIDX_EINVAL;
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  void *d_plan = c->d_small + SMALL_RESULT + sizeof(DevResult);
  static_assert(SMALL_RESULT + sizeof(DevResult) + sizeof(SlabPlan) <= SMALL_DETECT, "small layout");
  HIPCHK(sidx_launch_slab_combine(d_all, world, rank, fmt, expect_seq, d_plan, s), "combine launch");
  HIPCHK(hipMemcpyAsync(c->h_res, d_plan, sizeof(SlabPlan), hipMemcpyDeviceToHost, s), "plan copy");
  HIPCHK(hipStreamSynchronize(s), "combine sync");
  static_assert(sizeof(SlabPlan) == sizeof(shockidx_slab_plan), "plan layout");
  memcpy(plan, c->h_res, sizeof(SlabPlan));
  return SHOCKIDX_OK;
}

}  // extern "C"

// ---- Subset nodes ------------------------------------------------------------------------
namespace {

// strconv.Quote (strconv/quote.go appendQuotedWith / appendEscapedRune) for the Atoi error
// text; unicode.IsPrint exact for ASCII and Latin-1, approximated above.
u32 go_decode_rune(const uint8_t *s, size_t n, size_t *w) {
  const u32 c0 = s[0];
  if (c0 < 0x80) { *w = 1; return c0; }
  u32 sz = 0, lo = 0x80, hi = 0xBF;
  if (c0 >= 0xC2 && c0 <= 0xDF) sz = 2;
  else if (c0 == 0xE0) { sz = 3; lo = 0xA0; }
  else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) sz = 3;
  else if (c0 == 0xED) { sz = 3; hi = 0x9F; }
  else if (c0 == 0xF0) { sz = 4; lo = 0x90; }
  else if (c0 >= 0xF1 && c0 <= 0xF3) sz = 4;
  else if (c0 == 0xF4) { sz = 4; hi = 0x8F; }
  if (!sz || n < sz || s[1] < lo || s[1] > hi) { *w = 1; return 0xFFFD; }
  for (u32 i = 2; i < sz; ++i)
    if (s[i] < 0x80 || s[i] > 0xBF) { *w = 1; return 0xFFFD; }
  *w = sz;
  if (sz == 2) return ((c0 & 0x1F) << 6) | (s[1] & 0x3F);
  if (sz == 3) return ((c0 & 0x0F) << 12) | ((u32)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
  return ((c0 & 0x07) << 18) | ((u32)(s[1] & 0x3F) << 12) | ((u32)(s[2] & 0x3F) << 6) | (s[3] & 0x3F);
}
bool go_is_print(u32 r) {
  if (r < 0x80) return r >= 0x20 && r < 0x7F;
  if (r <= 0xA0 || r == 0xAD) return false;
  if (r < 0x100) return true;
  return !(r == 0x1680 || (r >= 0x2000 && r <= 0x200F) || (r >= 0x2028 && r <= 0x202F) ||
           (r >= 0x205F && r <= 0x206F) || r == 0x3000 || r == 0xFEFF || (r >= 0xFFF9 && r <= 0xFFFB) ||
           (r >= 0xD800 && r <= 0xDFFF) || r > 0x10FFFF);
}
std::string go_quote(const uint8_t *s, size_t n) {
  static const char hx[] = "0123456789abcdef";
  std::string q = "\"";
  for (size_t i = 0; i < n;) {
    size_t w;
    const u32 r = go_decode_rune(s + i, n - i, &w);
    if (w == 1 && r == 0xFFFD) {
      q += "\\x"; q += hx[s[i] >> 4]; q += hx[s[i] & 15];
    } else if (r == '"' || r == '\\') {
      q += '\\'; q += (char)r;
    } else if (go_is_print(r)) {
      q.append((const char *)s + i, w);
    } else if (r == '\a') q += "\\a";
    else if (r == '\b') q += "\\b";
    else if (r == '\f') q += "\\f";
    else if (r == '\n') q += "\\n";
    else if (r == '\r') q += "\\r";
    else if (r == '\t') q += "\\t";
    else if (r == '\v') q += "\\v";
    else if (r < ' ' || r == 0x7F) { q += "\\x"; q += hx[r >> 4]; q += hx[r & 15]; }
    else if (r < 0x10000) { q += "\\u"; for (int sh = 12; sh >= 0; sh -= 4) q += hx[(r >> sh) & 15]; }
    else { q += "\\U"; for (int sh = 28; sh >= 0; sh -= 4) q += hx[(r >> sh) & 15]; }
    i += w;
  }
  q += '"';
  return q;
}

void sub_reset(shockidx_subset_result *r) { memset(r, 0, sizeof *r); }
int sub_msg(shockidx_subset_result *r, int code, const std::string &m) {
  const size_t k = m.size() < sizeof r->err - 1 ? m.size() : sizeof r->err - 1;
  memcpy(r->err, m.data(), k);
  r->err[k] = 0;
  r->err_len = k;
  r->status = code;
  return code;
}
int sub_hip(shockidx_subset_result *r, hipError_t e, const char *what) {
  return sub_msg(r, SHOCKIDX_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define SUBCHK(expr, what)                                 \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return sub_hip(res, _e, what);   \
  } while (0)

// carve 256-byte-aligned pieces out of the context's subset workspace
struct Carver {
  uint8_t *base;
  u64 off = 0;
  template <class T> T *take(u64 n) {
    T *p = (T *)(base + off);
    off += (n * sizeof(T) + 255) / 256 * 256;
    return p;
  }
};

template <class T>
int d2h(shockidx_ctx *c, T *dst, const void *src, shockidx_subset_result *res) {
  SUBCHK(hipMemcpyAsync(dst, src, sizeof(T), hipMemcpyDeviceToHost, c->stream), "subset copy");
  SUBCHK(hipStreamSynchronize(c->stream), "subset sync");
  return 0;
}

// anonymize over a FASTA or SAM section (anonymize.go:28-56 through multi.Reader): the stream
// Read + Format deliver (sidx_filter.hip), count / size delivered, Read's error text.
int anonymize_other(shockidx_ctx *c, const uint8_t *dd, u64 n, int kfmt, uint8_t *d_out, u64 out_cap,
                    shockidx_subset_result *res, double t0) {
  hipStream_t s = c->stream;
  const bool fasta = kfmt == SHOCKIDX_FMT_FASTA;
  u64 K = 0;            // FASTA: boundaries (sequences before the EOF one); SAM: lines
  const u64 *B = nullptr;  // FASTA boundary positions / SAM line rows
  shockidx_result br;
  reset_result(&br);
  size_t tb = 0;
  u64 bstride = 1;  // B[k * bstride]
  bool indexed = false;
  if (fasta && n && !getenv("SHOCKIDX_ANON_SCAN")) {
    // Read's boundaries are the record index's (a '>' with a '\n' since the previous '>',
    // fasta.go:100-138); when the index builds without error they are its row starts 1..R-1,
    // found by the FASTA tile pass in one read.  Otherwise (the index validates pieces Read does
    // not) they come from the unvalidated scan below.
    const int brc = build_resident(c, dd, n, SHOCKIDX_RECORD, SHOCKIDX_FMT_FASTA, s, &br);
    if (brc < 0) return sub_msg(res, brc, std::string(br.err, br.err_len));
    if (brc == SHOCKIDX_OK) {
      indexed = true;
      res->kernel_ms += br.kernel_ms;
      K = br.count ? br.count - 1 : 0;
      B = c->d_rows + 2;
      bstride = 2;
      SUBCHK(sidx_scan_u64(nullptr, nullptr, K ? K : 1, nullptr, &tb, s), "scan size");
      shockidx_result wr;
      memset(&wr, 0, sizeof wr);
      if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, 8 * (K + 1) + 48 * (K + 1) + tb + 4096, 1, &wr))
        return sub_msg(res, rc, wr.err);
      SUBCHK(hipEventRecord(c->ek0, s), "event");
    }
  }
  if (fasta && !indexed) {
    const u64 nt = (n + TILE - 1) / TILE;
    size_t fb = 0;
    SUBCHK(sidx_fa_bnd_count(dd, n, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &fb, s),
           "scan size");
    const u64 slot_bytes = 2ull * sidx_fa_slot() * (nt + 1);
    const u64 need = 6 * 8 * (nt + 1) + slot_bytes + fb + 8 * 256;
    {
      shockidx_result wr;
      memset(&wr, 0, sizeof wr);
      if (int rc = ensure_dev(c, (void **)&c->d_cra, &c->cra_cap, need, 1, &wr)) return sub_msg(res, rc, wr.err);
    }
    Carver cv{c->d_cra};
    u64 *lnl = cv.take<u64>(nt + 1), *lgt = cv.take<u64>(nt + 1), *cnl = cv.take<u64>(nt + 1);
    u64 *cgt = cv.take<u64>(nt + 1), *tcnt = cv.take<u64>(nt + 1), *toff = cv.take<u64>(nt + 1);
    uint16_t *slot = cv.take<uint16_t>(sidx_fa_slot() * (nt + 1));
    void *tmp = cv.take<uint8_t>(fb);
    SUBCHK(hipEventRecord(c->ek0, s), "event");
    SUBCHK(sidx_fa_bnd_count(dd, n, lnl, lgt, cnl, cgt, tcnt, toff, slot, tmp, &fb, s), "boundaries");
    if (nt) {
      u64 a = 0, b = 0;
      if (int rc = d2h(c, &a, toff + nt - 1, res)) return rc;
      if (int rc = d2h(c, &b, tcnt + nt - 1, res)) return rc;
      K = a + b;
    }
    SUBCHK(sidx_scan_u64(nullptr, nullptr, K ? K : 1, nullptr, &tb, s), "scan size");
    {
      shockidx_result wr;
      memset(&wr, 0, sizeof wr);
      const u64 need2 = 8 * (K + 1) + 48 * (K + 1) + tb + 4096;
      if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, need2, 1, &wr)) return sub_msg(res, rc, wr.err);
    }
    u64 *Bw = (u64 *)c->d_sub;
    SUBCHK(sidx_fa_bnd_write(dd, n, cnl, cgt, tcnt, toff, slot, Bw, s), "boundary positions");
    B = Bw;
  } else if (!fasta) {
    const int brc = build_resident(c, dd, n, SHOCKIDX_LINE, SHOCKIDX_FMT_AUTO, s, &br);  // ReadBytes('\n')
    if (brc != SHOCKIDX_OK) return sub_msg(res, brc < 0 ? brc : SHOCKIDX_EINTERNAL, std::string(br.err, br.err_len));
    res->kernel_ms += br.kernel_ms;
    K = br.count;
    B = c->d_rows;
    SUBCHK(sidx_scan_u64(nullptr, nullptr, K ? K : 1, nullptr, &tb, s), "scan size");
    shockidx_result wr;
    memset(&wr, 0, sizeof wr);
    if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, 48 * (K + 1) + tb + 4096, 1, &wr))
      return sub_msg(res, rc, wr.err);
    SUBCHK(hipEventRecord(c->ek0, s), "event");
  }
  Carver cv{c->d_sub};
  if (fasta) (void)cv.take<u64>(K + 1);  // the boundary positions
  u64 *small = cv.take<u64>(4);
  u64 *span = cv.take<u64>(2 * (K + 1));
  u64 *outlen = cv.take<u64>(K + 1);
  u64 *outoff = cv.take<u64>(K + 1);
  void *scan_tmp = cv.take<uint8_t>(tb);
  SUBCHK(hipMemsetAsync(small, 0xFF, 16, s), "memset");
  SUBCHK(hipMemsetAsync(small + 2, 0, 8, s), "memset");
  if (fasta) SUBCHK(sidx_fa_anon_spans(dd, n, B, bstride, K, span, outlen, small, s), "anonymize spans");
  else SUBCHK(sidx_sam_anon_spans(dd, n, B, K, span, outlen, small, small + 1, s), "anonymize spans");
  u64 st[2] = {~0ull, ~0ull};
  SUBCHK(hipMemcpyAsync(st, small, 16, hipMemcpyDeviceToHost, s), "status copy");
  SUBCHK(hipStreamSynchronize(s), "status sync");
  const u64 bad = st[0], eof = fasta ? ~0ull : st[1];
  const u64 Ke = bad < K && bad < eof ? bad : (eof < K ? eof : K);  // the items Read delivers
  const bool err = bad < K && bad < eof;
  u64 total = 0;
  if (Ke) {
    SUBCHK(sidx_scan_u64(outlen, outoff, Ke, scan_tmp, &tb, s), "scan");
    u64 lo = 0, ll = 0;
    if (int rc = d2h(c, &lo, outoff + Ke - 1, res)) return rc;
    if (int rc = d2h(c, &ll, outlen + Ke - 1, res)) return rc;
    total = lo + ll;
  }
  res->size = total;
  res->count = fasta ? Ke : 0;
  if (total > out_cap) return sub_msg(res, SHOCKIDX_ESPACE, "output capacity too small");
  if (fasta) SUBCHK(sidx_fa_anon_write(dd, n, span, outoff, Ke, d_out, s), "anonymize write");
  else SUBCHK(sidx_sam_anon_write(dd, span, outlen, outoff, Ke, d_out, small + 2, s), "anonymize write");
  SUBCHK(hipEventRecord(c->ek1, s), "event");
  if (!fasta) {
    u64 cnt = 0;
    if (int rc = d2h(c, &cnt, small + 2, res)) return rc;
    res->count = cnt;
  }
  SUBCHK(hipStreamSynchronize(s), "anonymize sync");
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ek0, c->ek1);
  res->kernel_ms += ms;
  res->total_ms = now_ms() - t0;
  if (!err) return SHOCKIDX_OK;
  return sub_msg(res, SHOCKIDX_EFORMAT, fasta ? "Invalid fasta entry" : "sam alignment fields less than 11");
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// CreateSubsetNodeIndexes (subset.go:133-303) on the device, and optionally the subset node's
// bytes (single.go:500-517): the id lines (the line index kernel), then every count -- the
// non-blank ids, the first failing one, the accepted ids, the runs, oSize, the gathered bytes --
// stays on the device (SubCtl words) and the kernels read it there, so the host waits twice:
// for the id line count and once at the end.  d_data == nullptr: no gather.
int subset_build(shockidx_ctx *c, const void *d_ids, uint64_t ids_len, const void *d_parent, uint64_t parent_count,
                 int64_t ilength, void *d_rows, uint64_t rows_cap, void *d_runs, uint64_t runs_cap, const void *d_data,
                 uint64_t data_len, void *d_out, uint64_t out_cap, shockidx_subset_result *res) {
  sub_reset(res);
  if (!c || (!d_ids && ids_len) || ((uintptr_t)d_ids & 15) || (!d_parent && parent_count) ||
      (d_data && (((uintptr_t)d_data & 15) || ((uintptr_t)d_out & 15) || !d_runs)))
    return sub_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  SUBCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  // 1. lines of the id text (subset.go:189-199, ReadLine = ReadBytes('\n')): the position of
  // every '\n' (sidx_id_lines) into the context's row workspace, then their count to the host;
  // the bytes after the last '\n' are dropped like ReadLine's EOF line
  const u64 nb = (ids_len + 1023) / 1024;
  size_t ltmp = 0;
  SUBCHK(sidx_id_lines(nullptr, ids_len, nullptr, nullptr, nullptr, nullptr, &ltmp, s), "scan size");
  const u64 ends_bytes = (8 * (ids_len + 2) + 255) / 256 * 256;
  const u64 lbytes = ends_bytes + (4 * nb + 255) / 256 * 256 + (8 * nb + 255) / 256 * 256 + (ltmp + 255) / 256 * 256 + 256;
  {
    shockidx_result lr;
    memset(&lr, 0, sizeof lr);
    if (int rc = ensure_dev(c, (void **)&c->d_rows, &c->d_rows_cap, (lbytes + 15) / 16, 16, &lr))
      return sub_msg(res, rc, lr.err);
  }
  u64 *ends = c->d_rows;
  u64 m = 0;
  {
    Carver lc{(uint8_t *)c->d_rows + ends_bytes};
    u32 *cnt = lc.take<u32>(nb);
    u64 *base = lc.take<u64>(nb);
    void *tmp = lc.take<uint8_t>(ltmp);
    SUBCHK(hipEventRecord(c->ek0, s), "event");
    SUBCHK(sidx_id_lines((const uint8_t *)d_ids, ids_len, cnt, base, ends, tmp, &ltmp, s), "id lines");
    SUBCHK(hipEventRecord(c->ek1, s), "event");
    u64 b_last = 0;
    u32 c_last = 0;
    if (nb) {
      SUBCHK(hipMemcpyAsync(&b_last, base + nb - 1, 8, hipMemcpyDeviceToHost, s), "line count copy");
      SUBCHK(hipMemcpyAsync(&c_last, cnt + nb - 1, 4, hipMemcpyDeviceToHost, s), "line count copy");
    }
    SUBCHK(hipStreamSynchronize(s), "line count sync");
    m = b_last + c_last;
    float lms = 0.f;
    (void)hipEventElapsedTime(&lms, c->ek0, c->ek1);
    res->kernel_ms += lms;
  }
  // 2. workspace (every count is bounded by m; the gather's runs by min(m, runs_cap))
  const bool gather = d_data != nullptr;
  const u64 gb = gather ? (m < runs_cap ? m : runs_cap) : 0;
  size_t scan_bytes = 0, gscan = 0;
  SUBCHK(sidx_scan_flags(nullptr, nullptr, m ? m : 1, nullptr, &scan_bytes, s), "scan size");
  if (gather)
    SUBCHK(sidx_gather(nullptr, 0, nullptr, gb, nullptr, nullptr, nullptr, nullptr, &gscan, nullptr, nullptr, 0, nullptr,
                       nullptr, s),
           "scan size");
  const u64 gblocks = gather ? (out_cap < data_len ? out_cap : data_len) / sidx::GATHER_BLOCK + 2 : 0;
  const u64 need = 8 * SC_ALLWORDS + 64 * (m + 8) + scan_bytes + 16 * (gb + 8) + gscan + 8 * gblocks + 4096;
  {
    shockidx_result wr;
    memset(&wr, 0, sizeof wr);
    if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, need, 1, &wr)) return sub_msg(res, rc, wr.err);
  }
  Carver cv{c->d_sub};
  u64 *ctl = cv.take<u64>(SC_ALLWORDS);
  u32 *keep = cv.take<u32>(m + 1);
  i64 *val = cv.take<i64>(m + 1);
  u32 *st = cv.take<u32>(m + 1);
  u64 *rank = cv.take<u64>(m + 1);
  i64 *cval = cv.take<i64>(m + 1);
  u32 *cst = cv.take<u32>(m + 1);
  u64 *cline = cv.take<u64>(m + 1);
  void *scan_tmp = cv.take<uint8_t>(scan_bytes);
  u64 *lens = cv.take<u64>(gb + 1), *outoff = cv.take<u64>(gb + 1);
  void *gtmp = cv.take<uint8_t>(gscan);
  u64 *wfirst = cv.take<u64>(gblocks);
  u32 *startf = keep;  // reused after compaction
  u64 *runid = rank;
  SUBCHK(hipEventRecord(c->ek0, s), "event");
  SUBCHK(sidx_subset_init(ctl, 0, s), "init");
  if (m) {
    SUBCHK(sidx_subset_parse((const uint8_t *)d_ids, ends, m, keep, val, st, s), "parse");
    SUBCHK(sidx_scan_flags(keep, rank, m, scan_tmp, &scan_bytes, s), "scan");
    SUBCHK(sidx_subset_compact(keep, rank, val, st, m, cval, cst, cline, ctl, s), "compact");
  }
  // 3. per-id checks, row gather, run starts, Ke; 4. runs and oSize
  SUBCHK(sidx_subset_check(cval, cst, m, ctl, (const u64 *)d_parent, parent_count, ilength, (u64 *)d_rows, rows_cap,
                           startf, s),
         "check");
  if (m) SUBCHK(sidx_scan_flags(startf, runid, m, scan_tmp, &scan_bytes, s), "scan");
  SUBCHK(sidx_subset_runs((const u64 *)d_rows, startf, runid, m, ctl, (u64 *)d_runs, rows_cap, runs_cap, s), "runs");
  SUBCHK(hipEventRecord(c->ek1, s), "event");
  // 5. the node's bytes, when asked for (skipped on the device after an error or a short capacity)
  if (gather)
    SUBCHK(sidx_gather((const uint8_t *)d_data, data_len, (const u64 *)d_runs, gb, ctl, lens, outoff, gtmp, &gscan,
                       wfirst, (uint8_t *)d_out, out_cap, c->ev0, c->ev1, s),
           "gather");
  u64 w[SC_ALLWORDS];
  SUBCHK(hipMemcpyAsync(w, ctl, sizeof w, hipMemcpyDeviceToHost, s), "control copy");
  SUBCHK(hipStreamSynchronize(s), "subset sync");
  for (int i = 0; i < SC_SLOTS; ++i) w[SC_SIZE] += w[SC_NWORDS + i];  // oSize (k_sub_runs' slots)
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ek0, c->ek1);
  res->kernel_ms += ms;
  if (gather) {
    float gms = 0.f;
    (void)hipEventElapsedTime(&gms, c->ev0, c->ev1);
    res->gather_ms = gms;
  }
  const u64 firstbad = w[SC_FIRSTBAD], Ke = w[SC_KE], nstart = w[SC_NSTART], size = w[SC_SIZE];
  const bool bad = firstbad != ~0ull;
  res->total_ms = now_ms() - t0;
  if (w[SC_FLAGS] & 1) {
    res->count = Ke;
    return sub_msg(res, SHOCKIDX_ESPACE, "row capacity too small");
  }
  if (w[SC_FLAGS] & 2) {
    res->count = Ke;
    res->runs = nstart;
    return sub_msg(res, SHOCKIDX_ESPACE, "run capacity too small");
  }
  res->count = Ke;
  res->size = size;
  // coCount: runs flushed by subset.go:245-261, plus the final one when oSize != 0 (:285-291);
  // at an error the open run was never flushed
  res->runs = bad ? (nstart ? nstart - 1 : 0) : (size ? nstart : (nstart ? nstart - 1 : 0));
  if (gather && !bad) {
    if (w[SC_FLAGS] & 8) return sub_msg(res, SHOCKIDX_EINVAL, "runs exceed the data");
    if (w[SC_FLAGS] & 4) return sub_msg(res, SHOCKIDX_ESPACE, "output capacity too small");
  }
  if (!bad) return SHOCKIDX_OK;
  // Go's error text for the first failing id
  const u64 r = firstbad >> 3;
  const u32 code = (u32)(firstbad & 7);
  i64 v = 0, prev = 0;
  if (int rc = d2h(c, &v, cval + r, res)) return rc;
  if (r) {
    if (int rc = d2h(c, &prev, cval + r - 1, res)) return rc;
  }
  char buf[256];
  if (code == SUB_SYNTAX || code == SUB_RANGE) {
    u64 li = 0, ln[2];
    if (int rc = d2h(c, &li, cline + r, res)) return rc;
    u64 e2[2] = {~0ull, 0};  // ends[li - 1], ends[li]: line li is [ends[li - 1] + 1, ends[li]]
    SUBCHK(hipMemcpyAsync(li ? e2 : e2 + 1, c->d_rows + (li ? li - 1 : 0), li ? 16 : 8, hipMemcpyDeviceToHost, s),
           "line copy");
    SUBCHK(hipStreamSynchronize(s), "sync");
    ln[0] = e2[0] + 1;  // (li == 0: ~0 + 1 = 0)
    ln[1] = e2[1] + 1 - ln[0];
    const u64 k = ln[1] - 1 < 200 ? ln[1] - 1 : 200;  // enough for a 255-byte message
    uint8_t txt[200];
    if (k) {
      SUBCHK(hipMemcpyAsync(txt, (const uint8_t *)d_ids + ln[0], k, hipMemcpyDeviceToHost, s), "text copy");
      SUBCHK(hipStreamSynchronize(s), "sync");
    }
    return sub_msg(res, SHOCKIDX_EFORMAT, "strconv.Atoi: parsing " + go_quote(txt, k) + ": " +
                                              (code == SUB_SYNTAX ? "invalid syntax" : "value out of range"));
  }
  if (code == SUB_SORT)
    snprintf(buf, sizeof buf,
             "Subset indices must be numerically sorted and non-redundant, found value %lld after value %lld",
             (long long)v, (long long)prev);
  else if (code == SUB_EXIST)
    snprintf(buf, sizeof buf, "Subset index: %lld does not exist in parent index file.", (long long)v);
  else
    snprintf(buf, sizeof buf, "Subset index could not read parent index file for part: %lld", (long long)v);
  return sub_msg(res, SHOCKIDX_EFORMAT, buf);
}

}  // namespace

extern "C" {

int shockidx_subset_index(shockidx_ctx *c, const void *d_ids, uint64_t ids_len, const void *d_parent,
                          uint64_t parent_count, int64_t ilength, void *d_rows, uint64_t rows_cap, void *d_runs,
                          uint64_t runs_cap, shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  return subset_build(c, d_ids, ids_len, d_parent, parent_count, ilength, d_rows, rows_cap, d_runs, runs_cap, nullptr,
                      0, nullptr, 0, res ? res : &tmp);
}

int shockidx_subset_node(shockidx_ctx *c, const void *d_ids, uint64_t ids_len, const void *d_parent,
                         uint64_t parent_count, int64_t ilength, void *d_rows, uint64_t rows_cap, void *d_runs,
                         uint64_t runs_cap, const void *d_data, uint64_t data_len, void *d_out, uint64_t out_cap,
                         shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  if (!d_data) {
    if (!res) res = &tmp;
    sub_reset(res);
    return sub_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  }
  return subset_build(c, d_ids, ids_len, d_parent, parent_count, ilength, d_rows, rows_cap, d_runs, runs_cap, d_data,
                      data_len, d_out, out_cap, res ? res : &tmp);
}

int shockidx_subset_gather(shockidx_ctx *c, const void *d_data, uint64_t data_len, const void *d_runs, uint64_t nruns,
                           void *d_out, uint64_t out_cap, shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  if (!res) res = &tmp;
  sub_reset(res);
  if (!c || (!d_runs && nruns) || ((uintptr_t)d_data & 15) || ((uintptr_t)d_out & 15))
    return sub_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  SUBCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  res->runs = nruns;
  if (!nruns) return SHOCKIDX_OK;
  size_t scan_bytes = 0;
  SUBCHK(sidx_gather(nullptr, 0, nullptr, nruns, nullptr, nullptr, nullptr, nullptr, &scan_bytes, nullptr, nullptr, 0,
                     nullptr, nullptr, s),
         "scan size");
  // runs are disjoint pieces of the parent file, so the output is at most data_len bytes
  const u64 max_blocks = (out_cap < data_len ? out_cap : data_len) / sidx::GATHER_BLOCK + 2;
  const u64 need = 8 * SC_ALLWORDS + 16 * (nruns + 16) + scan_bytes + 8 * max_blocks + 4096;
  {
    shockidx_result wr;
    memset(&wr, 0, sizeof wr);
    if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, need, 1, &wr)) return sub_msg(res, rc, wr.err);
  }
  Carver cv{c->d_sub};
  u64 *ctl = cv.take<u64>(SC_ALLWORDS);
  u64 *lens = cv.take<u64>(nruns);
  u64 *outoff = cv.take<u64>(nruns);
  void *scan_tmp = cv.take<uint8_t>(scan_bytes);
  u64 *wfirst = cv.take<u64>(max_blocks);
  SUBCHK(sidx_subset_init(ctl, nruns, s), "init");
  SUBCHK(sidx_gather((const uint8_t *)d_data, data_len, (const u64 *)d_runs, nruns, ctl, lens, outoff, scan_tmp,
                     &scan_bytes, wfirst, (uint8_t *)d_out, out_cap, c->ek0, c->ek1, s),
         "gather");
  u64 w[SC_NWORDS];
  SUBCHK(hipMemcpyAsync(w, ctl, sizeof w, hipMemcpyDeviceToHost, s), "control copy");
  SUBCHK(hipStreamSynchronize(s), "gather sync");
  res->size = w[SC_TOTAL];
  res->total_ms = now_ms() - t0;
  if (w[SC_FLAGS] & 8) return sub_msg(res, SHOCKIDX_EINVAL, "runs exceed the data");
  if (w[SC_FLAGS] & 4) return sub_msg(res, SHOCKIDX_ESPACE, "output capacity too small");
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ek0, c->ek1);
  res->kernel_ms = ms;
  return SHOCKIDX_OK;
}

int shockidx_create_subset_index(shockidx_ctx *c, const void *d_ids, uint64_t ids_len, const void *d_parent,
                                 uint64_t parent_count, int64_t ilength, void *d_rows, uint64_t rows_cap,
                                 shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  if (!res) res = &tmp;
  // subset.go:36-128: the same per-id checks and rows as CreateSubsetNodeIndexes, no
  // compressed index; every error returns (-1, -1, err)
  const int rc = shockidx_subset_index(c, d_ids, ids_len, d_parent, parent_count, ilength, d_rows, rows_cap, nullptr,
                                       0, res);
  res->runs = 0;
  if (rc == SHOCKIDX_EFORMAT) res->count = res->size = ~0ull;
  return rc;
}

}  // extern "C"

// ---- Index read path: Idx.Part / Idx.Range (index/index.go:67-193) ------------------------
namespace {

const char E_IDX_RANGE[] = "Invalid index record range";  // errors/errors.go:21-23
const char E_IDX_BOUNDS[] = "Index record out of bounds";
const char E_IDX_NOFILE[] = "Index file is missing";

// strconv.ParseInt(s, 10, 64); any error (syntax or range) is reported the same by the callers
bool go_parse_int64(const char *s, size_t n, i64 *v) {
  size_t i = 0;
  bool neg = false;
  if (n == 0) return false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == n) return false;
  u64 u = 0;
  for (; i < n; ++i) {
    const unsigned d = (unsigned char)s[i] - '0';
    if (d > 9 || u > (~0ull - d) / 10) return false;
    u = u * 10 + d;
  }
  if (!neg && u > (u64)INT64_MAX) return false;
  if (neg && u > (u64)INT64_MAX + 1) return false;
  *v = neg ? (i64)(0 - u) : (i64)u;
  return true;
}

// the part string: 0 = one record, 1 = a range start-end (strings.Split(part, "-")[0], [1]),
// -1 = Go's error text in *e
int parse_part(const char *part, i64 idx_length, i64 *a, i64 *b, const char **e) {
  const char *dash = strchr(part, '-');
  if (dash) {  // index.go:77-84 / :129-136
    const char *s1 = dash + 1, *d2 = strchr(s1, '-');
    i64 start = 0, end = 0;
    const bool ok0 = go_parse_int64(part, (size_t)(dash - part), &start);
    const bool ok1 = go_parse_int64(s1, d2 ? (size_t)(d2 - s1) : strlen(s1), &end);
    if (!ok0 || !ok1 || start <= 0 || start > idx_length || end <= 0 || end > idx_length) {
      *e = E_IDX_RANGE;
      return -1;
    }
    *a = start;
    *b = end;
    return 1;
  }
  i64 p = 0;  // index.go:100-105 / :178-183
  if (!go_parse_int64(part, strlen(part), &p) || p <= 0 || p > idx_length) {
    *e = E_IDX_BOUNDS;
    return -1;
  }
  *a = *b = p;
  return 0;
}

// row i of the device table (16 bytes D2H); a row past the table reads as `dflt`
int read_row(shockidx_ctx *c, const void *d_rows, u64 nrows, u64 i, const u64 dflt[2], u64 out[2],
             shockidx_subset_result *res) {
  if (i >= nrows) {
    out[0] = dflt[0];
    out[1] = dflt[1];
    return 0;
  }
  SUBCHK(hipMemcpyAsync(out, (const u64 *)d_rows + 2 * i, 16, hipMemcpyDeviceToHost, c->stream), "row copy");
  SUBCHK(hipStreamSynchronize(c->stream), "row sync");
  return 0;
}

}  // namespace

extern "C" {

int shockidx_idx_part(shockidx_ctx *c, const void *d_rows, uint64_t nrows, const char *part, int64_t idx_length,
                      int64_t *pos, int64_t *length, shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  if (!res) res = &tmp;
  sub_reset(res);
  if (!c || !part || !pos || !length) return sub_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  *pos = 0;
  *length = 0;
  const double t0 = now_ms();
  if (!d_rows) return sub_msg(res, SHOCKIDX_EFORMAT, E_IDX_NOFILE);  // index.go:70-74
  SUBCHK(hipSetDevice(c->device), "hipSetDevice");
  i64 a = 0, b = 0;
  const char *e = nullptr;
  const int kind = parse_part(part, idx_length, &a, &b, &e);
  if (kind < 0) return sub_msg(res, SHOCKIDX_EFORMAT, e);
  // fresh zeroed records (index.go:88,94,109): a read past the file leaves zeros
  static const u64 zero[2] = {0, 0};
  u64 sr[2], er[2];
  if (int rc = read_row(c, d_rows, nrows, (u64)(a - 1), zero, sr, res)) return rc;
  if (kind == 0) {
    *pos = (i64)sr[0];
    *length = (i64)sr[1];
  } else {
    if (int rc = read_row(c, d_rows, nrows, (u64)(b - 1), zero, er, res)) return rc;
    *pos = (i64)sr[0];
    *length = (i64)(er[0] - sr[0] + er[1]);  // index.go:98-99 (int64 arithmetic wraps)
  }
  res->count = 1;
  res->total_ms = now_ms() - t0;
  return SHOCKIDX_OK;
}

int shockidx_idx_range(shockidx_ctx *c, const void *d_rows, uint64_t nrows, const char *part, int64_t idx_length,
                       void *d_recs, uint64_t recs_cap, shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  if (!res) res = &tmp;
  sub_reset(res);
  if (!c || !part || (!d_recs && recs_cap)) return sub_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  if (!d_rows) return sub_msg(res, SHOCKIDX_EFORMAT, E_IDX_NOFILE);  // index.go:122-126
  SUBCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  i64 a = 0, b = 0;
  const char *e = nullptr;
  const int kind = parse_part(part, idx_length, &a, &b, &e);
  if (kind < 0) return sub_msg(res, SHOCKIDX_EFORMAT, e);
  const u64 a0 = (u64)(a - 1);
  if (kind == 0 || a == b) {  // one record (index.go:146-150, :185-191): rec starts zeroed
    static const u64 zero[2] = {0, 0};
    u64 r[2];
    if (int rc = read_row(c, d_rows, nrows, a0, zero, r, res)) return rc;
    res->count = 1;
    if (recs_cap < 1) return sub_msg(res, SHOCKIDX_ESPACE, "record capacity too small");
    SUBCHK(hipMemcpyAsync(d_recs, r, 16, hipMemcpyHostToDevice, s), "rec copy");
    SUBCHK(hipStreamSynchronize(s), "rec sync");
    res->total_ms = now_ms() - t0;
    return SHOCKIDX_OK;
  }
  if (b < a) {  // the coalescing loop runs zero times: an empty list, no error
    res->total_ms = now_ms() - t0;
    return SHOCKIDX_OK;
  }
  const u64 nr = (u64)(b - a) + 1;
  if (nr > (u64)INT32_MAX) return sub_msg(res, SHOCKIDX_EINVAL, "range too large for one call");
  size_t scan_bytes = 0;
  SUBCHK(sidx_scan_flags(nullptr, nullptr, nr, nullptr, &scan_bytes, s), "scan size");
  const u64 need = 12 * (nr + 64) + scan_bytes + 4096;
  {
    shockidx_result wr;
    memset(&wr, 0, sizeof wr);
    if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, need, 1, &wr)) return sub_msg(res, rc, wr.err);
  }
  Carver cv{c->d_sub};
  u32 *flags = cv.take<u32>(nr);
  u64 *id = cv.take<u64>(nr);
  void *scan_tmp = cv.take<uint8_t>(scan_bytes);
  SUBCHK(hipEventRecord(c->ek0, s), "event");
  SUBCHK(sidx_range_flags((const u64 *)d_rows, nrows, a0, nr, flags, s), "range flags");
  SUBCHK(sidx_scan_flags(flags, id, nr, scan_tmp, &scan_bytes, s), "scan");
  u64 lid = 0;
  u32 lf = 0;
  if (int rc = d2h(c, &lid, id + nr - 1, res)) return rc;
  if (int rc = d2h(c, &lf, flags + nr - 1, res)) return rc;
  const u64 nrec = lid + lf;
  res->count = nrec;
  if (nrec > recs_cap) return sub_msg(res, SHOCKIDX_ESPACE, "record capacity too small");
  SUBCHK(sidx_range_emit((const u64 *)d_rows, nrows, a0, nr, flags, id, (u64 *)d_recs, s), "range emit");
  SUBCHK(hipEventRecord(c->ek1, s), "event");
  SUBCHK(hipStreamSynchronize(s), "range sync");
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ek0, c->ek1);
  res->kernel_ms = ms;
  res->total_ms = now_ms() - t0;
  return SHOCKIDX_OK;
}

}  // extern "C"

extern "C" {

struct shockidx_comm {
  ncclComm_t comm;
  hipStream_t stream;
  int device;
};

int shockidx_comm_unique_id(void *id128) {
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return SHOCKIDX_EHIP;
  memcpy(id128, &id, sizeof id);
  return SHOCKIDX_OK;
}

int shockidx_comm_init(shockidx_ctx *c, int world, int rank, const void *id128, shockidx_comm **out) {
  if (!c || !id128 || !out) return SHOCKIDX_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return SHOCKIDX_EHIP;
  ncclUniqueId id;
  memcpy(&id, id128, sizeof id);
  shockidx_comm *m = new shockidx_comm();
  m->stream = c->stream;
  m->device = c->device;
  if (ncclCommInitRank(&m->comm, world, id, rank) != ncclSuccess) {
    delete m;
    return SHOCKIDX_EHIP;
  }
  *out = m;
  return SHOCKIDX_OK;
}

int shockidx_comm_allgather(shockidx_comm *m, const void *d_send, void *d_recv, uint64_t bytes) {
  if (!m) return SHOCKIDX_EINVAL;
  if (hipSetDevice(m->device) != hipSuccess) return SHOCKIDX_EHIP;
  if (ncclAllGather(d_send, d_recv, bytes, ncclUint8, m->comm, m->stream) != ncclSuccess) return SHOCKIDX_EHIP;
  return SHOCKIDX_OK;
}

int shockidx_comm_count(const shockidx_comm *m, int *nranks) {
  if (!m || !nranks) return SHOCKIDX_EINVAL;
  int n = 0;
  if (ncclCommCount(m->comm, &n) != ncclSuccess) return SHOCKIDX_EHIP;
  *nranks = n;
  return SHOCKIDX_OK;
}

int shockidx_comm_destroy(shockidx_comm *m) {
  if (!m) return SHOCKIDX_EINVAL;
  ncclCommDestroy(m->comm);
  delete m;
  return SHOCKIDX_OK;
}

int shockidx_detect(shockidx_ctx *c, const void *data, uint64_t n, int *fmt, int *mask) {
  shockidx_result tmp;
  shockidx_result *res = &tmp;
  reset_result(res);
  if (!c || (!data && n) || !fmt) return SHOCKIDX_EINVAL;
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  const u64 m = n < 32768 ? n : 32768;
  if (int rc = ensure_dev(c, (void **)&c->d_in, &c->d_in_cap, m + 64, 1, res, true)) return rc;
  if (m) {
    memcpy(c->h_stage[0], data, m);
    HIPCHK(hipMemcpyAsync(c->d_in, c->h_stage[0], m, hipMemcpyHostToDevice, s), "H2D");
  }
  int *d_det = (int *)(c->d_small + SMALL_DETECT);
  HIPCHK(sidx_launch_detect(c->d_in, m, d_det, s), "detect launch");
  HIPCHK(hipMemcpyAsync(c->h_det, d_det, 2 * sizeof(int), hipMemcpyDeviceToHost, s), "detect copy");
  HIPCHK(hipStreamSynchronize(s), "detect sync");
  *fmt = c->h_det[0];
  if (mask) *mask = c->h_det[1];
  return SHOCKIDX_OK;
}

}  // extern "C"

// ---- Download filters on device: fq2fa / anonymize (node/filter/) --------------------------
extern "C" {

int shockidx_filter_device(shockidx_ctx *c, const char *filter, const void *d_data, uint64_t n, void *d_out,
                           uint64_t out_cap, shockidx_subset_result *res) {
  shockidx_subset_result tmp;
  if (!res) res = &tmp;
  sub_reset(res);
  if (!c || !filter || (!d_data && n) || ((uintptr_t)d_data & 15) || (!d_out && out_cap))
    return sub_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  int kind = 0;  // filter.go:13-16
  if (!strcmp(filter, "fq2fa")) kind = 1;
  else if (!strcmp(filter, "anonymize")) kind = 2;
  else return sub_msg(res, SHOCKIDX_EINVAL, "unknown filter");
  const double t0 = now_ms();
  SUBCHK(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  const uint8_t *dd = (const uint8_t *)d_data;
  shockidx_result br;
  reset_result(&br);
  if (kind == 2) {  // anonymize reads through multi.Reader: DetermineFormat first (multi.go:43-62)
    int kfmt = 0;
    if (int rc = resolve_format(c, dd, n, SHOCKIDX_RECORD, SHOCKIDX_FMT_AUTO, s, &kfmt, &br))
      return sub_msg(res, rc, std::string(br.err, br.err_len));
    if (kfmt != SHOCKIDX_FMT_FASTQ) return anonymize_other(c, dd, n, kfmt, (uint8_t *)d_out, out_cap, res, t0);
  }
  // the record index (GetReadOffset) gives the record boundaries up to its first error; its tile
  // pass keeps every record's line ends for the spans
  c->want_spans = !getenv("SHOCKIDX_FILTER_RESCAN");
  const int brc = build_resident(c, dd, n, SHOCKIDX_RECORD, SHOCKIDX_FMT_FASTQ, s, &br);
  c->want_spans = false;
  if (brc < 0) return sub_msg(res, brc, std::string(br.err, br.err_len));
  const u64 K = br.count;
  res->kernel_ms += br.kernel_ms;
  size_t scan_bytes = 0;
  SUBCHK(sidx_scan_u64(nullptr, nullptr, K ? K : 1, nullptr, &scan_bytes, s), "scan size");
  // the output blocks' first records: the output is at most the section + 11 bytes per record
  const u64 nwf = (n + 11 * K) / sidx_filter_block() + 4;
  const u64 need = 48 * (K + 8) + scan_bytes + 8 * nwf + 4096;
  {
    shockidx_result wr;
    memset(&wr, 0, sizeof wr);
    if (int rc = ensure_dev(c, (void **)&c->d_sub, &c->d_sub_cap, need, 1, &wr)) return sub_msg(res, rc, wr.err);
  }
  Carver cv{c->d_sub};
  u64 *small = cv.take<u64>(8);
  u32 *spans = cv.take<u32>(6 * (K + 1));
  u64 *outlen = cv.take<u64>(K + 1);
  u64 *outoff = cv.take<u64>(K + 1);
  void *scan_tmp = cv.take<uint8_t>(scan_bytes);
  u64 *wfirst = cv.take<u64>(nwf);
  SUBCHK(hipEventRecord(c->ek0, s), "event");
  SUBCHK(hipMemsetAsync(small, 0xFF, 8, s), "memset");
  if (c->last_spans && K) {  // the certified records' spans from the tile pass; k_fq_spans does the rest
    SUBCHK(hipMemsetAsync(outlen, 0, 8 * K, s), "memset");
    SUBCHK(sidx_launch_fq_spans_place(&c->last_p, spans, outlen, K, kind, s), "spans place");
  }
  SUBCHK(sidx_filter_spans(dd, n, c->d_rows, K, kind, spans, outlen, small, s), "filter spans");
  u64 firstbad = ~0ull;
  if (int rc = d2h(c, &firstbad, small, res)) return rc;
  // Read()'s first failing record: one the index accepted but Read rejects (a blank-looking ID
  // or sequence line), else the index's own terminal record re-checked in Read's order
  u64 Ke = K;
  u32 code = ST_END;
  if (firstbad != ~0ull) {
    Ke = firstbad >> 4;
    code = (u32)(firstbad & 15);
  } else if (brc == SHOCKIDX_EFORMAT) {
    u64 last[2] = {0, 0};
    if (K) SUBCHK(hipMemcpyAsync(last, c->d_rows + 2 * (K - 1), 16, hipMemcpyDeviceToHost, s), "row copy");
    SUBCHK(sidx_filter_read_status(dd, n, K ? last[0] + last[1] : 0, (u32 *)(small + 1), s), "read status");
    u32 st = 0;
    if (int rc = d2h(c, &st, small + 1, res)) return rc;
    if (st == ST_OK || st == ST_END) return sub_msg(res, SHOCKIDX_EINTERNAL, "internal error: filter terminal record");
    code = st;
  } else if (K) {  // the last record's quality line ends at EOF: Read returns it with io.EOF, dropped
    u64 last[2] = {0, 0};
    uint8_t lastb = '\n';
    SUBCHK(hipMemcpyAsync(last, c->d_rows + 2 * (K - 1), 16, hipMemcpyDeviceToHost, s), "row copy");
    if (n) SUBCHK(hipMemcpyAsync(&lastb, dd + n - 1, 1, hipMemcpyDeviceToHost, s), "byte copy");
    SUBCHK(hipStreamSynchronize(s), "sync");
    if (last[0] + last[1] == n && lastb != '\n') Ke = K - 1;
  }
  u64 total = 0;
  if (Ke) {
    SUBCHK(sidx_scan_u64(outlen, outoff, Ke, scan_tmp, &scan_bytes, s), "scan");
    u64 lo = 0, ll = 0;
    if (int rc = d2h(c, &lo, outoff + Ke - 1, res)) return rc;
    if (int rc = d2h(c, &ll, outlen + Ke - 1, res)) return rc;
    total = lo + ll;
  }
  res->count = Ke;
  res->size = total;
  if (total > out_cap) return sub_msg(res, SHOCKIDX_ESPACE, "output capacity too small");
  if (total / sidx_filter_block() + 1 > nwf) return sub_msg(res, SHOCKIDX_EINTERNAL, "internal error: filter plan size");
  SUBCHK(sidx_filter_write(dd, n, c->d_rows, spans, outlen, outoff, Ke, total, kind, wfirst, (uint8_t *)d_out, s),
         "filter write");
  SUBCHK(hipEventRecord(c->ek1, s), "event");
  SUBCHK(hipStreamSynchronize(s), "filter sync");
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ek0, c->ek1);
  res->kernel_ms += ms;
  res->total_ms = now_ms() - t0;
  if (code == ST_END) return SHOCKIDX_OK;
  const char *m = status_message(code);
  return sub_msg(res, SHOCKIDX_EFORMAT, m ? m : "internal error: filter status");
}

}  // extern "C"
