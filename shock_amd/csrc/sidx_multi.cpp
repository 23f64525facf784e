// sidx_multi.cpp -- one node file indexed across several GPUs from a single process.
//
// The Shock server is one process: node.AsyncIndexer runs Indexers[type](f).Create(out) in a
// goroutine (shock-server/node/index.go:107-121), record.Create reads the file once
// (node/file/index/record.go:34-90).  A multi-device group replaces that call on a multi-GPU
// node with the slab protocol of SURVEY.md §8(e), driven from one process:
//   1. cut the file into 16-byte-aligned byte slabs, one per device; stage slab k (with 64 KiB
//      in front and a 4 MiB halo after it) into devices[k]'s HBM -- all devices at once, each
//      over its own PCIe link;
//   2. guess each slab's incoming reader state and index it (shockidx_slab_guess / _index: the
//      tile passes), concurrently on every device;
//   3. all-gather the 64-byte slab summaries -- one RCCL all-gather over xGMI, communicators
//      from ncclCommInitAll (or through host memory when a device is listed twice);
//   4. fold them on every device (shockidx_slab_combine): true incoming states, each slab's
//      first global record, the global count / first error; re-run a slab whose guess was
//      wrong and exchange again (never on well-formed data);
//   5. copy each slab's owned rows into the caller's table at its first global record.
// The table, count and Go error text equal shockidx_build_host's on the same bytes.  A record
// longer than the halo that crosses a slab end is rebuilt on devices[0] alone.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/shockidx.h"
#include "sidx_host.hpp"

using namespace sidx_host;

namespace {

typedef uint64_t u64;
constexpr u64 FRONT = 64ull << 10;  // bytes staged before a slab (state guess, trim look-behind)
constexpr u64 HALO = 4ull << 20;    // bytes staged after a slab (records crossing its end)
constexpr u64 ALIGN = 16;           // slab cuts: 16-byte aligned device loads
// device statuses (sidx_common.hpp)
constexpr uint32_t ST_OK = 0, ST_END = 1, ST_FA_INVALID = 10, ST_NEEDMORE = 12, ST_ABSENT = 13;
constexpr int HALO_EXHAUSTED = 1000;  // internal: rebuild on one device

// [lo, hi) per slab, equal up to alignment; only slab 0 starts at 0; empty slabs come last
// (the cuts of shock_amd/dist.py plan_slabs / slab_window)
void plan_slabs(u64 size, int world, u64 *lo, u64 *hi, u64 *wlo, u64 *whi) {
  std::vector<u64> cut(world + 1);
  cut[0] = 0;
  cut[world] = size;
  for (int r = 1; r < world; ++r) {
    u64 c = ((size * (u64)r / (u64)world + ALIGN - 1) / ALIGN) * ALIGN;
    if (c < ALIGN) c = ALIGN;
    cut[r] = c < size ? c : size;
  }
  for (int r = 0; r < world; ++r) {
    lo[r] = cut[r];
    hi[r] = cut[r + 1] > cut[r] ? cut[r + 1] : cut[r];
    wlo[r] = (lo[r] > FRONT ? lo[r] - FRONT : 0) / ALIGN * ALIGN;
    whi[r] = hi[r] + HALO < size ? hi[r] + HALO : size;
  }
}

// a state with its record count dropped: what a slab is indexed against (dist.local_state)
u64 local_state(int fmt, u64 s) {
  if (fmt == SHOCKIDX_FMT_FASTQ || fmt == SHOCKIDX_FMT_SAM) return s & 3;
  if (fmt == SHOCKIDX_FMT_FASTA) return s & 1;
  return 0;
}

struct Slab {
  shockidx_slab sl;
  void *d_rows = nullptr;
  u64 cap = 0;
  u64 local_count = 0;
  uint32_t local_flags = 0;
  u64 row_base = 0;
  shockidx_result r;
  shockidx_slab_plan plan;
  int rc = 0;
};

// f(k) for every slab on its own thread; the first failing slab's code
template <class F>
int par(int n, F f) {
  std::vector<int> rc(n, 0);
  std::vector<std::thread> th;
  for (int k = 1; k < n; ++k) th.emplace_back([&, k] { rc[k] = f(k); });
  rc[0] = f(0);
  for (auto &t : th) t.join();
  for (int k = 0; k < n; ++k)
    if (rc[k]) return rc[k];
  return 0;
}

}  // namespace

struct shockidx_multi {
  int n = 0;
  std::vector<int> dev;
  std::vector<shockidx_ctx *> ctx;
  std::vector<uint8_t *> d_sum;   // per slab on its device: 64-byte summary | 64 x n gathered
  std::vector<ncclComm_t> comm;   // one per device (empty: host exchange)
  std::vector<void *> d_rows;     // row tables of the host / fd builds (grow-only)
  std::vector<u64> rows_cap;
  uint32_t builds = 0;            // builds run: each slab index is tagged (builds << 4 | round)
  std::vector<uint32_t> expect;   // per slab: the tag its summary must carry at the next fold
  uint32_t inject = 0;            // test hooks (shockidx_multi_debug_inject): bit0 the host
                                  // exchange skips its copy into the gathered buffers
};

namespace {

int exchange(shockidx_multi *m, shockidx_result *res) {
  const int n = m->n;
  if (!m->comm.empty()) {  // one RCCL all-gather of 64 B per device over xGMI
    if (ncclGroupStart() != ncclSuccess) return set_msg(res, SHOCKIDX_EHIP, "ncclGroupStart");
    for (int k = 0; k < n; ++k) {
      if (ncclAllGather(m->d_sum[k], m->d_sum[k] + 64, 64, ncclUint8, m->comm[k], ctx_stream(m->ctx[k])) !=
          ncclSuccess) {
        (void)ncclGroupEnd();
        return set_msg(res, SHOCKIDX_EHIP, "ncclAllGather");
      }
    }
    if (ncclGroupEnd() != ncclSuccess) return set_msg(res, SHOCKIDX_EHIP, "ncclGroupEnd");
    for (int k = 0; k < n; ++k) {
      hipError_t e = hipSetDevice(m->dev[k]);
      if (e == hipSuccess) e = hipStreamSynchronize(ctx_stream(m->ctx[k]));
      if (e != hipSuccess) return set_hip(res, e, "all-gather sync");
    }
    return 0;
  }
  // Both copies go on the slab's own stream and are waited for there.  The context streams are
  // non-blocking, so a null-stream hipMemcpy is not ordered with them, and a pageable
  // host-to-device hipMemcpy may return before its DMA lands: k_slab_combine on the slab's stream
  // could then read the previous round's gathered summaries (seen once as a short count).
  std::vector<uint8_t> all(64 * (size_t)n);
  if (m->inject & 1) return 0;  // test hook: the gathered buffers keep what the last exchange left
  for (int k = 0; k < n; ++k) {
    hipStream_t s = ctx_stream(m->ctx[k]);
    hipError_t e = hipSetDevice(m->dev[k]);
    if (e == hipSuccess) e = hipMemcpyAsync(all.data() + 64 * k, m->d_sum[k], 64, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return set_hip(res, e, "summary copy");
  }
  for (int k = 0; k < n; ++k) {
    hipStream_t s = ctx_stream(m->ctx[k]);
    hipError_t e = hipSetDevice(m->dev[k]);
    if (e == hipSuccess) e = hipMemcpyAsync(m->d_sum[k] + 64, all.data(), all.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return set_hip(res, e, "summary copy");
  }
  return 0;
}

// Index slab k against `state`; a row table that turns out too small is grown (when the group
// owns it) and the slab indexed again.
int index_slab(shockidx_multi *m, Slab *S, int k, int fmt, u64 state, bool own_rows, uint32_t seq) {
  Slab &s = S[k];
  s.sl.seq = seq;
  m->expect[k] = seq;
  for (int attempt = 0; attempt < 2; ++attempt) {
    int rc = shockidx_slab_index(m->ctx[k], &s.sl, fmt, state, s.d_rows, s.cap, m->d_sum[k], &s.r);
    if (rc) return rc;
    s.local_count = s.r.count;
    s.local_flags = s.r.flags;
    if (!(s.local_flags & 1)) return 0;
    if (!own_rows) return set_msg(&s.r, SHOCKIDX_ESPACE, "row capacity too small");
    const u64 want = s.local_count + 1024;
    if (hipSetDevice(m->dev[k]) != hipSuccess) return SHOCKIDX_EHIP;
    (void)hipFree(m->d_rows[k]);
    m->d_rows[k] = nullptr;
    m->rows_cap[k] = 0;
    if (hipMalloc(&m->d_rows[k], 16 * want) != hipSuccess) return set_msg(&s.r, SHOCKIDX_ENOMEM, "hipMalloc(rows)");
    m->rows_cap[k] = want;
    s.d_rows = m->d_rows[k];
    s.cap = want;
  }
  return set_msg(&s.r, SHOCKIDX_EINTERNAL, "internal error: row capacity");
}

// steps 2-4 of the protocol over slabs whose windows are staged; S[k].plan filled
int run_slabs(shockidx_multi *m, Slab *S, int fmt, bool own_rows, shockidx_result *res) {
  const int n = m->n;
  const uint32_t build = ++m->builds;
  int rc = par(n, [&](int k) -> int {
    u64 g = 0;
    if (int r = shockidx_slab_guess(m->ctx[k], &S[k].sl, fmt, &g)) return r;
    return index_slab(m, S, k, fmt, g, own_rows, build << 4);
  });
  if (rc == SHOCKIDX_ESPACE) {  // caller-owned row tables too short: the rows the largest slab needs
    res->count = 0;
    for (int k = 0; k < n; ++k)
      if ((S[k].local_flags & 1) && S[k].local_count > res->count) res->count = S[k].local_count;
    return set_msg(res, rc, "row capacity too small");
  }
  for (int k = 0; k < n && rc; ++k)
    if (S[k].r.status < 0 || S[k].r.err_len) return set_msg(res, rc, S[k].r.err);
  if (rc) return set_msg(res, rc, "slab index failed");
  for (int round = 1;; ++round) {
    if (round > 4) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: slab states did not converge");
    if (int r = exchange(m, res)) return r;
    for (int k = 0; k < n; ++k) {
      if (int r = shockidx_slab_combine(m->ctx[k], m->d_sum[k] + 64, n, k, fmt, m->expect.data(), &S[k].plan))
        return set_msg(res, r, "slab combine failed");
      if (S[k].plan.flags & 32) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: stale slab summary");
    }
    const uint32_t bad = S[0].plan.inconsistent;
    if (!bad) break;
    rc = par(n, [&](int k) -> int {
      return ((bad >> k) & 1)
                 ? index_slab(m, S, k, fmt, local_state(fmt, S[k].plan.state_in), own_rows, (build << 4) | (uint32_t)round)
                 : 0;
    });
    if (rc == SHOCKIDX_ESPACE) {
      res->count = 0;
      for (int k = 0; k < n; ++k)
        if ((S[k].local_flags & 1) && S[k].local_count > res->count) res->count = S[k].local_count;
      return set_msg(res, rc, "row capacity too small");
    }
    if (rc) return set_msg(res, rc, "slab re-index failed");
  }
  for (int k = 0; k < n; ++k) {
    const shockidx_slab_plan &p = S[k].plan;
    if (p.code == ST_NEEDMORE || (p.flags & 4)) return HALO_EXHAUSTED;
    if (p.flags & 2) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: device invariant violated");
  }
  for (int k = 0; k < n; ++k) {
    res->kernel_ms = S[k].r.kernel_ms > res->kernel_ms ? S[k].r.kernel_ms : res->kernel_ms;
    res->index_ms = S[k].r.index_ms > res->index_ms ? S[k].r.index_ms : res->index_ms;
    if (S[k].sl.n) res->path = (res->path == 0 || res->path == S[k].r.path) ? S[k].r.path : 2u;
  }
  return 0;
}

u64 rows_owned(const shockidx_slab_plan &p, u64 local_count, u64 row_base) {
  const u64 delta = p.first_record - row_base;  // global - local record numbers (mod 2^64)
  if (p.count < delta) return 0;
  const u64 local_end = local_count < p.count - delta ? local_count : p.count - delta;
  return local_end > row_base ? local_end - row_base : 0;
}

// End-of-build invariants of a slab build (record.go:51-83: row i + 1 starts where row i ends):
// the slabs' owned rows add up to the count, each slab's first row starts where the rows before
// it end (the first at 0), and a successful build's rows end at the file end -- FASTQ: or before
// trailing blank lines (fastq.go:141-156).  row(k, i, out) reads owned row i of slab k, fetch
// file bytes.  A violation is an internal error, never a short table.
template <class Row, class Fetch>
int check_seams(const Slab *S, int w, u64 size, int kfmt, u64 count, Row row, Fetch fetch, shockidx_result *res) {
  u64 sum = 0, next = 0, last_len = 0;
  for (int k = 0; k < w; ++k) {
    const u64 own = rows_owned(S[k].plan, S[k].local_count, S[k].row_base);
    if (!own) continue;
    if (S[k].plan.first_record != sum) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: slab rows out of order");
    u64 a[2], b[2];
    if (int rc = row(k, 0, a)) return rc;
    if (int rc = row(k, own - 1, b)) return rc;
    if (a[0] != next) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: a slab's first row does not start where the previous slab's rows end");
    next = b[0] + b[1];
    last_len = b[1];
    sum += own;
  }
  if (sum != count) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: slab rows do not add up to the count");
  const uint32_t code = S[0].plan.code;
  if (code == ST_OK || code == ST_END || code == ST_ABSENT) {
    bool bad = next > size || (next < size && kfmt != SHOCKIDX_FMT_FASTQ);
    if (!bad && next < size) {
      uint8_t x = 0, y = 0;
      if (int rc = fetch(next, 1, &x)) return rc;
      if (int rc = fetch(size - 1, 1, &y)) return rc;
      bad = x != '\n' || y != '\n';
    }
    if (!bad && kfmt == SHOCKIDX_FMT_LINE && last_len && size) {  // the last row: the bytes after the last '\n'
      uint8_t z = 0;
      if (int rc = fetch(size - 1, 1, &z)) return rc;
      bad = z == '\n';
    }
    if (bad) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: the rows do not end at the end of the file");
  }
  return 0;
}

// Go's (status, text) for the folded result; FASTA pieces are read by fetch(pos, n, dst)
template <class Fetch>
int finish_status(const shockidx_slab_plan &p, shockidx_result *res, Fetch fetch) {
  if (p.code == ST_OK || p.code == ST_END || p.code == ST_ABSENT) {
    res->status = SHOCKIDX_OK;
    return SHOCKIDX_OK;
  }
  if (p.code == ST_FA_INVALID) {  // fasta.go:115-121
    static const char pre[] = "Invalid fasta entry: ";
    const u64 show = p.err_len < 50 ? p.err_len : 50;
    memcpy(res->err, pre, sizeof pre - 1);
    if (show)
      if (int rc = fetch(p.err_pos, show, (uint8_t *)res->err + sizeof pre - 1)) return rc;
    res->err_len = sizeof pre - 1 + show;
    res->err[res->err_len] = 0;
    res->status = SHOCKIDX_EFORMAT;
    return SHOCKIDX_EFORMAT;
  }
  const char *msg = status_message(p.code);
  if (!msg) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: unknown status");
  return set_msg(res, SHOCKIDX_EFORMAT, msg);
}

int resolve_fmt(shockidx_multi *m, const uint8_t *head, u64 hn, int kind, int fmt, int *out, shockidx_result *res) {
  if (kind == SHOCKIDX_LINE) { *out = SHOCKIDX_FMT_LINE; return 0; }
  if (kind != SHOCKIDX_RECORD) return set_msg(res, SHOCKIDX_EINVAL, "invalid index kind");
  if (fmt == SHOCKIDX_FMT_AUTO) {
    int f = 0, mask = 0;
    if (int rc = shockidx_detect(m->ctx[0], head, hn, &f, &mask)) return set_msg(res, rc, "format detection failed");
    if (f == SHOCKIDX_FMT_NONE) return set_msg(res, SHOCKIDX_EFORMAT, "Invalid file type for filter");  // errors.go:20
    fmt = f;
  }
  if (fmt != SHOCKIDX_FMT_FASTA && fmt != SHOCKIDX_FMT_FASTQ && fmt != SHOCKIDX_FMT_SAM && fmt != SHOCKIDX_FMT_LINE)
    return set_msg(res, SHOCKIDX_EINVAL, "invalid format");
  *out = fmt;
  return 0;
}

void set_geometry(Slab &s, const uint8_t *d_win, u64 size, u64 lo, u64 hi, u64 wlo, u64 whi, int k) {
  s.sl.d_data = d_win + (lo - wlo);
  s.sl.n = hi - lo;
  s.sl.end = whi - lo;
  s.sl.front = lo - wlo;
  s.sl.base = lo;
  s.sl.is_first = (k == 0);
  s.sl.is_last = (whi == size);
  s.row_base = k == 0 ? 0 : 1;  // record 0 belongs to the first slab
}

// build_host / build_fd: data (or fd) of n bytes -> *rows (malloc'ed)
int multi_build(shockidx_multi *m, const void *data, int fd, u64 n, int kind, int fmt, uint64_t **rows,
                shockidx_result *res) {
  const double t0 = now_ms();
  const int w = m->n;
  auto single = [&]() -> int {  // one device: the plain build
    const int rc = data ? shockidx_build_host(m->ctx[0], data, n, kind, fmt, rows, res)
                        : shockidx_build_fd(m->ctx[0], fd, n, kind, fmt, rows, res);
    res->total_ms = now_ms() - t0;
    return rc;
  };
  if (w == 1 || n == 0) return single();
  // bytes of the file for the format head and the FASTA error text
  auto fetch = [&](u64 pos, u64 len, uint8_t *dst) -> int {
    if (data) {
      memcpy(dst, (const uint8_t *)data + pos, len);
      return 0;
    }
    u64 got = 0;
    while (got < len) {
      const ssize_t r = pread(fd, dst + got, len - got, (off_t)(pos + got));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) return set_msg(res, SHOCKIDX_EIO, r < 0 ? strerror(errno) : "unexpected end of file");
      got += (u64)r;
    }
    return 0;
  };
  std::vector<uint8_t> head(n < 32768 ? n : 32768);
  if (int rc = fetch(0, head.size(), head.data())) return rc;
  int kfmt = 0;
  if (int rc = resolve_fmt(m, head.data(), head.size(), kind, fmt, &kfmt, res)) return rc;
  res->format = kfmt;
  std::vector<u64> lo(w), hi(w), wlo(w), whi(w);
  plan_slabs(n, w, lo.data(), hi.data(), wlo.data(), whi.data());
  std::vector<Slab> S(w);
  // 1. stage every window on its device (all PCIe links at once) and size its row table
  const double ts = now_ms();
  int rc = par(w, [&](int k) -> int {
    Slab &s = S[k];
    memset(&s.r, 0, sizeof s.r);
    const uint8_t *d_win = nullptr;
    if (int r = ctx_stage(m->ctx[k], data, fd, wlo[k], whi[k] - wlo[k], &d_win, &s.r)) return r;
    set_geometry(s, d_win, n, lo[k], hi[k], wlo[k], whi[k], k);
    const u64 bytes = hi[k] - lo[k];
    const u64 want = (kfmt == SHOCKIDX_FMT_LINE ? bytes / 16 : bytes / 32) + 4096;
    if (m->rows_cap[k] < want) {
      if (hipSetDevice(m->dev[k]) != hipSuccess) return SHOCKIDX_EHIP;
      (void)hipFree(m->d_rows[k]);
      m->d_rows[k] = nullptr;
      m->rows_cap[k] = 0;
      if (hipMalloc(&m->d_rows[k], 16 * want) != hipSuccess) return set_msg(&s.r, SHOCKIDX_ENOMEM, "hipMalloc(rows)");
      m->rows_cap[k] = want;
    }
    s.d_rows = m->d_rows[k];
    s.cap = m->rows_cap[k];
    return 0;
  });
  if (rc) {
    for (int k = 0; k < w; ++k)
      if (S[k].r.err_len) return set_msg(res, rc, S[k].r.err);
    return set_msg(res, rc, "slab staging failed");
  }
  res->h2d_ms = now_ms() - ts;
  // 2-4. guess, index, exchange, fold
  rc = run_slabs(m, S.data(), kfmt, true, res);
  if (rc == HALO_EXHAUSTED) {
    const double h2d = res->h2d_ms;
    rc = single();
    res->h2d_ms += h2d;
    return rc;
  }
  if (rc) return rc;
  // 5. rows owned by each slab into the table at its first global record
  const u64 count = S[0].plan.count;
  const double td = now_ms();
  uint64_t *out = alloc_rows(count * 16);
  if (!out) return set_msg(res, SHOCKIDX_ENOMEM, "out of host memory");
  rc = par(w, [&](int k) -> int {
    const u64 own = rows_owned(S[k].plan, S[k].local_count, S[k].row_base);
    if (!own) return 0;
    return ctx_to_host(m->ctx[k], S[k].d_rows, own * 16, out + 2 * S[k].plan.first_record, &S[k].r);
  });
  if (rc) {
    free(out);
    return set_msg(res, rc, "rows copy failed");
  }
  res->d2h_ms = now_ms() - td;
  rc = check_seams(S.data(), w, n, kfmt, count,
                   [&](int k, u64 i, u64 *o) -> int {
                     memcpy(o, out + 2 * (S[k].plan.first_record + i), 16);
                     return 0;
                   },
                   fetch, res);
  if (rc) {
    free(out);
    return rc;
  }
  res->count = count;
  rc = finish_status(S[0].plan, res, fetch);
  if (rc < 0) {
    free(out);
    return rc;
  }
  *rows = out;
  res->total_ms = now_ms() - t0;
  return rc;
}

}  // namespace

extern "C" {

int shockidx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int shockidx_multi_create(const int *devices, int n, shockidx_multi **out) {
  if (!devices || n < 1 || n > 32 || !out) return SHOCKIDX_EINVAL;
  *out = nullptr;
  shockidx_multi *m = new shockidx_multi();
  m->n = n;
  m->dev.assign(devices, devices + n);
  m->ctx.assign(n, nullptr);
  m->d_sum.assign(n, nullptr);
  m->d_rows.assign(n, nullptr);
  m->rows_cap.assign(n, 0);
  m->expect.assign(n, 0);
  int rc = SHOCKIDX_OK;
  for (int k = 0; k < n && rc == SHOCKIDX_OK; ++k) {
    rc = shockidx_ctx_create(devices[k], &m->ctx[k]);
    if (rc == SHOCKIDX_OK && (hipSetDevice(devices[k]) != hipSuccess ||
                              hipMalloc((void **)&m->d_sum[k], 64 + 64 * (size_t)n) != hipSuccess))
      rc = SHOCKIDX_EHIP;
  }
  if (rc != SHOCKIDX_OK) {
    shockidx_multi_destroy(m);
    return rc;
  }
  // RCCL when every device is distinct (one communicator per device, one process; a group of
  // one device is a world-1 communicator)
  bool distinct = true;
  for (int a = 0; a < n && distinct; ++a)
    for (int b = a + 1; b < n; ++b)
      if (devices[a] == devices[b]) distinct = false;
  const char *ex = getenv("SHOCKIDX_MULTI_EXCHANGE");
  if (distinct && !(ex && !strcmp(ex, "host"))) {
    m->comm.assign(n, nullptr);
    if (ncclCommInitAll(m->comm.data(), n, devices) != ncclSuccess) m->comm.clear();  // host exchange then
  }
  *out = m;
  return SHOCKIDX_OK;
}

void shockidx_multi_destroy(shockidx_multi *m) {
  if (!m) return;
  for (auto c : m->comm)
    if (c) (void)ncclCommDestroy(c);
  for (int k = 0; k < m->n; ++k) {
    if (hipSetDevice(m->dev[k]) == hipSuccess) {
      (void)hipFree(m->d_sum[k]);
      (void)hipFree(m->d_rows[k]);
    }
    shockidx_ctx_destroy(m->ctx[k]);
  }
  delete m;
}

int shockidx_multi_rccl(const shockidx_multi *m) { return m && !m->comm.empty() ? 1 : 0; }

// Diagnostic (not in the public header): slab k's context (its test hooks)
shockidx_ctx *shockidx_multi_debug_ctx(shockidx_multi *m, int k) { return m && k >= 0 && k < m->n ? m->ctx[k] : nullptr; }

// Diagnostic (not in the public header): the group's test hooks (shockidx_multi::inject);
// returns the previous flags.
int shockidx_multi_debug_inject(shockidx_multi *m, uint32_t flags) {
  if (!m) return SHOCKIDX_EINVAL;
  const int old = (int)m->inject;
  m->inject = flags;
  return old;
}

int shockidx_multi_build_host(shockidx_multi *m, const void *data, uint64_t n, int kind, int fmt, uint64_t **rows,
                              shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  memset(res, 0, sizeof *res);
  if (!m || !rows || (!data && n)) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  *rows = nullptr;
  return multi_build(m, data ? data : "", -1, n, kind, fmt, rows, res);
}

int shockidx_multi_build_fd(shockidx_multi *m, int fd, uint64_t n, int kind, int fmt, uint64_t **rows,
                            shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  memset(res, 0, sizeof *res);
  if (!m || !rows || fd < 0) return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  *rows = nullptr;
  return multi_build(m, nullptr, fd, n, kind, fmt, rows, res);
}

int shockidx_multi_create_index(shockidx_multi *m, int fd, uint64_t n, int kind, const char *tmpdir,
                                const char *outpath, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  uint64_t *rows = nullptr;
  int rc = shockidx_multi_build_fd(m, fd, n, kind, SHOCKIDX_FMT_AUTO, &rows, res);
  if (rc != SHOCKIDX_OK) {  // record.go:65-87: nothing is renamed into place on an error
    free(rows);
    return rc;
  }
  const double t0 = now_ms();
  const int wr = shockidx_write_idx(rows, res->count, tmpdir, outpath, res->err, sizeof res->err);
  free(rows);
  if (wr != SHOCKIDX_OK) {
    res->err_len = strlen(res->err);
    res->status = wr;
    return wr;
  }
  res->total_ms += now_ms() - t0;
  return SHOCKIDX_OK;
}

int shockidx_multi_plan(const shockidx_multi *m, uint64_t size, uint64_t *lo, uint64_t *hi, uint64_t *wlo,
                        uint64_t *whi) {
  if (!m || !lo || !hi || !wlo || !whi) return SHOCKIDX_EINVAL;
  plan_slabs(size, m->n, (u64 *)lo, (u64 *)hi, (u64 *)wlo, (u64 *)whi);
  return SHOCKIDX_OK;
}

int shockidx_multi_build_resident(shockidx_multi *m, uint64_t size, int kind, int fmt, const void *const *d_win,
                                  void *const *d_rows, const uint64_t *row_cap, uint64_t *first_record,
                                  uint64_t *rows_owned_out, shockidx_result *res) {
  shockidx_result tmp;
  if (!res) res = &tmp;
  memset(res, 0, sizeof *res);
  if (!m || !d_win || !d_rows || !row_cap || !first_record || !rows_owned_out || !size)
    return set_msg(res, SHOCKIDX_EINVAL, "invalid argument");
  const double t0 = now_ms();
  const int w = m->n;
  std::vector<u64> lo(w), hi(w), wlo(w), whi(w);
  plan_slabs(size, w, lo.data(), hi.data(), wlo.data(), whi.data());
  auto fetch = [&](u64 pos, u64 len, uint8_t *dst) -> int {  // from the window that holds pos
    int k = 0;
    while (k + 1 < w && !(pos >= wlo[k] && pos + len <= whi[k])) ++k;
    hipError_t e = hipSetDevice(m->dev[k]);
    if (e == hipSuccess) e = hipMemcpy(dst, (const uint8_t *)d_win[k] + (pos - wlo[k]), len, hipMemcpyDeviceToHost);
    return e == hipSuccess ? 0 : set_hip(res, e, "error text copy");
  };
  uint8_t head[32768];
  const u64 hn = whi[0] - wlo[0] < sizeof head ? whi[0] - wlo[0] : sizeof head;
  if (int rc = fetch(0, hn, head)) return rc;
  int kfmt = 0;
  if (int rc = resolve_fmt(m, head, hn, kind, fmt, &kfmt, res)) return rc;
  res->format = kfmt;
  std::vector<Slab> S(w);
  for (int k = 0; k < w; ++k) {
    memset(&S[k].r, 0, sizeof S[k].r);
    set_geometry(S[k], (const uint8_t *)d_win[k], size, lo[k], hi[k], wlo[k], whi[k], k);
    S[k].d_rows = d_rows[k];
    S[k].cap = row_cap[k];
  }
  int rc = run_slabs(m, S.data(), kfmt, false, res);
  if (rc == HALO_EXHAUSTED) return set_msg(res, SHOCKIDX_EINTERNAL, "internal error: slab halo exhausted");
  if (rc) return rc;
  rc = check_seams(S.data(), w, size, kfmt, S[0].plan.count,
                   [&](int k, u64 i, u64 *o) -> int {
                     return ctx_to_host(m->ctx[k], (const u64 *)d_rows[k] + 2 * i, 16, o, res);
                   },
                   fetch, res);
  if (rc) return rc;
  for (int k = 0; k < w; ++k) {
    first_record[k] = S[k].plan.first_record;
    rows_owned_out[k] = rows_owned(S[k].plan, S[k].local_count, S[k].row_base);
  }
  res->count = S[0].plan.count;
  rc = finish_status(S[0].plan, res, fetch);
  res->total_ms = now_ms() - t0;
  return rc;
}

}  // extern "C"
