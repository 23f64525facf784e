// sidx_filter.hip -- gfx950 kernels of the download filters:
// ?filter=fq2fa and ?filter=anonymize over a FASTQ node, as whole-section transforms on the
// device-resident record index.
//
// Reference semantics (paths relative to /root/reference/shock-server/):
//   node/filter/fq2fa/fq2fa.go:58-84       Read: fastq.Reader.Read() per record, fasta.Format
//   node/filter/anonymize/anonymize.go:28-56  Read: multi.Reader (format detected), ID =
//                                           fmt.Sprint(counter) from 1, the format's Format
//   node/file/format/fastq/fastq.go:50-132  Reader.Read: the checks of GetReadOffset, except
//       the ID and the sequence are tested after TrimSpace ("missing sequence ID" for "@ \n",
//       "empty sequence" for a blank-looking sequence line); a record whose quality line ends
//       at EOF comes back together with io.EOF, and the filters drop it
//   fasta/fasta.go:216-218 Format ">" ID "\n" Seq "\n";  fastq.go:283-285 Format
//       "@" ID "\n" Seq "\n+\n" Qual "\n"  (ID / Seq / Qual are the trimmed spans)
//
// Pipeline: record index (the FASTQ tile pass keeping each record's line ends) -> k_fq_spans_place
// (the certified records' spans, no re-read) -> k_fq_spans (the rest) (one lane per record: its three inner line
// ends, the trimmed ID / sequence / quality spans, the output length, Read's extra checks)
// -> exclusive scan of the output lengths -> k_fw_plan + k_fq_write (one workgroup per 16 KiB
// output block, 16 output bytes per thread).  The terminal record (the index's first error) is re-checked with
// Read's order by k_fq_read_status (one wave).
#include <hip/hip_runtime.h>
#include "sidx_scan.hpp"

#include "sidx_common.hpp"
#include "sidx_device.hpp"

namespace sidx {

enum FilterKind : int { FILT_FQ2FA = 1, FILT_ANON_FQ = 2 };
constexpr u64 NOLIM = ~0ull;

struct GAcc {  // plain global-memory byte view for trim_space
  const uint8_t *g;
  __device__ __forceinline__ u32 byte(u64 p) const { return g[p]; }
  __device__ __forceinline__ const uint8_t *ptr() const { return g; }
  __device__ __forceinline__ u64 base() const { return 0; }
};

__device__ __forceinline__ u32 ndigits(u64 v) {  // compares, no divisions
  u32 d = 1;
  u64 p = 10;
#pragma unroll
  for (int k = 1; k < 20; ++k) {
    d += v >= p ? 1u : 0u;
    p *= 10;
  }
  return d;
}

// Per record: spans relative to the record start (id_lo, id_len, seq_lo, seq_len, qual_lo,
// qual_len), the output length and Read's status for the checks the index did not make.
__global__ __launch_bounds__(256) void k_fq_spans(const uint8_t *data, u64 n, const u64 *rows, u64 K, int kind,
                                                  u32 *spans, u64 *outlen, u64 *firstbad) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  {  // spans already placed from the tile pass (sidx_kernels.hip k_fq_spans_place): drop the mark
    const u64 ol = outlen[i];
    if (ol >> 63) {
      outlen[i] = ol & ~(1ull << 63);
      return;
    }
  }
  const u64 off = rows[2 * i], len = rows[2 * i + 1], end = off + len;
  // the first three '\n' of the record (the index guarantees they exist inside it)
  u64 e0 = 0, e1 = 0, e2 = 0;
  u32 found = 0;
  // SIDX_SP_BATCH x 16 bytes per step, the loads issued together (one load per step cost a memory round
  // trip per 16 bytes: 6.1 ms per 10 GiB section)
#ifndef SIDX_SP_BATCH
#define SIDX_SP_BATCH 4  // 16-byte loads issued together per step (4: 11.8 ms fq2fa, 8: 12.0, 16: 12.7)
#endif
  for (u64 b0 = off & ~15ull; b0 < end && found < 3; b0 += 16 * SIDX_SP_BATCH) {
    uint4 v[SIDX_SP_BATCH];
#pragma unroll
    for (int k = 0; k < SIDX_SP_BATCH; ++k) {
      const u64 b = b0 + 16 * (u64)k;
      v[k] = (b + 16 <= n) ? load16(data + b) : (b < n ? load16_partial(data, b, n) : make_uint4(0, 0, 0, 0));
    }
#pragma unroll
    for (int k = 0; k < SIDX_SP_BATCH; ++k) {
      const u64 b = b0 + 16 * (u64)k;
      u32 m = b < end ? eq16(v[k], '\n') : 0u;
      if (b < off) m &= ~0u << (u32)(off - b);
      while (m && found < 3) {
        const u64 pos = b + (u64)__builtin_ctz(m);
        if (pos >= end) break;
        if (found == 0) e0 = pos;
        else if (found == 1) e1 = pos;
        else e2 = pos;
        ++found;
        m &= m - 1;
      }
    }
  }
  const GAcc a{data};
  u64 ilo, ihi, slo, shi, qlo, qhi;
  // the common record in one round of independent byte loads: every trimmed edge is a printable
  // ASCII byte and the record ends in '\n' -- TrimSpace then only drops the line ends; anything
  // else goes through trim_space (its dependent edge loops cost ~1.9 of 5.4 ms per 10 GiB)
  const bool shape = e0 >= off + 2 && e1 >= e0 + 2 && end >= e2 + 3;
  bool fast = false;
  if (shape) {
    const u32 c0 = data[off + 1], c1 = data[e0 - 1], c2 = data[e0 + 1], c3 = data[e1 - 1], c4 = data[e2 + 1],
              c5 = data[end - 2], c6 = data[end - 1];
    auto ok = [](u32 c) { return c < 0x80 && !ascii_space(c); };
    fast = ok(c0) && ok(c1) && ok(c2) && ok(c3) && ok(c4) && ok(c5) && c6 == '\n';
  }
  if (fast) {
    ilo = off + 1; ihi = e0; slo = e0 + 1; shi = e1; qlo = e2 + 1; qhi = end - 1;
  } else {
    trim_space(a, off + 1, e0 + 1, ilo, ihi);  // seqId = TrimSpace(seqId[1:])  (fastq.go:83)
    trim_space(a, e0 + 1, e1 + 1, slo, shi);   // seqBody (:96)
    trim_space(a, e2 + 1, end, qlo, qhi);      // qualBody (:123)
  }
  u32 st = ST_OK;
  if (ihi == ilo) st = ST_FQ_NOID;              // :84-87
  else if (shi == slo) st = ST_FQ_EMPTYSEQ;     // :97-100
  if (st != ST_OK) atomicMin((unsigned long long *)firstbad, (unsigned long long)((i << 4) | st));
  u32 *sp = spans + 6 * i;
  sp[0] = (u32)(ilo - off); sp[1] = (u32)(ihi - ilo);
  sp[2] = (u32)(slo - off); sp[3] = (u32)(shi - slo);
  sp[4] = (u32)(qlo - off); sp[5] = (u32)(qhi - qlo);
  outlen[i] = kind == FILT_FQ2FA ? (ihi - ilo) + (shi - slo) + 3
                                 : (u64)ndigits(i + 1) + (shi - slo) + (qhi - qlo) + 6;
}

// ---- k_fq_write: output-centric (round 3) ----------------------------------------------------
// One workgroup per 32 KiB block of the OUTPUT, each thread 16 aligned output bytes per step
// (a non-temporal 16-byte store): a record's output is a handful of segments -- literals, the
// counter's digits, runs of the section (ID / sequence / quality) -- and a chunk is the OR of
// the segments overlapping it, a run's bytes by two aligned 16-byte loads and a funnel shift
// (as k_gather).  The records overlapping a block are staged in LDS; the first one comes from
// k_fw_plan.  The one-wave-per-record copy it replaced moved bytes one lane at a time with byte
// stores (fq2fa 15.0 ms per 10 GiB section).
#ifndef SIDX_FW_RECS
#define SIDX_FW_RECS 512  // records staged per block (with the block: at most 64 output bytes per record on average)
#endif
#ifndef SIDX_FW_BLOCK
#define SIDX_FW_BLOCK 32768  // output bytes per workgroup
#endif
constexpr u32 FW_BLOCK = SIDX_FW_BLOCK, FW_THREADS = 256, FW_RECS = SIDX_FW_RECS;

__global__ void k_fw_plan(const u64 *outoff, const u64 *outlen, u64 K, u64 nblocks, u64 *wfirst) {
  const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= K) return;
  const u64 a = outoff[r], len = outlen[r];
  if (!len) return;
  for (u64 w = (a + FW_BLOCK - 1) / FW_BLOCK; w <= (a + len - 1) / FW_BLOCK && w < nblocks; ++w) wfirst[w] = r;
}

__device__ __forceinline__ u32 fw_fsh(u32 lo, u32 hi, u32 sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }
#ifndef SIDX_FW_CMAP
#define SIDX_FW_CMAP 1  // chunk -> record map in LDS (1) or a binary search per chunk (0)
#endif
// bytes [sh, sh + 16) of x:y, branch-free
__device__ __forceinline__ uint4 fw_shift16(const uint4 x, const uint4 y, u32 sh16) {
  const bool h = (sh16 & 8u) != 0, q = (sh16 & 4u) != 0;
  const u32 sh = sh16 & 3u;
  const u32 a0 = h ? x.z : x.x, a1 = h ? x.w : x.y, a2 = h ? y.x : x.z, a3 = h ? y.y : x.w, a4 = h ? y.z : y.x,
            a5 = h ? y.w : y.y;
  const u32 b0 = q ? a1 : a0, b1 = q ? a2 : a1, b2 = q ? a3 : a2, b3 = q ? a4 : a3, b4 = q ? a5 : a4;
  return make_uint4(fw_fsh(b0, b1, sh), fw_fsh(b1, b2, sh), fw_fsh(b2, b3, sh), fw_fsh(b3, b4, sh));
}
__device__ __forceinline__ u32 fw_m4(u32 b, u32 lo, u32 hi) {  // bytes [lo, hi) of the dword at byte b
  const u32 l = lo > b ? (lo - b < 4 ? lo - b : 4) : 0, h = hi > b ? (hi - b < 4 ? hi - b : 4) : 0;
  const u32 mh = h >= 4 ? ~0u : ((1u << (8 * h)) - 1u), ml = l >= 4 ? ~0u : ((1u << (8 * l)) - 1u);
  return mh & ~ml;
}
__device__ __forceinline__ void fw_or_masked(uint4 &acc, const uint4 d, u32 lo, u32 hi) {
  acc.x |= d.x & fw_m4(0, lo, hi); acc.y |= d.y & fw_m4(4, lo, hi);
  acc.z |= d.z & fw_m4(8, lo, hi); acc.w |= d.w & fw_m4(12, lo, hi);
}
__device__ __forceinline__ void fw_set_byte(uint4 &acc, u32 k, u32 c) {
  const u32 v = c << (8 * (k & 3u));
  const u32 w = k >> 2;
  acc.x |= w == 0 ? v : 0u; acc.y |= w == 1 ? v : 0u; acc.z |= w == 2 ? v : 0u; acc.w |= w == 3 ? v : 0u;
}
__device__ __forceinline__ u64 pow10u(u32 e) {
  u64 p = 1;
  for (u32 i = 0; i < e; ++i) p *= 10;
  return p;
}
// The record's output layout: fq2fa ">" ID "\n" Seq "\n"; anonymize "@" counter "\n" Seq "\n+\n"
// Qual "\n".  sp = {run-1 source offset, run-1 length, run-2 source offset, run-2 length} relative
// to the record (fq2fa: ID, Seq; anonymize: Seq, Qual); nd = the counter's digits (anonymize).
// Output bytes [lo, hi) of the chunk at o, the record's output starting at ra; false when a run's
// aligned window would leave the section (the caller then goes byte by byte).
__device__ __forceinline__ bool fw_record(const uint8_t *data, u64 n, int kind, u64 off, uint4 sp, u64 ctr, u32 nd,
                                          u64 dig, u64 ra, u64 o, uint4 &acc) {
  const u64 oe = o + 16;
  auto lit = [&](u64 p, u32 c) {
    if (p >= o && p < oe) fw_set_byte(acc, (u32)(p - o), c);
  };
  auto run = [&](u64 a, u64 src, u32 len) -> bool {
    const u64 b = a + len;
    if (!len || b <= o || a >= oe) return true;
    const u32 bl = (u32)((a > o ? a : o) - o), bh = (u32)((b < oe ? b : oe) - o);
    if (a > o && src < a - o) return false;  // the window would start before the section
    const u64 s = src + o - a, al = s & ~15ull;
    if (al + 32 > n) return false;
    const uint4 *q = reinterpret_cast<const uint4 *>(data + al);
    fw_or_masked(acc, fw_shift16(q[0], q[1], (u32)s & 15u), bl, bh);
    return true;
  };
  if (kind == FILT_FQ2FA) {
    lit(ra, '>');
    if (!run(ra + 1, off + sp.x, sp.y)) return false;
    lit(ra + 1 + sp.y, '\n');
    if (!run(ra + 2 + sp.y, off + sp.z, sp.w)) return false;
    lit(ra + 2 + sp.y + sp.w, '\n');
    return true;
  }
  // short literals as one 128-bit insert: "@" digits "\n" (the digits staged per record)
  typedef unsigned __int128 u128;
  auto ins = [&](u64 p, u128 v, u32 len) {
    if (p >= oe || p + len <= o) return;
    const i64 sh = (i64)p - (i64)o;  // (-len, 16)
    v = sh >= 0 ? v << (8 * sh) : v >> (8 * -sh);
    acc.x |= (u32)v; acc.y |= (u32)(v >> 32); acc.z |= (u32)(v >> 64); acc.w |= (u32)(v >> 96);
  };
  if (nd <= 8) {
    ins(ra, (u128)'@' | ((u128)dig << 8) | ((u128)'\n' << (8 * (nd + 1))), nd + 2);
  } else {
    lit(ra, '@');
    if (ra + 1 < oe && ra + 1 + nd > o) {  // more than 8 digits
      const u32 k0 = (u32)((ra + 1 > o ? ra + 1 : o) - (ra + 1)), k1 = (u32)((ra + 1 + nd < oe ? ra + 1 + nd : oe) - (ra + 1));
      u64 v = ctr;
      for (u32 k = nd; k > k1; --k) v /= 10;
      for (u32 k = k1; k > k0; --k) {
        lit(ra + k, '0' + (u32)(v % 10));
        v /= 10;
      }
    }
    lit(ra + 1 + nd, '\n');
  }
  if (!run(ra + 2 + nd, off + sp.x, sp.y)) return false;
  const u64 pl = ra + 2 + nd + sp.y;
  ins(pl, (u128)'\n' | ((u128)'+' << 8) | ((u128)'\n' << 16), 3);
  if (!run(pl + 3, off + sp.z, sp.w)) return false;
  lit(pl + 3 + sp.w, '\n');
  return true;
}
// byte rel of record r's output (the byte path)
__device__ u32 fw_byte(const uint8_t *data, int kind, u64 off, uint4 sp, u64 ctr, u32 nd, u64 rel) {
  if (kind == FILT_FQ2FA) {
    if (rel == 0) return '>';
    if (rel < 1 + sp.y) return data[off + sp.x + rel - 1];
    if (rel == 1 + sp.y) return '\n';
    if (rel < 2 + sp.y + sp.w) return data[off + sp.z + rel - 2 - sp.y];
    return '\n';
  }
  if (rel == 0) return '@';
  if (rel < 1 + nd) return '0' + (u32)((ctr / pow10u(nd - (u32)rel)) % 10);
  if (rel == 1 + nd) return '\n';
  const u64 p = 2 + nd + sp.y;
  if (rel < p) return data[off + sp.x + rel - 2 - nd];
  if (rel == p || rel == p + 2) return '\n';
  if (rel == p + 1) return '+';
  if (rel < p + 3 + sp.w) return data[off + sp.z + rel - p - 3];
  return '\n';
}
// the decimal digits of v (at most 8) as ASCII, the most significant in the low byte
__device__ __forceinline__ u64 fw_digits(u64 v, u32 nd) {
  u64 d = 0;
  if (nd > 8) return 0;
  u32 x = (u32)v;
  for (u32 k = nd; k-- > 0;) {
    d |= (u64)('0' + x % 10u) << (8 * k);
    x /= 10u;
  }
  return d;
}
__device__ __forceinline__ uint4 fw_spans(const u32 *spans, u64 r, int kind) {
  const u32 *q = spans + 6 * r;
  return kind == FILT_FQ2FA ? make_uint4(q[0], q[1], q[2], q[3]) : make_uint4(q[2], q[3], q[4], q[5]);
}
__device__ __forceinline__ void fw_store(uint8_t *p, const uint4 v) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(p));
}

template <int kind>  // the filter as a template argument: one code path per kernel
__global__ __launch_bounds__(FW_THREADS) void k_fq_write(const uint8_t *data, u64 n, const u64 *rows, const u32 *spans,
                                                         const u64 *outoff, const u64 *wfirst, u64 K, u64 total,
                                                         uint8_t *out) {
  __shared__ u64 s_out[FW_RECS + 1];
  __shared__ u64 s_off[FW_RECS];
  __shared__ uint4 s_sp[FW_RECS];
  __shared__ uint8_t s_nd[FW_RECS];  // the counter's digit count and digits (anonymize)
  __shared__ u64 s_dig[FW_RECS];
#if SIDX_FW_CMAP
  __shared__ uint16_t s_cmap[FW_BLOCK / 16];  // chunk c of the block -> its staged record (the one holding byte 16 c)
#endif
  const u64 nblocks = (total + FW_BLOCK - 1) / FW_BLOCK;
  const u64 b = blockIdx.x;
  if (b >= nblocks) return;
  const u64 blo = b * FW_BLOCK, bhi = blo + FW_BLOCK < total ? blo + FW_BLOCK : total;
  const u64 r0 = wfirst[b];
  const u64 rl = b + 1 < nblocks ? wfirst[b + 1] + 1 : K;
  const u64 nr = rl - r0 < K - r0 ? rl - r0 : K - r0;
  const u32 nb = (u32)(nr < FW_RECS ? nr : FW_RECS);
  for (u32 i = threadIdx.x; i < nb; i += FW_THREADS) {
    s_out[i] = outoff[r0 + i];
    s_off[i] = rows[2 * (r0 + i)];
    s_sp[i] = fw_spans(spans, r0 + i, kind);
    const u32 nd = ndigits(r0 + i + 1);
    s_nd[i] = (uint8_t)nd;
    s_dig[i] = kind == FILT_ANON_FQ ? fw_digits(r0 + i + 1, nd) : 0;
  }
  if (threadIdx.x == 0) s_out[nb] = r0 + nb < K ? outoff[r0 + nb] : total;
  __syncthreads();
  const u64 covered = s_out[nb];
#if SIDX_FW_CMAP
  // every chunk start of the block lies in exactly one staged record's output (they tile it):
  // each record marks the chunk starts it holds, replacing a binary search per chunk
  for (u32 j = threadIdx.x; j < nb; j += FW_THREADS) {
    const u64 a = s_out[j], e = s_out[j + 1];
    u64 o = a > blo ? (a - blo + 15) & ~15ull : 0;
    const u64 oe = (e < bhi ? e : bhi) - blo;
    for (; o < oe; o += 16) s_cmap[o >> 4] = (uint16_t)j;
  }
  __syncthreads();
#endif
  for (u64 o = blo + (u64)threadIdx.x * 16; o < bhi; o += (u64)FW_THREADS * 16) {
    const u64 oe = o + 16 < bhi ? o + 16 : bhi;
    bool slow = oe != o + 16 || oe > covered;
    uint4 acc = make_uint4(0, 0, 0, 0);
    if (!slow) {
#if SIDX_FW_CMAP
      const u32 lo = s_cmap[(o - blo) >> 4];  // last staged record with s_out <= o
#else
      u32 lo = 0, hi = nb;  // last staged record with s_out <= o
      while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (s_out[mid] <= o) lo = mid; else hi = mid;
      }
#endif
      for (u32 j = lo; j < nb && s_out[j] < oe; ++j) {
        const u64 ctr = r0 + j + 1;
        if (!fw_record(data, n, kind, s_off[j], s_sp[j], ctr, s_nd[j], s_dig[j], s_out[j], o, acc)) { slow = true; break; }
      }
    }
    if (!slow) {
      fw_store(out + o, acc);
      continue;
    }
    // byte by byte: records past the staged ones, windows at the section's ends, the last chunk
    u64 lo = 0, hi = K;  // last record with outoff <= o
    while (hi - lo > 1) {
      const u64 mid = (lo + hi) >> 1;
      if (outoff[mid] <= o) lo = mid; else hi = mid;
    }
    u64 r = lo;
    for (u64 p = o; p < oe; ++p) {
      while (r + 1 < K && outoff[r + 1] <= p) ++r;
      out[p] = (uint8_t)fw_byte(data, kind, rows[2 * r], fw_spans(spans, r, kind), r + 1, ndigits(r + 1), p - outoff[r]);
    }
  }
}

// fastq.go:50-132 Reader.Read for the record at s (one wave; WaveAcc scans cooperatively).
// Returns ST_OK / ST_END (no record: only blank lines or nothing left) or the error status.
template <class A>
__device__ u32 fastq_read_status(A &a, u64 s) {
  u64 e0, e1, e2, e3;
  u32 r;
  if (s >= a.end) return ST_END;                // ReadBytes -> ("", EOF)  (:56-66)
  r = a.find(C_NL, s, NOLIM, e0);
  if (r == FR_NONE) return ST_FQ_TRUNC;         // non-empty id line at EOF (:68-72)
  if (e0 == s) {                                // blank lines: skipped only up to EOF
    u64 y, z;
    r = a.find(C_NOTNL, s, NOLIM, y);
    if (r == FR_NONE) return ST_END;
    r = a.find(C_NL, y, NOLIM, z);
    return r == FR_FOUND ? ST_FQ_EMPTYLINES : ST_FQ_TRUNC;  // (:76-78) / (:68-72)
  }
  if (a.byte(s) != '@') return ST_FQ_NOAT;      // :79-81
  u64 ilo, ihi;
  trim_space(a, s + 1, e0 + 1, ilo, ihi);
  if (ihi == ilo) return ST_FQ_NOID;            // :83-87
  r = a.find(C_NL, e0 + 1, NOLIM, e1);            // :89-95
  if (r == FR_NONE) return ST_FQ_TRUNC;
  u64 slo, shi;
  trim_space(a, e0 + 1, e1 + 1, slo, shi);
  if (shi == slo) return ST_FQ_EMPTYSEQ;        // :96-100
  r = a.find(C_NL, e1 + 1, NOLIM, e2);            // :102-110
  if (r == FR_NONE) return ST_FQ_TRUNC;
  if (a.byte(e1 + 1) != '+') return ST_FQ_NOPLUS;
  u64 plo, phi;
  trim_space(a, e1 + 1, e2 + 1, plo, phi);      // :111-115
  if (phi - plo > 1) {
    if (ihi - ilo != phi - plo - 1) return ST_FQ_IDMISMATCH;
    for (u64 k = 0; k < ihi - ilo; ++k)
      if (a.byte(ilo + k) != a.byte(plo + 1 + k)) return ST_FQ_IDMISMATCH;
  }
  r = a.find(C_NL, e2 + 1, NOLIM, e3);            // :117-126, EOF tolerated
  const u64 qend = (r == FR_FOUND) ? e3 + 1 : a.end;
  u64 qlo, qhi;
  trim_space(a, e2 + 1, qend, qlo, qhi);
  if (shi - slo != qhi - qlo) return ST_FQ_LENMISMATCH;
  return ST_OK;
}

__global__ void k_fq_read_status(const uint8_t *data, u64 n, u64 s, u32 *out) {
  WaveAcc wa;
  wa.g = data; wa.end = n; wa.eof = 1; wa.lane = threadIdx.x & 63; wa.front = 0;
  const u32 st = fastq_read_status(wa, s);
  if (threadIdx.x == 0) *out = st;
}

// ---- anonymize over a FASTA section (fasta.go:40-88 Read, :216-218 Format) -----------------
// Read's sequences end at the FASTA boundaries (a '>' with a '\n' since the previous '>'): the
// same set GetReadOffset uses, but Read validates the whole read (TrimSpace(TrimRight(read, ">"))
// must hold a '\n', "Invalid fasta entry" without a snippet) where the index validates only
// the last piece.  When the record index builds without error its row starts are the boundaries
// (the host passes them with a stride of 2); otherwise they are found here without validation:
//   k_fa_last   per 16 KiB tile: the last '\n' and the last '>' (position + 1, 0: none)
//   (max scans over the tiles: the carry into every tile)
//   k_fa_bnd    per tile: every '>' whose last '\n' before it comes after its last '>' before
//               it; counts, positions kept in a per-tile slot when they fit
//   (scan) k_fa_bwrite: boundary positions B[0..m) in order.
// Sequence k < m is the read [start_k, B[k]) (start_0 = 0, else B[k-1]; leading '>'s are the
// lone ">" pieces Read skips); the last one (to EOF) comes back with io.EOF and is dropped.
constexpr u32 FSLOT = 64;

__device__ __forceinline__ void masks64(const uint8_t *d, u64 n, u64 a, u64 &mnl, u64 &mgt) {
  mnl = mgt = 0;
  if (a + 64 <= n) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = load16(d + a + 16 * k);
      mnl |= (u64)eq16(v, '\n') << (16 * k);
      mgt |= (u64)eq16(v, '>') << (16 * k);
    }
  } else {
    for (u64 i = 0; i < 64 && a + i < n; ++i) {
      const u32 c = d[a + i];
      mnl |= (u64)(c == '\n') << i;
      mgt |= (u64)(c == '>') << i;
    }
  }
}
__device__ __forceinline__ u64 last1(u64 m, u64 a) { return m ? a + 64 - __builtin_clzll(m) : 0; }  // pos + 1

__device__ __forceinline__ u64 wave_max(u64 v) {
  for (int o = 32; o > 0; o >>= 1) {
    const u64 y = __shfl_xor(v, o, 64);
    v = v > y ? v : y;
  }
  return v;
}

__global__ __launch_bounds__(256) void k_fa_last(const uint8_t *d, u64 n, u64 *lnl, u64 *lgt) {
  __shared__ u64 r[2][4];
  const u64 a = (u64)blockIdx.x * TILE + 64ull * threadIdx.x;
  u64 mnl = 0, mgt = 0;
  if (a < n) masks64(d, n, a, mnl, mgt);
  const u64 x = wave_max(last1(mnl, a)), y = wave_max(last1(mgt, a));
  if ((threadIdx.x & 63) == 0) { r[0][threadIdx.x >> 6] = x; r[1][threadIdx.x >> 6] = y; }
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 p = 0, q = 0;
    for (int i = 0; i < 4; ++i) { p = p > r[0][i] ? p : r[0][i]; q = q > r[1][i] ? q : r[1][i]; }
    lnl[blockIdx.x] = p;
    lgt[blockIdx.x] = q;
  }
}

// the boundary '>' bits of the thread's 64-byte word; cnl / cgt: last '\n' / '>' (pos + 1)
// before the word
__device__ __forceinline__ u64 bnd_bits(u64 mnl, u64 mgt, u64 a, u64 cnl, u64 cgt) {
  u64 out = 0, m = mgt;
  while (m) {
    const int i = __builtin_ctzll(m);
    m &= m - 1;
    const u64 below = (1ull << i) - 1;
    const u64 ln = (mnl & below) ? a + 64 - __builtin_clzll(mnl & below) : cnl;
    const u64 lg = (mgt & below) ? a + 64 - __builtin_clzll(mgt & below) : cgt;
    if (ln > lg) out |= 1ull << i;
  }
  return out;
}

// per-thread carries inside the tile: exclusive max-scan of the words' last positions
__device__ __forceinline__ void word_carry(u64 mnl, u64 mgt, u64 a, u64 tin_nl, u64 tin_gt, u64 &cnl, u64 &cgt,
                                           u64 (*ws)[4]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 x = last1(mnl, a), y = last1(mgt, a);
  for (int o = 1; o < 64; o <<= 1) {
    const u64 x2 = __shfl_up(x, o, 64), y2 = __shfl_up(y, o, 64);
    if (lane >= o) { x = x > x2 ? x : x2; y = y > y2 ? y : y2; }
  }
  if (lane == 63) { ws[0][wv] = x; ws[1][wv] = y; }
  __syncthreads();
  u64 px = __shfl_up(x, 1, 64), py = __shfl_up(y, 1, 64);
  if (lane == 0) { px = 0; py = 0; }
  cnl = tin_nl > px ? tin_nl : px;
  cgt = tin_gt > py ? tin_gt : py;
  for (int i = 0; i < wv; ++i) {
    cnl = cnl > ws[0][i] ? cnl : ws[0][i];
    cgt = cgt > ws[1][i] ? cgt : ws[1][i];
  }
}

__device__ __forceinline__ u64 block_excl_add(u64 c, u64 *ws, u64 &total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 x = c;
  for (int o = 1; o < 64; o <<= 1) {
    const u64 y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[wv] = x;
  __syncthreads();
  u64 off = x - c;
  for (int i = 0; i < wv; ++i) off += ws[i];
  total = ws[0] + ws[1] + ws[2] + ws[3];
  return off;
}

__global__ __launch_bounds__(256) void k_fa_bnd(const uint8_t *d, u64 n, const u64 *cin_nl, const u64 *cin_gt,
                                                u64 *tcnt, uint16_t *slot) {
  __shared__ u64 ws[2][4];
  __shared__ u64 wc[4];
  const u64 a = (u64)blockIdx.x * TILE + 64ull * threadIdx.x;
  u64 mnl = 0, mgt = 0;
  if (a < n) masks64(d, n, a, mnl, mgt);
  u64 cnl, cgt;
  word_carry(mnl, mgt, a, cin_nl[blockIdx.x], cin_gt[blockIdx.x], cnl, cgt, ws);
  u64 b = bnd_bits(mnl, mgt, a, cnl, cgt), total = 0;
  u64 off = block_excl_add((u64)__builtin_popcountll(b), wc, total);
  if (total <= FSLOT) {
    uint16_t *sl = slot + (u64)blockIdx.x * FSLOT;
    while (b) {
      sl[off++] = (uint16_t)(64u * threadIdx.x + (u32)__builtin_ctzll(b));
      b &= b - 1;
    }
  }
  if (threadIdx.x == 0) tcnt[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_fa_bwrite(const uint8_t *d, u64 n, const u64 *cin_nl, const u64 *cin_gt,
                                                   const u64 *tcnt, const u64 *toff, const uint16_t *slot, u64 *B) {
  __shared__ u64 ws[2][4];
  __shared__ u64 wc[4];
  const u64 c_t = tcnt[blockIdx.x], base = toff[blockIdx.x], t0 = (u64)blockIdx.x * TILE;
  if (c_t <= FSLOT) {
    if (threadIdx.x < c_t) B[base + threadIdx.x] = t0 + slot[(u64)blockIdx.x * FSLOT + threadIdx.x];
    return;
  }
  const u64 a = t0 + 64ull * threadIdx.x;
  u64 mnl = 0, mgt = 0;
  if (a < n) masks64(d, n, a, mnl, mgt);
  u64 cnl, cgt;
  word_carry(mnl, mgt, a, cin_nl[blockIdx.x], cin_gt[blockIdx.x], cnl, cgt, ws);
  u64 b = bnd_bits(mnl, mgt, a, cnl, cgt), total = 0;
  u64 off = base + block_excl_add((u64)__builtin_popcountll(b), wc, total);
  while (b) {
    B[off++] = a + (u64)__builtin_ctzll(b);
    b &= b - 1;
  }
}

// wave: first '\n' in [lo, hi) (hi if none) and the number of '\n' in [lo, hi).  Counts stay in
// the lanes until the end (one reduction), and the next 1 KiB step's load is in flight while this
// step is classified.
__device__ void wave_nl(const uint8_t *d, u64 n, u64 lo, u64 hi, int lane, u64 &first, u64 &count) {
  first = hi;
  auto ld = [&](u64 b) {
    if (b >= hi) return make_uint4(0, 0, 0, 0);
    return (b + 16 <= n) ? load16(d + b) : load16_partial(d, b, n);
  };
  u32 cl = 0;
  u64 b0 = lo & ~15ull;
  uint4 vn = ld(b0 + 16ull * lane);
  for (; b0 < hi; b0 += 64 * 16) {
    const u64 b = b0 + 16ull * lane;
    const uint4 v = vn;
    if (b0 + 1024 < hi) vn = ld(b + 1024);
    u32 m = 0;
    if (b < hi) {
      m = eq16(v, '\n');
      if (b < lo) m &= ~0u << (u32)(lo - b);
      if (b + 16 > hi) m &= (hi - b >= 16) ? ~0u : ((1u << (u32)(hi - b)) - 1u);
    }
    cl += (u32)__builtin_popcount(m);
    if (first == hi) {
      const u64 bal = __ballot(m != 0);
      if (bal) {
        const int L = __builtin_ctzll(bal);
        const u64 f = b + (m ? (u64)__builtin_ctz(m) : 0);
        first = (u64)__shfl((long long)f, L, 64);
      }
    }
  }
  u64 c = cl;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  count = c;
}

// one wave per sequence k < m: the body span (after the label's '\n', to the trimmed end),
// the output length ">" counter "\n" body-without-'\n' "\n", Read's validity
#ifndef SIDX_FAS_WPE
#define SIDX_FAS_WPE 0  // k_fa_anon_spans: amdgpu_waves_per_eu for variant builds (8 spilled: slower)
#endif
#if SIDX_FAS_WPE > 0
#define SIDX_FAS_ATTR __attribute__((amdgpu_waves_per_eu(SIDX_FAS_WPE)))
#else
#define SIDX_FAS_ATTR
#endif
__global__ __launch_bounds__(256) SIDX_FAS_ATTR void k_fa_anon_spans(const uint8_t *d, u64 n, const u64 *B, u64 bstride, u64 m,
                                                       u64 *bspan, u64 *outlen, u64 *firstbad) {
  const int lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * (blockDim.x / 64);
  for (u64 k = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < m; k += nw) {
    u64 s = k ? B[(k - 1) * bstride] : 0;
    const u64 e0 = B[k * bstride];
    // the common sequence in one round of loads (lanes 0-3: its first two and last two bytes):
    // '>' then a printable ASCII byte other than '>', and a printable last byte or a space after
    // one -- the serial '>' and TrimSpace loops below then stop at once (they cost ~8 dependent
    // round trips per sequence)
    bool fast = false;
    u64 lo = 0, hi = 0;
    if (e0 >= s + 4) {
      const u64 at = lane == 0 ? s : lane == 1 ? s + 1 : lane == 2 ? e0 - 1 : e0 - 2;
      const u32 cb = lane < 4 ? (u32)d[at] : 0u;
      const u32 a0 = (u32)__shfl((int)cb, 0, 64), a1 = (u32)__shfl((int)cb, 1, 64);
      const u32 z1 = (u32)__shfl((int)cb, 2, 64), z2 = (u32)__shfl((int)cb, 3, 64);
      auto ok = [](u32 c) { return c < 0x80 && !ascii_space(c); };
      if (a0 == '>' && a1 != '>' && ok(a1) && z1 != '>') {
        if (ok(z1)) { fast = true; lo = s + 1; hi = e0; }
        else if (z1 < 0x80 && ascii_space(z1) && ok(z2)) { fast = true; lo = s + 1; hi = e0 - 1; }
      }
    }
    if (!fast) {
      if (s < e0 && d[s] == '>') {  // the lone ">" pieces (fasta.go:58-64)
        ++s;
        while (s < e0 && d[s] == '>') ++s;
      }
      u64 e = e0;  // TrimRight(read, ">") of [s, e0]: the boundary '>' and any before it
      while (e > s && d[e - 1] == '>') --e;
      if (lane == 0) {
        const GAcc ga{d};
        trim_space(ga, s, e, lo, hi);
      }
      lo = (u64)__shfl((long long)lo, 0, 64);
      hi = (u64)__shfl((long long)hi, 0, 64);
    }
    u64 f, c;
    wave_nl(d, n, lo, hi, lane, f, c);
    if (lane == 0) {
      if (f >= hi) {
        atomicMin((unsigned long long *)firstbad, (unsigned long long)k);
        outlen[k] = 0;
      } else {
        bspan[2 * k] = f + 1;
        bspan[2 * k + 1] = hi;
        outlen[k] = 1 + ndigits(k + 1) + 1 + (hi - f - 1 - (c - 1)) + 1;
      }
    }
  }
}

// one wave per sequence: ">" counter "\n", the body with its '\n's dropped, "\n"
// Each wave assembles its sequence's output in an LDS window aligned to the output's 16-byte
// blocks and stores every block it owns whole as one 16-byte store; only the blocks shared with the
// neighbouring sequences' outputs (at most one at each end) go byte by byte.  Byte stores to
// global memory (the round-2 writer) ran 14-15 ms per 10 GiB section.
#ifndef SIDX_FA_STEPK
#define SIDX_FA_STEPK 2  // k_fa_anon_write: KiB of input per step (1 to 4)
#endif
#ifndef SIDX_FA_PREFETCH
#define SIDX_FA_PREFETCH 0  // k_fa_anon_write: 1 = the next step's loads in flight during this one
#endif
// window bytes per wave: < 16 carried + a 22-byte header + one step
constexpr u32 FA_STG = 64 + 1024 * SIDX_FA_STEPK;
#ifndef SIDX_FA_ABL
#define SIDX_FA_ABL 0  // profiling ablation (variant builds): 1 = k_fa_anon_write stores nothing
#endif
__device__ __forceinline__ void fa_flush(uint8_t *out, const uint8_t *stg, u64 blk, u64 end, u64 obase, u64 cur,
                                         int lane) {
  if (SIDX_FA_ABL == 1) return;
  // blocks [blk, end) of the window (end 16-aligned): whole when every byte is this sequence's
  for (u64 b = blk + 16 * (u64)lane; b < end; b += 1024) {
    const u32 r = (u32)(b - blk);
    if (b >= obase && b + 16 <= cur) {
      fw_store(out + b, *reinterpret_cast<const uint4 *>(stg + r));
    } else {
      for (u32 t = 0; t < 16; ++t)
        if (b + t >= obase && b + t < cur) out[b + t] = stg[r + t];
    }
  }
}
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// A step is SK 1 KiB chunks; chunk j's lane L holds input bytes [p + 1024 j + 16 L, +16).  The
// kept-byte counts of the SK chunks are packed in 16-bit fields of one 64-bit value (a chunk keeps
// at most 1024 bytes), so one wave scan places every lane's bytes of every chunk.  A sequence
// (~1.7 KB) is one step: its loads all go out in one round trip, and there is one flush per step.
#ifndef SIDX_FA_WPE
#define SIDX_FA_WPE 8  // k_fa_anon_write: amdgpu_waves_per_eu (its register budget; 0 = none)
#endif
#if SIDX_FA_WPE > 0
#define SIDX_FA_ATTR __attribute__((amdgpu_waves_per_eu(SIDX_FA_WPE)))
#else
#define SIDX_FA_ATTR
#endif
__global__ __launch_bounds__(256) SIDX_FA_ATTR void k_fa_anon_write(const uint8_t *d, u64 n, const u64 *bspan, const u64 *outoff,
                                                       u64 K, uint8_t *out) {
  constexpr int SK = SIDX_FA_STEPK;
  static_assert(SK >= 1 && SK <= 4, "16-bit count fields: at most four chunks per step");
  constexpr u64 STEP = 1024ull * SK;
  __shared__ __attribute__((aligned(16))) uint8_t stg_all[4][FA_STG];
  const int lane = threadIdx.x & 63;
  uint8_t *stg = stg_all[threadIdx.x >> 6];
  const u64 nw = (u64)gridDim.x * (blockDim.x / 64);
  for (u64 k = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < K; k += nw) {
    const u64 obase = outoff[k];
    u64 blk = obase & ~15ull;  // output byte of stg[0]
    const u64 id = k + 1;
    const u32 nd = ndigits(id);
    const u32 h0 = (u32)(obase - blk);
    if (lane == 0) stg[h0] = '>';
    if (lane < (int)nd) {
      u64 v = id;
      for (u32 q = 0; q < nd - 1 - (u32)lane; ++q) v /= 10;
      stg[h0 + 1 + lane] = (uint8_t)('0' + v % 10);
    }
    if (lane == 0) stg[h0 + 1 + nd] = '\n';
    u64 cur = obase + 2 + nd;  // the next output byte
    const u64 lo = bspan[2 * k], hi = bspan[2 * k + 1];
    // a sequence (~1.7 KB) is one 4 KiB step: its loads all go out together
    auto chunk_load = [&](u64 q) {
      if (q >= hi) return make_uint4(0, 0, 0, 0);
      return q + 16 <= n ? load16(d + q) : load16_partial(d, q, n);  // q 16-aligned, below hi <= n
    };
    uint4 vn[SIDX_FA_PREFETCH ? SK : 1];
    if (SIDX_FA_PREFETCH) {
#pragma unroll
      for (int j = 0; j < SK; ++j) vn[j] = chunk_load((lo & ~15ull) + 1024ull * j + 16 * (u64)lane);
    }
    for (u64 p = lo & ~15ull; p < hi; p += STEP) {
      uint4 v[SK];
      u32 keep[SK];
      u64 c = 0;
#pragma unroll
      for (int j = 0; j < SK; ++j) {
        const u64 q = p + 1024ull * j + 16 * (u64)lane;
        if (SIDX_FA_PREFETCH) {
          v[j] = vn[j];
          if (p + STEP < hi) vn[j] = chunk_load(q + STEP);
        } else {
          v[j] = chunk_load(q);
        }
        keep[j] = 0;
        if (q < hi) {
          keep[j] = ~eq16(v[j], '\n') & 0xFFFFu;
          if (q < lo) keep[j] &= 0xFFFFu << (u32)(lo - q);
          if (hi - q < 16) keep[j] &= (1u << (u32)(hi - q)) - 1u;
        }
        c |= (u64)__builtin_popcount(keep[j]) << (16 * j);
      }
      u64 x = c;  // inclusive scan of the packed counts over the wave
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const u64 y = (u64)__shfl_up((long long)x, dd, 64);
        if (lane >= dd) x += y;
      }
      const u64 tot = (u64)__shfl((long long)x, 63, 64);
      u32 base = (u32)(cur - blk);
#pragma unroll
      for (int j = 0; j < SK; ++j) {
        u32 r = base + ((u32)((x - c) >> (16 * j)) & 0xFFFFu);
        const uint4 w = v[j];
        for (u32 m = keep[j]; m; m &= m - 1) {
          const u32 i = (u32)__builtin_ctz(m);
          const u32 wd = (i >> 2) == 0 ? w.x : (i >> 2) == 1 ? w.y : (i >> 2) == 2 ? w.z : w.w;
          stg[r++] = (uint8_t)(wd >> (8 * (i & 3u)));
        }
        base += (u32)(tot >> (16 * j)) & 0xFFFFu;
      }
      cur = blk + base;
      wave_sync_lds();
      // the complete blocks out; the partial last block moves to the window's front
      const u64 fend = cur & ~15ull;
      fa_flush(out, stg, blk, fend, obase, cur, lane);
      const u32 t0 = (u32)(fend - blk);
      const uint8_t tb = lane < 16 ? stg[t0 + lane] : 0;
      wave_sync_lds();
      if (lane < 16) stg[lane] = tb;
      blk = fend;
      wave_sync_lds();
    }
    if (lane == 0) stg[cur - blk] = '\n';
    ++cur;
    wave_sync_lds();
    fa_flush(out, stg, blk, (cur + 15) & ~15ull, obase, cur, lane);
    wave_sync_lds();
  }
}

// ---- anonymize over a SAM section (sam.go:44-81 Read, :146-148 Format) ----------------------
// Lines from the line index; a line without '\n' (the last) is io.EOF and ends the stream.
// Per line (one wave): TrimSpace; blank and '@' lines are skipped; fewer than 11 tab-separated
// fields is Read's error; otherwise the trimmed line + "\n".
__global__ __launch_bounds__(256) void k_sam_anon_spans(const uint8_t *d, u64 n, const u64 *rows, u64 K, u64 *span,
                                                        u64 *outlen, u64 *firstbad, u64 *firsteof) {
  const int lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * (blockDim.x / 64);
  for (u64 k = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < K; k += nw) {
    const u64 off = rows[2 * k], len = rows[2 * k + 1];
    if (len == 0 || d[off + len - 1] != '\n') {  // ReadBytes' io.EOF
      if (lane == 0) { atomicMin((unsigned long long *)firsteof, (unsigned long long)k); outlen[k] = 0; }
      continue;
    }
    u64 lo = 0, hi = 0;
    if (lane == 0) {
      const GAcc ga{d};
      trim_space(ga, off, off + len, lo, hi);
    }
    lo = (u64)__shfl((long long)lo, 0, 64);
    hi = (u64)__shfl((long long)hi, 0, 64);
    if (hi == lo || d[lo] == '@') {
      if (lane == 0) outlen[k] = 0;
      continue;
    }
    u64 tabs = 0;
    for (u64 p = lo + (u64)lane; p < hi; p += 64) tabs += d[p] == '\t';
    for (int o = 32; o > 0; o >>= 1) tabs += __shfl_xor(tabs, o, 64);
    if (lane == 0) {
      if (tabs + 1 < 11) {
        atomicMin((unsigned long long *)firstbad, (unsigned long long)k);
        outlen[k] = 0;
      } else {
        span[2 * k] = lo;
        span[2 * k + 1] = hi;
        outlen[k] = hi - lo + 1;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_sam_anon_write(const uint8_t *d, const u64 *span, const u64 *outlen,
                                                        const u64 *outoff, u64 K, uint8_t *out, u64 *count) {
  const int lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * (blockDim.x / 64);
  u64 mine = 0;
  for (u64 k = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < K; k += nw) {
    if (!outlen[k]) continue;
    const u64 lo = span[2 * k], hi = span[2 * k + 1];
    uint8_t *o = out + outoff[k];
    for (u64 p = (u64)lane; p < hi - lo; p += 64) o[p] = d[lo + p];
    if (lane == 0) { o[hi - lo] = '\n'; ++mine; }
  }
  if (lane == 0 && mine) atomicAdd((unsigned long long *)count, (unsigned long long)mine);
}

}  // namespace sidx

using namespace sidx;

extern "C" hipError_t sidx_filter_spans(const uint8_t *data, u64 n, const u64 *rows, u64 K, int kind, u32 *spans,
                                        u64 *outlen, u64 *firstbad, hipStream_t s) {
  if (K) hipLaunchKernelGGL(k_fq_spans, dim3((u32)((K + 255) / 256)), dim3(256), 0, s, data, n, rows, K, kind, spans,
                            outlen, firstbad);
  return hipGetLastError();
}

// wfirst: total / FW_BLOCK + 1 words (the first record of every output block)
extern "C" hipError_t sidx_filter_write(const uint8_t *data, u64 n, const u64 *rows, const u32 *spans, const u64 *outlen,
                                        const u64 *outoff, u64 K, u64 total, int kind, u64 *wfirst, uint8_t *out,
                                        hipStream_t s) {
  if (!K || !total) return hipSuccess;
  const u64 nblocks = (total + FW_BLOCK - 1) / FW_BLOCK;
  hipLaunchKernelGGL(k_fw_plan, dim3((u32)((K + 255) / 256)), dim3(256), 0, s, outoff, outlen, K, nblocks, wfirst);
  if (kind == FILT_FQ2FA)
    hipLaunchKernelGGL(k_fq_write<FILT_FQ2FA>, dim3((u32)nblocks), dim3(FW_THREADS), 0, s, data, n, rows, spans, outoff,
                       wfirst, K, total, out);
  else
    hipLaunchKernelGGL(k_fq_write<FILT_ANON_FQ>, dim3((u32)nblocks), dim3(FW_THREADS), 0, s, data, n, rows, spans, outoff,
                       wfirst, K, total, out);
  return hipGetLastError();
}
extern "C" u64 sidx_filter_block() { return FW_BLOCK; }

extern "C" u32 sidx_fa_slot() { return FSLOT; }
// FASTA boundaries (anonymize): lnl / lgt / cnl / cgt / tcnt / toff: ntile = ceil(n / TILE)
// words each; slot: ntile * FSLOT u16s; tmp: the max / sum scans (null -> size query, the
// larger of the two)
extern "C" hipError_t sidx_fa_bnd_count(const uint8_t *d, u64 n, u64 *lnl, u64 *lgt, u64 *cnl, u64 *cgt, u64 *tcnt,
                                        u64 *toff, uint16_t *slot, void *tmp, size_t *tmp_bytes, hipStream_t s) {
  const u64 nt = (n + TILE - 1) / TILE;
  if (!tmp) return dscan::run<u64, dscan::Max, true>(nullptr, tmp_bytes, lnl, cnl, nt ? nt : 1, s);  // (sum: same size)
  if (!nt) return hipSuccess;
  hipLaunchKernelGGL(k_fa_last, dim3((u32)nt), dim3(256), 0, s, d, n, lnl, lgt);
  hipError_t e = dscan::run<u64, dscan::Max, true>(tmp, tmp_bytes, lnl, cnl, nt, s);
  if (e == hipSuccess) e = dscan::run<u64, dscan::Max, true>(tmp, tmp_bytes, lgt, cgt, nt, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fa_bnd, dim3((u32)nt), dim3(256), 0, s, d, n, cnl, cgt, tcnt, slot);
  return dscan::run<u64, dscan::Sum, true>(tmp, tmp_bytes, tcnt, toff, nt, s);
}
extern "C" hipError_t sidx_fa_bnd_write(const uint8_t *d, u64 n, const u64 *cnl, const u64 *cgt, const u64 *tcnt,
                                        const u64 *toff, const uint16_t *slot, u64 *B, hipStream_t s) {
  const u64 nt = (n + TILE - 1) / TILE;
  if (nt) hipLaunchKernelGGL(k_fa_bwrite, dim3((u32)nt), dim3(256), 0, s, d, n, cnl, cgt, tcnt, toff, slot, B);
  return hipGetLastError();
}
static u32 wave_grid(u64 K) { return (u32)((K + 3) / 4 < 65536 ? (K + 3) / 4 : 65536); }
extern "C" hipError_t sidx_fa_anon_spans(const uint8_t *d, u64 n, const u64 *B, u64 bstride, u64 m, u64 *bspan, u64 *outlen,
                                         u64 *firstbad, hipStream_t s) {
  if (m) hipLaunchKernelGGL(k_fa_anon_spans, dim3(wave_grid(m)), dim3(256), 0, s, d, n, B, bstride, m, bspan, outlen, firstbad);
  return hipGetLastError();
}
extern "C" hipError_t sidx_fa_anon_write(const uint8_t *d, u64 n, const u64 *bspan, const u64 *outoff, u64 K,
                                         uint8_t *out, hipStream_t s) {
  if (K) hipLaunchKernelGGL(k_fa_anon_write, dim3(wave_grid(K)), dim3(256), 0, s, d, n, bspan, outoff, K, out);
  return hipGetLastError();
}
extern "C" hipError_t sidx_sam_anon_spans(const uint8_t *d, u64 n, const u64 *rows, u64 K, u64 *span, u64 *outlen,
                                          u64 *firstbad, u64 *firsteof, hipStream_t s) {
  if (K) hipLaunchKernelGGL(k_sam_anon_spans, dim3(wave_grid(K)), dim3(256), 0, s, d, n, rows, K, span, outlen,
                            firstbad, firsteof);
  return hipGetLastError();
}
extern "C" hipError_t sidx_sam_anon_write(const uint8_t *d, const u64 *span, const u64 *outlen, const u64 *outoff,
                                          u64 K, uint8_t *out, u64 *count, hipStream_t s) {
  if (K) hipLaunchKernelGGL(k_sam_anon_write, dim3(wave_grid(K)), dim3(256), 0, s, d, span, outlen, outoff, K, out,
                            count);
  return hipGetLastError();
}

extern "C" hipError_t sidx_filter_read_status(const uint8_t *data, u64 n, u64 start, u32 *out, hipStream_t s) {
  hipLaunchKernelGGL(k_fq_read_status, dim3(1), dim3(64), 0, s, data, n, start, out);
  return hipGetLastError();
}
