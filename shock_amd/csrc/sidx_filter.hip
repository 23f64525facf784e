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
// Pipeline: record index (k_pipe) -> k_fq_spans (one lane per record: its three inner line
// ends, the trimmed ID / sequence / quality spans, the output length, Read's extra checks)
// -> exclusive scan of the output lengths -> k_fq_write (one wave per record, lanes copy
// 64 bytes per step).  The terminal record (the index's first error) is re-checked with
// Read's order by k_fq_read_status (one wave).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

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

__device__ __forceinline__ u32 ndigits(u64 v) {
  u32 d = 1;
  while (v >= 10) { v /= 10; ++d; }
  return d;
}

// Per record: spans relative to the record start (id_lo, id_len, seq_lo, seq_len, qual_lo,
// qual_len), the output length and Read's status for the checks the index did not make.
__global__ __launch_bounds__(256) void k_fq_spans(const uint8_t *data, u64 n, const u64 *rows, u64 K, int kind,
                                                  u32 *spans, u64 *outlen, u64 *firstbad) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K) return;
  const u64 off = rows[2 * i], len = rows[2 * i + 1], end = off + len;
  // the first three '\n' of the record (the index guarantees they exist inside it)
  u64 e0 = 0, e1 = 0, e2 = 0;
  u32 found = 0;
  for (u64 b = off & ~15ull; b < end && found < 3; b += 16) {
    const uint4 v = (b + 16 <= n) ? load16(data + b) : load16_partial(data, b, n);
    u32 m = eq16(v, '\n');
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
  const GAcc a{data};
  u64 ilo, ihi, slo, shi, qlo, qhi;
  trim_space(a, off + 1, e0 + 1, ilo, ihi);  // seqId = TrimSpace(seqId[1:])  (fastq.go:83)
  trim_space(a, e0 + 1, e1 + 1, slo, shi);   // seqBody (:96)
  trim_space(a, e2 + 1, end, qlo, qhi);      // qualBody (:123)
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

// lanes copy src[0, len) to dst[0, len), 64 bytes per step
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, u64 len, int lane) {
  for (u64 k = (u64)lane; k < len; k += 64) dst[k] = src[k];
}

// One wave per record (grid-stride): the formatted record at outoff[i].
__global__ __launch_bounds__(256) void k_fq_write(const uint8_t *data, const u64 *rows, const u32 *spans,
                                                  const u64 *outoff, u64 K, int kind, uint8_t *out) {
  const int lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * (blockDim.x / 64);
  for (u64 i = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < K; i += nw) {
    const u64 off = rows[2 * i];
    const u32 *sp = spans + 6 * i;
    uint8_t *o = out + outoff[i];
    if (kind == FILT_FQ2FA) {  // ">" ID "\n" Seq "\n"
      if (lane == 0) o[0] = '>';
      wave_copy(o + 1, data + off + sp[0], sp[1], lane);
      o += 1 + sp[1];
      if (lane == 0) o[0] = '\n';
      wave_copy(o + 1, data + off + sp[2], sp[3], lane);
      if (lane == 0) o[1 + sp[3]] = '\n';
    } else {  // "@" counter "\n" Seq "\n+\n" Qual "\n"
      const u64 id = i + 1;
      const u32 nd = ndigits(id);
      if (lane == 0) o[0] = '@';
      if (lane < (int)nd) {
        u64 v = id;
        for (u32 k = 0; k < nd - 1 - (u32)lane; ++k) v /= 10;
        o[1 + lane] = (uint8_t)('0' + v % 10);
      }
      o += 1 + nd;
      if (lane == 0) o[0] = '\n';
      wave_copy(o + 1, data + off + sp[2], sp[3], lane);
      o += 1 + sp[3];
      if (lane == 0) { o[0] = '\n'; o[1] = '+'; o[2] = '\n'; }
      wave_copy(o + 3, data + off + sp[4], sp[5], lane);
      if (lane == 0) o[3 + sp[5]] = '\n';
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

}  // namespace sidx

using namespace sidx;

extern "C" hipError_t sidx_filter_spans(const uint8_t *data, u64 n, const u64 *rows, u64 K, int kind, u32 *spans,
                                        u64 *outlen, u64 *firstbad, hipStream_t s) {
  if (K) hipLaunchKernelGGL(k_fq_spans, dim3((u32)((K + 255) / 256)), dim3(256), 0, s, data, n, rows, K, kind, spans,
                            outlen, firstbad);
  return hipGetLastError();
}

extern "C" hipError_t sidx_filter_write(const uint8_t *data, const u64 *rows, const u32 *spans, const u64 *outoff,
                                        u64 K, int kind, uint8_t *out, hipStream_t s) {
  if (K) {
    const u64 blocks = (K + 3) / 4 < 65536 ? (K + 3) / 4 : 65536;  // 4 waves per block, grid-stride
    hipLaunchKernelGGL(k_fq_write, dim3((u32)blocks), dim3(256), 0, s, data, rows, spans, outoff, K, kind, out);
  }
  return hipGetLastError();
}

extern "C" hipError_t sidx_filter_read_status(const uint8_t *data, u64 n, u64 start, u32 *out, hipStream_t s) {
  hipLaunchKernelGGL(k_fq_read_status, dim3(1), dim3(64), 0, s, data, n, start, out);
  return hipGetLastError();
}
