// sidx_kernels.hip -- gfx950 kernels of the MI355X record indexer.
//
//   k_detect       format detection (multi.go:43-62), one workgroup, <= 32 KiB inspected
//   k_fq_tiles     FASTQ tile pass: LDS-DMA staged 16 KiB tiles, '\n' masks, the record phase
//                  read off the tile, records certified from LDS into a provisional row table
//   k_fa_tiles     FASTA tile pass (the FastaMonoid boundaries, pieces validated from LDS)
//   k_line_tiles   line tile pass ('\n' positions per tile)
//   k_scan_excl<M> device-wide exclusive scan of the per-tile aggregates (decoupled look-back)
//   k_*_place      final 16-byte rows at their global record numbers; k_fixup / k_fa_fixup
//                  re-validate from global memory what a tile could not settle
//   k_tile_agg<F> + k_index1<F>  the two-pass build (SAM, FASTA / line slabs, re-runs)
//   k_finalize   folds the slab's terminal state + first-bad key into a DevResult
//
// Reference semantics restated (paths relative to /root/reference/shock-server/):
//   record driver  node/file/index/record.go:34-90     line driver node/file/index/line.go:33-85
//   FASTQ          node/file/format/fastq/fastq.go:134-213
//   FASTA          node/file/format/fasta/fasta.go:93-140
//   SAM            node/file/format/sam/sam.go:83-98
//   line           node/file/format/line/line.go:37-45
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <atomic>

#include "sidx_common.hpp"
#include "sidx_device.hpp"
#include <stdlib.h>
#include <string.h>

namespace sidx {

constexpr u64 INF = ~0ull;

// Diagnostics (phase timing, ablation knobs) exist only in the SIDX_DIAG=1 variant build
// (make variant V=diag VFLAGS=-DSIDX_DIAG=1): runtime-uniform flags in the production
// kernels would make the compiler clone the hot loops once per flag combination.
#ifndef SIDX_DIAG
#define SIDX_DIAG 0
#endif
__device__ __forceinline__ u32 dbg(const SlabParams &p) { return SIDX_DIAG ? p.debug : 0u; }
__device__ __forceinline__ u64 *tmg(const SlabParams &p) { return SIDX_DIAG ? p.timing : nullptr; }

// ====================================================================================
// Validators (one record; templated on the accessor).  Return ST_*; set len on ST_OK.
// ====================================================================================
__device__ __forceinline__ u32 fr_to_st(u32 r) { return r == FR_DEFER ? ST_DEFER : ST_NEEDMORE; }

// fastq.go:134-213 for the group (record) starting at s.
template <class A>
__device__ u32 fastq_record(A &a, u64 s, u64 &len) {
  u64 e0, e1, e2, e3;
  u32 r;
  if (s >= a.end) return a.eof ? ST_END : ST_NEEDMORE;  // id line absent: (0, EOF)
  r = a.find(C_NL, s, INF, e0);
  if (r >= FR_DEFER) return fr_to_st(r);
  if (r == FR_NONE) return ST_FQ_TRUNC;  // non-empty id line without '\n' at EOF (:154-156)
  if (e0 == s) {                          // blank line where an id line is due (:143-152)
    // a group whose 4 preceding bytes are all '\n' follows another blank group: only the
    // first group of a blank run can be the terminating one (keeps the scans linear)
    if ((s >= 4 || a.front >= 4) && a.byte(s - 1) == '\n' && a.byte(s - 2) == '\n' &&
        a.byte(s - 3) == '\n' && a.byte(s - 4) == '\n')
      return ST_DONTCARE;
    u64 y, z;
    r = a.find(C_NOTNL, s, INF, y);
    if (r >= FR_DEFER) return fr_to_st(r);
    if (r == FR_NONE) return ST_END;  // only blank lines up to EOF (:154-158, len 0)
    r = a.find(C_NL, y, INF, z);
    if (r >= FR_DEFER) return fr_to_st(r);
    return r == FR_FOUND ? ST_FQ_EMPTYLINES : ST_FQ_TRUNC;  // (:161-163) / (:154-156)
  }
  if (a.byte(s) != '@') return ST_FQ_NOAT;   // :164-166
  if (e0 - s == 1) return ST_FQ_NOID;        // "@\n" (:167-169)
  r = a.find(C_NL, e0 + 1, INF, e1);         // sequence line (:173-182)
  if (r >= FR_DEFER) return fr_to_st(r);
  if (r == FR_NONE) return ST_FQ_TRUNC;
  if (e1 == e0 + 1) return ST_FQ_EMPTYSEQ;
  r = a.find(C_NL, e1 + 1, INF, e2);         // plus line (:185-199)
  if (r >= FR_DEFER) return fr_to_st(r);
  if (r == FR_NONE) return ST_FQ_TRUNC;
  if (a.byte(e1 + 1) != '+') return ST_FQ_NOPLUS;
  u64 plo, phi;
  trim_space(a, e1 + 1, e2 + 1, plo, phi);
  if (phi - plo > 1) {
    u64 ilo, ihi;
    trim_space(a, s + 1, e0 + 1, ilo, ihi);
    if (ihi - ilo != phi - plo - 1) return ST_FQ_IDMISMATCH;
    for (u64 k = 0; k < ihi - ilo; ++k)
      if (a.byte(ilo + k) != a.byte(plo + 1 + k)) return ST_FQ_IDMISMATCH;
  }
  r = a.find(C_NL, e2 + 1, INF, e3);         // quality line (:202-209), EOF tolerated
  if (r >= FR_DEFER) return fr_to_st(r);
  const u64 qend = (r == FR_FOUND) ? e3 + 1 : a.end;
  u64 slo, shi, qlo, qhi;
  trim_space(a, e0 + 1, e1 + 1, slo, shi);
  trim_space(a, e2 + 1, qend, qlo, qhi);
  if (shi - slo != qhi - qlo) return ST_FQ_LENMISMATCH;
  len = qend - s;                            // :211
  return ST_OK;
}

// fasta.go:111-121: piece [lo, hi) (its '>' excluded) is valid iff TrimSpace of it holds a
// '\n' (Split(...)[1:] joined non-empty).
template <class A>
__device__ u32 fasta_piece_ok(A &a, u64 lo, u64 hi, bool &ok) {
  u64 tl, th, q;
  trim_space(a, lo, hi, tl, th);
  if (th <= tl) { ok = false; return FR_FOUND; }
  const u32 r = a.find(C_NL, tl, th, q);
  if (r >= FR_DEFER) return r;
  ok = (r == FR_FOUND);
  return FR_FOUND;
}

// fasta.go:93-140 for the record starting at rs; the scan for '>' starts at lo (one past
// the '>' that precedes it, or 0 for a file not starting with '>').
template <class A>
__device__ u32 fasta_record(A &a, u64 rs, u64 lo, u64 &len, u64 &epos, u64 &elen) {
  if (rs >= a.end) return a.eof ? ST_ABSENT : ST_NEEDMORE;
  for (;;) {
    u64 g, q;
    u32 r = a.find(C_X, lo, INF, g);
    if (r >= FR_DEFER) return fr_to_st(r);
    if (r == FR_NONE) {  // EOF piece [lo, end): validated iff len > 1 && holds '\n' (:111)
      if (a.end - lo > 1) {
        r = a.find(C_NL, lo, a.end, q);
        if (r >= FR_DEFER) return fr_to_st(r);
        if (r == FR_FOUND) {
          bool ok;
          r = fasta_piece_ok(a, lo, a.end, ok);
          if (r >= FR_DEFER) return fr_to_st(r);
          if (!ok) { epos = lo; elen = a.end - lo; return ST_FA_INVALID; }
        }
      }
      len = a.end - rs;  // :123-125
      return ST_OK;
    }
    r = a.find(C_NL, lo, g, q);  // '\n' since the previous '>' -> record boundary
    if (r >= FR_DEFER) return fr_to_st(r);
    if (r == FR_FOUND) {
      bool ok;
      r = fasta_piece_ok(a, lo, g, ok);
      if (r >= FR_DEFER) return fr_to_st(r);
      if (!ok) { epos = lo; elen = g + 1 - lo; return ST_FA_INVALID; }  // piece incl. '>'
      len = g - rs;  // :126-128 (UnreadByte)
      return ST_OK;
    }
    lo = g + 1;  // embedded '>' (:131-132)
  }
}

// sam.go:83-98 for the record starting at s.
template <class A>
__device__ u32 sam_record(A &a, u64 s, u64 &len) {
  if (s >= a.end) return a.eof ? ST_ABSENT : ST_NEEDMORE;
  u64 p = s;
  for (;;) {
    u64 q;
    const u32 r = a.find(C_NL, p, INF, q);
    if (r >= FR_DEFER) return fr_to_st(r);
    if (r == FR_NONE) { len = a.end - s; return ST_OK; }  // last line / leftover
    if (q > p && a.byte(p) != '@') { len = q + 1 - s; return ST_OK; }  // terminator line
    p = q + 1;
    if (p >= a.end) {
      if (!a.eof) return ST_NEEDMORE;
      len = a.end - s;
      return ST_OK;
    }
  }
}

// line.go:37-45 for the line starting at s (always a row, possibly empty at EOF).
template <class A>
__device__ u32 line_record(A &a, u64 s, u64 &len) {
  u64 q;
  const u32 r = a.find(C_NL, s, INF, q);
  if (r >= FR_DEFER) return fr_to_st(r);
  len = (r == FR_FOUND) ? q + 1 - s : a.end - s;
  return ST_OK;
}

// ====================================================================================
// Format traits
// ====================================================================================
template <int F> struct Traits;
template <> struct Traits<F_FASTQ> { typedef CountMonoid M; static constexpr bool kX = false; static constexpr u32 xc = 0; };
template <> struct Traits<F_LINE>  { typedef CountMonoid M; static constexpr bool kX = false; static constexpr u32 xc = 0; };
template <> struct Traits<F_FASTA> { typedef FastaMonoid M; static constexpr bool kX = true; static constexpr u32 xc = '>'; };
template <> struct Traits<F_SAM>   { typedef SamMonoid M;   static constexpr bool kX = true; static constexpr u32 xc = '@'; };

// FASTQ / LINE keep the tile's '\n' positions (tile-relative u16) in LDS: a record is then
// 4 (FASTQ) or 1 (line) consecutive entries and needs no search.  Tiles with more newlines
// than NLCAP (lines shorter than 8 bytes on average) use the region walk instead.
constexpr int NLCAP = TILE / 8;
constexpr int NLHALO = 4;  // newlines past the tile end kept in nlpos (one FASTQ record)
template <int F> constexpr bool kNlArray() { return F == F_FASTQ || F == F_LINE; }

template <int F, int NLC = NLCAP>
struct __align__(16) Smem {
  uint8_t raw[FRONT + TILE + HALO];  // raw[0] = byte tlo - FRONT
  u64 mnl[(TILE + HALO) / 64];
  u64 mx[Traits<F>::kX ? (TILE + HALO) / 64 : 1];
  uint16_t nlpos[kNlArray<F>() ? NLC : 1];
  u64 wtot[NWAVES];
  u64 tile_in;
  u64 badkey;
  u64 defer_s[MAX_DEFER];
  u64 defer_k[MAX_DEFER];
  u64 defer_aux[MAX_DEFER];
  u32 ndefer;
  u32 nh;  // newlines past the tile end in nlpos[T..T+nh)
  // FASTA: nextx[w] = tile-relative position of the first '>' in mask words >= w of
  // tile + halo (0xFFFF: none), so a lane finds the next '>' without walking the words
  uint16_t nextx[F == F_FASTA ? (TILE + HALO) / 64 + 1 : 1];
};

// any set bit of the 128-bit region mask (w0 | w1 << 64) in [lo, hi)
__device__ __forceinline__ bool any128(u64 w0, u64 w1, u32 lo, u32 hi) {
  if (lo >= hi) return false;
  u64 m0 = 0, m1 = 0;
  if (lo < 64) m0 = (~0ull << lo) & (hi >= 64 ? ~0ull : lowmask(hi));
  if (hi > 64) m1 = (lo > 64 ? (~0ull << (lo - 64)) : ~0ull) & lowmask(hi - 64);
  return (w0 & m0) || (w1 & m1);
}

// One record for the emission / deferred paths: validate and write its row or bad key.
struct Bad {
  u64 key = KEY_NONE, pos = 0, len = 0;
};

template <int F, class A>
__device__ __forceinline__ u32 run_record(A &a, u64 s, u64 aux, u64 &len, u64 &epos, u64 &elen) {
  if (F == F_FASTQ) return fastq_record(a, s, len);
  if (F == F_FASTA) return fasta_record(a, s, aux, len, epos, elen);
  if (F == F_SAM) return sam_record(a, s, len);
  return line_record(a, s, len);
}
// out-of-line instances for the rare / cold call sites (keeps the hot loop small)
template <int F, class A>
__device__ __noinline__ u32 run_record_cold(A &a, u64 s, u64 aux, u64 &len, u64 &epos, u64 &elen) {
  return run_record<F>(a, s, aux, len, epos, elen);
}

__device__ __forceinline__ void put_row(const SlabParams &p, u64 k, u64 s, u64 len) {
  const u64 i = k - p.row_base;
  if (k >= p.row_base && i < p.row_cap) {
    ulonglong2 v;
    v.x = p.base + s;
    v.y = len;
    reinterpret_cast<ulonglong2 *>(p.rows)[i] = v;
  }
}

__device__ __forceinline__ void note_bad(Bad &b, u64 k, u32 tile, u32 st, u64 pos, u64 len) {
  const u64 key = (k << KEY_REC_SHIFT) | ((u64)(tile & ((1u << KEY_TILE_BITS) - 1)) << 4) | st;
  if (key < b.key) { b.key = key; b.pos = pos; b.len = len; }
}

template <int F>
__device__ __forceinline__ void defer_record(const SlabParams &p, Smem<F> *sm, u64 s, u64 k, u64 aux) {
  const u32 slot = atomicAdd(&sm->ndefer, 1u);
  if (slot < MAX_DEFER) {
    sm->defer_s[slot] = s;
    sm->defer_k[slot] = k;
    sm->defer_aux[slot] = aux;
  } else {
    atomicAdd(&p.counters[1], 1u);  // never silently dropped: finalize flags an error
  }
}

template <int F, class A>
__device__ __forceinline__ void finish_record(const SlabParams &p, A &a, u32 tile, u64 s, u64 k,
                                              u64 aux, Bad &bad, Smem<F> *sm) {
  u64 len = 0, epos = 0, elen = 0;
  const u32 st = run_record<F>(a, s, aux, len, epos, elen);
  if (st == ST_OK) put_row(p, k, s, len);
  else if (st == ST_DEFER) defer_record<F>(p, sm, s, k, aux);
  else note_bad(bad, k, tile, st, p.base + epos, elen);
}

__device__ __forceinline__ bool ascii_nonspace(u32 c) { return c < 0x80 && !ascii_space(c); }

template <class A>
__device__ __forceinline__ u64 trimmed_len(A &a, u64 lo, u64 hi) {
  u64 tl, th;
  trim_space(a, lo, hi, tl, th);
  return th - tl;
}

// fastq.go:134-213 for a group whose four line ends e0..e3 are known (tile-relative, all
// staged in LDS): no searching, just the checks in Go's order.  A plus line that carries an
// ID (:195-199) is reported through needcmp/ilo/plo1/clen and compared by the whole wave;
// the length check (:202-207) that follows it comes back in lenbad.  Blank id lines take
// the general validator (ST_SLOW).
__device__ __forceinline__ u32 fq_known(const LaneAcc &a, u32 s, u32 e0, u32 e1, u32 e2, u32 e3, u32 &len,
                                        bool &needcmp, u32 &ilo, u32 &plo1, u32 &clen, bool &lenbad) {
  const uint8_t *r = a.raw + FRONT;
  if (e0 == s) return ST_SLOW;  // blank: skip-loop semantics (general validator)
  if (r[s] != '@') return ST_FQ_NOAT;
  if (e0 - s == 1) return ST_FQ_NOID;
  if (e1 == e0 + 1) return ST_FQ_EMPTYSEQ;
  if (r[e1 + 1] != '+') return ST_FQ_NOPLUS;
  const u64 tlo = a.tlo;
  if (e2 - e1 != 2) {
    u64 plo, phi;
    trim_space(a, tlo + e1 + 1, tlo + e2 + 1, plo, phi);
    if (phi - plo > 1) {
      u64 il, ih;
      trim_space(a, tlo + s + 1, tlo + e0 + 1, il, ih);
      if (ih - il != phi - plo - 1) return ST_FQ_IDMISMATCH;
      needcmp = ih > il;
      ilo = (u32)(il - tlo); plo1 = (u32)(plo + 1 - tlo); clen = (u32)(ih - il);
    }
  }
  u32 sl, ql;
  if (ascii_nonspace(r[e0 + 1]) && ascii_nonspace(r[e1 - 1])) sl = e1 - e0 - 1;
  else sl = (u32)trimmed_len(a, tlo + e0 + 1, tlo + e1 + 1);
  if (e3 > e2 + 1 && ascii_nonspace(r[e2 + 1]) && ascii_nonspace(r[e3 - 1])) ql = e3 - e2 - 1;
  else ql = (u32)trimmed_len(a, tlo + e2 + 1, tlo + e3 + 1);
  lenbad = sl != ql;
  len = e3 + 1 - s;
  return ST_OK;
}

// ====================================================================================
// Look-back (wave 0).  Status words are read and written through global (address space
// 1) agent-scope atomics only -- global_load/store ... sc1, never flat (guide §6 G16).
// ====================================================================================
typedef __attribute__((address_space(1))) u64 gu64;

__device__ __forceinline__ u64 st_load(gu64 *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(gu64 *p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 wflag(u64 w, u32 epoch) {
  return (((u32)(w >> EPOCH_SHIFT)) & EPOCH_MASK) == epoch ? (u32)(w >> 62) : 0u;
}


// ====================================================================================
// Two-pass build (k_index1<F>): one tile per workgroup, 16 B/lane buffer loads staged into
// LDS with the tile's class masks, incoming state from the scanned tile aggregates.
// ====================================================================================
__device__ __forceinline__ uint4 to_u4(__attribute__((ext_vector_type(4))) unsigned int x) {
  return make_uint4(x[0], x[1], x[2], x[3]);
}
// zero the bytes of v at index >= nb (0 < nb < 16)
__device__ __forceinline__ uint4 keep_bytes(uint4 v, u32 nb) {
  const u32 k0 = nb >= 4 ? ~0u : ((1u << (8 * nb)) - 1u);
  const u32 k1 = nb >= 8 ? ~0u : (nb <= 4 ? 0u : ((1u << (8 * (nb - 4))) - 1u));
  const u32 k2 = nb >= 12 ? ~0u : (nb <= 8 ? 0u : ((1u << (8 * (nb - 8))) - 1u));
  const u32 k3 = nb <= 12 ? 0u : ((1u << (8 * (nb - 12))) - 1u);
  return make_uint4(v.x & k0, v.y & k1, v.z & k2, v.w & k3);
}

// Tile loads through a buffer descriptor covering exactly [tlo, lhi).  The range check works
// on whole dwords: a dword that is not entirely inside returns 0, so only the last, partial
// dword of a slab needs bytes of its own (trim_tile).  The descriptor is built from
// wave-uniform values made explicitly scalar: a descriptor the compiler cannot prove uniform
// becomes a waterfall loop that waits for every load.  No loaded value is touched here (the
// loads stay in flight until stage_tile).
__device__ __forceinline__ u32 tile_llen(const SlabParams &p, u64 tile) {
  const u64 tlo = tile * TILE;
  const u64 lhi = (tlo + TILE + HALO < p.end) ? tlo + TILE + HALO : p.end;
  return (u32)(lhi - tlo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const SlabParams &p, u64 tile, u32 &llen) {
  const u64 ba = (u64)(p.data + tile * TILE);
  llen = (u32)__builtin_amdgcn_readfirstlane((int)tile_llen(p, tile));
  const uint8_t *sbase = (const uint8_t *)(((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)ba)) |
                                           ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)(ba >> 32)) << 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)sbase, (short)0, (int)llen, 0x00020000);
}
__device__ __forceinline__ void load_tile_buf(const SlabParams &p, u64 tile, int tid, uint4 (&v)[CPT + 1]) {
  const u64 tlo = tile * TILE;
  u32 llen;
  const auto rs = tile_rsrc(p, tile, llen);
  // one VGPR offset (this thread's chunk) + a constant scalar offset per chunk: no per-chunk
  // address registers to keep live (or spill) across the loop
  const int voff = tid * CHUNK;
#pragma unroll
  for (int k = 0; k < CPT; ++k)
    v[k] = to_u4(__builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * NTHREADS * CHUNK, 0));
  if (tid < HALO_CHUNKS) {
    v[CPT] = to_u4(__builtin_amdgcn_raw_buffer_load_b128(rs, voff, CPT * NTHREADS * CHUNK, 0));
  } else if (tid == HALO_CHUNKS) {
    v[CPT] = (tlo >= FRONT || p.front >= FRONT) ? load16(p.data + tlo - FRONT) : make_uint4(0, 0, 0, 0);
  }
}
// the readable end falls inside a dword (a slab's last tile only): fetch its bytes
__device__ __forceinline__ u32 tail_dword(const __amdgpu_buffer_rsrc_t rs, u32 llen) {
  const u32 d = llen & ~3u;
  u32 w = 0;
  for (u32 i = 0; i < (llen & 3u); ++i) w |= (u32)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(d + i), 0, 0) << (8 * i);
  return w;
}
__device__ __forceinline__ void patch_tail(uint4 &x, u32 off, u32 llen, u32 w) {
  const u32 q = ((llen & ~3u) - off) >> 2;  // dword of the chunk holding the end
  if (q == 0) x.x = w; else if (q == 1) x.y = w; else if (q == 2) x.z = w; else x.w = w;
}
__device__ __forceinline__ void trim_tile(const SlabParams &p, u64 tile, int tid, uint4 (&v)[CPT + 1]) {
  if (tile_llen(p, tile) >= (u32)(TILE + HALO) || (tile_llen(p, tile) & 3u) == 0) return;  // uniform
  u32 llen;
  const auto rs = tile_rsrc(p, tile, llen);
  const u32 w = tail_dword(rs, llen);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const u32 off = (u32)(k * NTHREADS + tid) * CHUNK;
    if (off < llen && off + CHUNK > llen) patch_tail(v[k], off, llen, w);
  }
  if (tid < HALO_CHUNKS) {
    const u32 off = (u32)(CPT * NTHREADS + tid) * CHUNK;
    if (off < llen && off + CHUNK > llen) patch_tail(v[CPT], off, llen, w);
  }
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() carries a workgroup-scope
// fence that waits vmcnt(0): on gfx950 (GFX9 counters) that drains every outstanding
// global load AND store of the wave -- the next tile's prefetch, the row stores, the
// look-back status stores -- at every barrier.  All intra-workgroup communication here is
// through LDS, so waiting for this wave's LDS operations is enough.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ u64 stamp() {
  u64 t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int F>
__device__ __forceinline__ void process_tile(const SlabParams &p, gu64 *status, u32 tile, Smem<F> &sm,
                                             int tid, int lane, int wid, u64 *ts) {
  typedef typename Traits<F>::M M;
  const u64 tlo = (u64)tile * TILE;
  const u64 thi = (tlo + TILE < p.n) ? tlo + TILE : p.n;
  const u32 tlen = (u32)(thi - tlo);

  // ---- region (128 contiguous bytes per thread) aggregates + ordered block scan --------
  const u32 rlo = (u32)tid * REGION;
  const u32 len0 = tlen > rlo ? (tlen - rlo >= 64 ? 64u : tlen - rlo) : 0u;
  const u32 len1 = tlen > rlo + 64 ? (tlen - rlo - 64 >= 64 ? 64u : tlen - rlo - 64) : 0u;
  // only bytes the slab owns: the halo past a slab's end belongs to the next slab's records
  const u64 nl0 = sm.mnl[2 * tid] & lowmask(len0), nl1 = sm.mnl[2 * tid + 1] & lowmask(len1);
  const u64 x0 = Traits<F>::kX ? sm.mx[2 * tid] & lowmask(len0) : 0;
  const u64 x1 = Traits<F>::kX ? sm.mx[2 * tid + 1] & lowmask(len1) : 0;
  const u64 ragg = M::combine(M::seg(nl0, x0, len0), M::seg(nl1, x1, len1));
  const u64 incl = wave_incl_scan<M>(ragg, lane);
  if (lane == 63) sm.wtot[wid] = incl;
  u64 lexcl = __shfl_up(incl, 1, 64);
  if (lane == 0) lexcl = M::identity();
  lds_barrier();
  u64 wpre = M::identity();
  for (int w = 0; w < wid; ++w) wpre = M::combine(wpre, sm.wtot[w]);
  const u64 texcl = M::combine(wpre, lexcl);
  u64 tagg = M::identity();
  for (int w = 0; w < NWAVES; ++w) tagg = M::combine(tagg, sm.wtot[w]);
  if (ts) ts[1] = stamp();

  // ---- incoming state: the exclusive prefix of the tile aggregates (scanned beforehand) ----
  if (wid == 0 && lane == 0) sm.tile_in = M::apply(p.state_in, p.tile_excl[tile]);
  // nlpos[0..T) = the tile's '\n' positions in order; nlpos[T..T+nh) = the first NLHALO
  // newlines past the tile end (line ends of the records that cross it), found by the last
  // wave
  const bool use_arr = kNlArray<F>() && tagg + NLHALO <= (u64)NLCAP;
  if (kNlArray<F>() && use_arr) {
    u32 o = (u32)texcl;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u64 m = h ? nl1 : nl0;
      while (m) {
        sm.nlpos[o++] = (uint16_t)(rlo + 64 * h + ctz64(m));
        m &= m - 1;
      }
    }
    if (wid == NWAVES - 1) {
      const u32 lhi_rel = (u32)(((tlo + TILE + HALO < p.end) ? tlo + TILE + HALO : p.end) - tlo);
      const u32 wb = tlen >> 6;  // first mask word holding bytes past the tile end
      u32 c = 0;
      u64 m = 0;
      const u32 wd = wb + (u32)lane;
      if (wd * 64 < lhi_rel) {
        m = sm.mnl[wd];
        if (wd == wb) m &= ~lowmask(tlen & 63);
        if (wd * 64 + 64 > lhi_rel) m &= lowmask(lhi_rel - wd * 64);
        c = popc64(m);
      }
      u32 pre = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(pre, d, 64);
        if (lane >= d) pre += y;
      }
      u32 o2 = pre - c;
      while (m && o2 < (u32)NLHALO) {
        sm.nlpos[(u32)tagg + o2] = (uint16_t)(wd * 64 + ctz64(m));
        ++o2;
        m &= m - 1;
      }
      if (lane == 63) sm.nh = pre < (u32)NLHALO ? pre : (u32)NLHALO;
    }
  }
  if (tid == 0) { sm.ndefer = 0; sm.badkey = KEY_NONE; }
  if (F == F_FASTA && wid == NWAVES - 1) {  // suffix min over the '>' mask words, 64 per step
    constexpr u32 NW = (TILE + HALO) / 64;
    u32 carry = 0xFFFFu;
    if (lane == 0) sm.nextx[NW] = 0xFFFFu;
    for (int b = (int)((NW - 1) / 64) * 64; b >= 0; b -= 64) {
      const u32 w = (u32)b + (u32)lane;
      u32 x = 0xFFFFu;
      if (w < NW) {
        const u64 m = sm.mx[w];
        if (m) x = w * 64 + ctz64(m);
      }
      // suffix min within the wave (lane i: min over lanes >= i), then the carry from above
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u32 y = (u32)__shfl_down((int)x, d, 64);
        if (lane + d < 64 && y < x) x = y;
      }
      if (carry < x) x = carry;
      if (w < NW) sm.nextx[w] = (uint16_t)x;
      carry = (u32)__shfl((int)x, 0, 64);
    }
  }
  if (ts) ts[2] = stamp();
  lds_barrier();
  if (ts) ts[3] = stamp();
  if (dbg(p) & 1) return;  // ablation: scan only
  const u64 tile_state = sm.tile_in;
  const u64 tin = M::apply(tile_state, texcl);  // state before this thread's region

  // ---- emission: records owned by this tile ---------------------------------------------
  LaneAcc acc;
  acc.raw = sm.raw; acc.mnl = sm.mnl; acc.mx = sm.mx;
  if (F == F_FASTA) acc.nextx = sm.nextx;
  acc.tlo = tlo; acc.lhi = (tlo + TILE + HALO < p.end) ? tlo + TILE + HALO : p.end;
  acc.end = p.end; acc.eof = p.eof; acc.dbg = dbg(p); acc.front = p.front;
  Bad bad;

  if (kNlArray<F>() && use_arr) {
    const u32 T = (u32)tagg;  // newlines in the tile; nlpos[0..T)
    const u64 j0 = tile_state;  // rank of the tile's first '\n'
    if (F == F_FASTQ) {
      // groups start after '\n' #j with j % 4 == 3 (and at file offset 0); a group whose four
      // line ends are in nlpos (tile + halo) is checked by fq_known, the rest (blank lines,
      // EOF, records longer than the halo) by the general validator
      const u32 TT = T + sm.nh;
      const u32 i0 = (u32)((3 - (j0 & 3)) & 3);
      const u32 ng = i0 < T ? (T - i0 + 3) / 4 : 0;
      for (u32 qb = (u32)wid * 64; qb < ng + 1; qb += NTHREADS) {  // wave-uniform trip count
        const u32 q = qb + (u32)lane;
        bool act = q < ng + 1;
        u32 s = 0, i = 0;
        u64 g = 0;
        if (act && q == ng) {  // the file-start group, owned by tile 0
          act = p.file_start && tile == 0;
        } else if (act) {
          const u32 d = i0 + 4 * q;
          s = sm.nlpos[d] + 1u; g = (j0 + d + 1) >> 2; i = d + 1;
        }
        if (dbg(p) & 32) act = false;
        u32 st = ST_SLOW, len = 0, ilo = 0, plo1 = 0, clen = 0;
        bool needcmp = false, lenbad = false;
        if (act && i + 3 < TT)
          st = fq_known(acc, s, sm.nlpos[i], sm.nlpos[i + 1], sm.nlpos[i + 2], sm.nlpos[i + 3], len, needcmp,
                        ilo, plo1, clen, lenbad);
        // fastq.go:195-199 ID compare, wave-cooperative: one record at a time, 64 bytes per step
        u64 mc = __ballot(act && st == ST_OK && needcmp);
        bool idmis = false;
        while (mc) {
          const int L = (int)ctz64(mc);
          mc &= mc - 1;
          const u32 a = (u32)__shfl((int)ilo, L, 64), b = (u32)__shfl((int)plo1, L, 64);
          const u32 n = (u32)__shfl((int)clen, L, 64);
          bool ne = false;
          for (u32 k = (u32)lane; k < n; k += 64) ne |= sm.raw[FRONT + a + k] != sm.raw[FRONT + b + k];
          const bool any = __ballot(ne) != 0;
          if (lane == L) idmis = any;
        }
        if (st == ST_OK && needcmp && idmis) st = ST_FQ_IDMISMATCH;
        else if (st == ST_OK && lenbad) st = ST_FQ_LENMISMATCH;
        if (!act) continue;
        u64 glen = len, epos = 0, elen = 0;
        if (st == ST_SLOW) st = run_record_cold<F>(acc, tlo + s, 0, glen, epos, elen);
        if (st == ST_OK) { if (!(dbg(p) & 16)) put_row(p, g, tlo + s, glen); }
        else if (st == ST_DEFER) defer_record<F>(p, &sm, tlo + s, g, 0);
        else note_bad(bad, g, tile, st, 0, 0);
      }
    } else {  // F_LINE: one row per line, row j+1 starts after '\n' #j
      for (u32 q = tid; q < T + 1; q += NTHREADS) {
        u64 s, k;
        u32 i;
        if (q == T) {
          if (!(p.file_start && tile == 0)) continue;
          s = 0; k = 0; i = 0;
        } else {
          s = sm.nlpos[q] + 1u; k = j0 + q + 1; i = q + 1;
        }
        if (i < T + sm.nh) put_row(p, k, tlo + s, (u64)sm.nlpos[i] + 1 - s);
        else finish_record<F>(p, acc, tile, tlo + s, k, 0, bad, &sm);
      }
    }
  } else {
    if (p.file_start && tile == 0 && tid == 0) {  // record 0 starts at file offset 0
      u64 aux = 0;
      if (F == F_FASTA) aux = (p.end > 0 && acc.byte(0) == '>') ? 1 : 0;
      finish_record<F>(p, acc, tile, 0, 0, aux, bad, &sm);
    }
    if (F == F_FASTQ || F == F_LINE) {
      u64 j = tin;  // global '\n' rank of the next newline
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u64 m = h ? nl1 : nl0;
        while (m) {
          const u64 q = tlo + rlo + 64 * h + ctz64(m);
          m &= m - 1;
          if (F == F_LINE) finish_record<F>(p, acc, tile, q + 1, j + 1, 0, bad, &sm);
          else if ((j & 3) == 3) finish_record<F>(p, acc, tile, q + 1, (j + 1) >> 2, 0, bad, &sm);
          ++j;
        }
      }
    } else if (F == F_FASTA) {
      u64 cnt = tin >> 1;
      u32 armed = tin & 1;
      u32 pos = 0;  // region-relative
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u64 m = h ? x1 : x0;
        while (m) {
          const u32 g = 64 * h + ctz64(m);
          m &= m - 1;
          if (any128(nl0, nl1, pos, g)) armed = 1;  // '\n' since the previous '>'
          if (armed) {
            ++cnt;
            const u64 b = tlo + rlo + g;
            finish_record<F>(p, acc, tile, b, cnt, b + 1, bad, &sm);
          }
          armed = 0;
          pos = g + 1;
        }
      }
    } else {  // F_SAM
      u64 cnt = tin >> 2;
      const u32 st0 = tin & 3;
      bool first = true;
      u64 prev = 0;  // tile-relative position of the previous '\n' in this region
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u64 m = h ? nl1 : nl0;
        while (m) {
          const u64 q = rlo + 64 * h + ctz64(m);
          m &= m - 1;
          bool term;
          if (first && st0 != 0) {
            term = (st0 == 1);
          } else {
            const u64 ls = first ? (u64)rlo : prev + 1;
            term = (ls < q) && acc.byte(tlo + ls) != '@';
          }
          first = false;
          prev = q;
          if (term) {
            ++cnt;
            finish_record<F>(p, acc, tile, tlo + q + 1, cnt, 0, bad, &sm);
          }
        }
      }
    }
  }
  if (ts) ts[4] = stamp();
  lds_barrier();
  if (ts) ts[5] = stamp();

  // ---- deferred records: wave-cooperative global-memory path -----------------------------
  if (!(dbg(p) & 4)) {
    const u32 nd = sm.ndefer < MAX_DEFER ? sm.ndefer : MAX_DEFER;
    WaveAcc wa;
    wa.g = p.data; wa.end = p.end; wa.eof = p.eof; wa.lane = lane; wa.front = p.front;
    for (u32 i = wid; i < nd; i += NWAVES) {
      const u64 s = sm.defer_s[i], k = sm.defer_k[i], aux = sm.defer_aux[i];
      u64 len = 0, epos = 0, elen = 0;
      // inline: an out-of-line call here saved ~5 KB of registers to scratch per tile
      const u32 st = run_record<F>(wa, s, aux, len, epos, elen);
      if (lane == 0) {
        if (st == ST_OK) put_row(p, k, s, len);
        else note_bad(bad, k, tile, st, p.base + epos, elen);
      }
    }
  }

  // ---- first bad record of the tile -> slab-wide min ----------------------------------------
  if (ts) ts[6] = stamp();
  if (bad.key != KEY_NONE) atomicMin(&sm.badkey, bad.key);
  lds_barrier();
  const u64 tkey = sm.badkey;
  if (tkey != KEY_NONE) {
    if (bad.key == tkey) {
      p.detail[2 * (u64)tile] = bad.pos;
      p.detail[2 * (u64)tile + 1] = bad.len;
    }
    if (tid == 0) atomicMin(p.badkey, tkey);  // one device-scope atomic per tile with a bad record
  }
}

// stage a loaded tile: raw bytes + per-byte class masks into LDS
template <int F, class SM>
__device__ __forceinline__ void stage_tile(SM &sm, const uint4 (&v)[CPT + 1], int tid) {
  uint16_t *mnl16 = reinterpret_cast<uint16_t *>(sm.mnl);
  uint16_t *mx16 = reinterpret_cast<uint16_t *>(sm.mx);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const u32 c = (u32)(k * NTHREADS + tid);
    *reinterpret_cast<uint4 *>(&sm.raw[FRONT + c * CHUNK]) = v[k];
    mnl16[c] = (uint16_t)eq16(v[k], '\n');
    if (Traits<F>::kX) mx16[c] = (uint16_t)eq16(v[k], Traits<F>::xc);
  }
  if (tid < HALO_CHUNKS) {
    const u32 c = (u32)(CPT * NTHREADS + tid);
    *reinterpret_cast<uint4 *>(&sm.raw[FRONT + c * CHUNK]) = v[CPT];
    mnl16[c] = (uint16_t)eq16(v[CPT], '\n');
    if (Traits<F>::kX) mx16[c] = (uint16_t)eq16(v[CPT], Traits<F>::xc);
  } else if (tid == HALO_CHUNKS) {
    *reinterpret_cast<uint4 *>(&sm.raw[0]) = v[CPT];
  }
}

// k_tile_agg<F>: pass 1 of a two-pass build -- the monoid aggregate of every tile (bytes
// [tlo, thi) only), no staging of the raw bytes: 16-B/lane loads -> per-chunk class masks in
// LDS -> per-thread 128-byte regions in byte order -> ordered block reduce.
template <int F>
__global__ __launch_bounds__(NTHREADS) void k_tile_agg(const SlabParams p, u64 *agg) {
  typedef typename Traits<F>::M M;
  __shared__ u64 mnl[TILE / 64], mx[Traits<F>::kX ? TILE / 64 : 1], wtot[NWAVES];
  // a wrongly speculated format: the two-pass kernels exit like the tile passes
  if (gated_off(p)) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u64 tile = blockIdx.x, tlo = tile * TILE;
  const u32 tlen = (u32)(((tlo + TILE < p.n) ? tlo + TILE : p.n) - tlo);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p.data + tlo), (short)0, (int)tlen, 0x00020000);
  uint4 v[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k)
    v[k] = to_u4(__builtin_amdgcn_raw_buffer_load_b128(rs, (int)((u32)(k * NTHREADS + tid) * CHUNK), 0, 0));
  if (tlen & 3u) {  // the slab's last dword is partial: its bytes one by one
    const u32 w = tail_dword(rs, tlen);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const u32 off = (u32)(k * NTHREADS + tid) * CHUNK;
      if (off < tlen && off + CHUNK > tlen) patch_tail(v[k], off, tlen, w);
    }
  }
  uint16_t *m16 = reinterpret_cast<uint16_t *>(mnl), *x16 = reinterpret_cast<uint16_t *>(mx);
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const u32 c = (u32)(k * NTHREADS + tid);
    m16[c] = (uint16_t)eq16(v[k], '\n');
    if (Traits<F>::kX) x16[c] = (uint16_t)eq16(v[k], Traits<F>::xc);
  }
  __syncthreads();
  const u32 rlo = (u32)tid * REGION;
  const u32 len0 = tlen > rlo ? (tlen - rlo >= 64 ? 64u : tlen - rlo) : 0u;
  const u32 len1 = tlen > rlo + 64 ? (tlen - rlo - 64 >= 64 ? 64u : tlen - rlo - 64) : 0u;
  const u64 nl0 = mnl[2 * tid] & lowmask(len0), nl1 = mnl[2 * tid + 1] & lowmask(len1);
  const u64 x0 = Traits<F>::kX ? mx[2 * tid] & lowmask(len0) : 0, x1 = Traits<F>::kX ? mx[2 * tid + 1] & lowmask(len1) : 0;
  const u64 ragg = M::combine(M::seg(nl0, x0, len0), M::seg(nl1, x1, len1));
  const u64 incl = wave_incl_scan<M>(ragg, lane);
  if (lane == 63) wtot[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    u64 t = M::identity();
    for (int w = 0; w < NWAVES; ++w) t = M::combine(t, wtot[w]);
    agg[tile] = t;
  }
}

// the slab aggregate of a two-pass build, where k_finalize reads it (last status word)
__global__ void k_tile_total(const SlabParams p, const u64 *agg, const u64 *excl, int fmt) {
  if (threadIdx.x || blockIdx.x || gated_off(p)) return;
  const u64 t = p.ntiles - 1;
  u64 tot;
  if (fmt == F_FASTA) tot = FastaMonoid::combine(excl[t], agg[t]);
  else if (fmt == F_SAM) tot = SamMonoid::combine(excl[t], agg[t]);
  else tot = CountMonoid::combine(excl[t], agg[t]);
  ((u64 *)p.status)[t] = FLAG_INC | ((u64)p.epoch << EPOCH_SHIFT) | tot;
}

// k_index1<F>: one tile per workgroup (grid = ntiles), no register prefetch: latency is
// hidden by the other workgroups resident on the CU rather than inside the workgroup.
template <int F>
__global__ __launch_bounds__(NTHREADS) void k_index1(const SlabParams p) {
  __shared__ Smem<F> sm;
  if (gated_off(p)) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 tile = blockIdx.x;
  const bool timing = tmg(p) && tid == 0;
  u64 tsb[8];
  if (timing) tsb[0] = stamp();
  {
    uint4 v[CPT + 1];
    load_tile_buf(p, tile, tid, v);
    trim_tile(p, tile, tid, v);
    stage_tile<F>(sm, v, tid);
  }
  lds_barrier();
  if (timing) tsb[7] = stamp();
  process_tile<F>(p, (gu64 *)p.status, tile, sm, tid, lane, wid, timing ? tsb : nullptr);
  if (timing) {  // diagnostic: phase sums into 65536 slots (summed by the host)
    const u64 te = stamp();
    u64 *o = tmg(p) + (u64)(blockIdx.x & 65535) * 9;
    atomicAdd(&o[0], tsb[7] - tsb[0]);
    atomicAdd(&o[1], tsb[1] - tsb[7]);
    atomicAdd(&o[2], tsb[2] - tsb[1]);
    atomicAdd(&o[3], tsb[3] - tsb[2]);
    atomicAdd(&o[4], tsb[4] - tsb[3]);
    atomicAdd(&o[5], tsb[5] - tsb[4]);
    atomicAdd(&o[6], te - tsb[5]);
    atomicAdd(&o[8], 1ull);
  }
}


// ====================================================================================
// Tile-pass building blocks (k_fq_tiles / k_fa_tiles / k_line_tiles): result encodings,
// the k_fixup queue, the LDS certifiers and the device-scope atomics they use.
// ====================================================================================
constexpr int RCAP = TILE / 64;  // records per tile kept in the provisional row slot
constexpr u32 GUESS_NONE = 4;


constexpr u32 FIX_HALO = 0x80000000u;  // FixRec::tile flag (FASTA / line slabs): a record closed in the halo
struct FixRec {          // k_fixup work item: one record, or one whole tile (start == ~0)
  u64 start;             // file-relative start of the record (slab offset)
  u64 g;                 // its global record number; for a tile: the tile's rank j0
  u32 tile;
  u32 pad;
};


// ASCII bytes.TrimSpace bounds of r[lo, hi); false if a byte >= 0x80 decides (Unicode path)
__device__ __forceinline__ bool trim_ascii(const uint8_t *r, u32 lo, u32 hi, u32 &tl, u32 &th) {
  while (lo < hi) {
    const u32 c = r[lo];
    if (c >= 0x80) return false;
    if (!ascii_space(c)) break;
    ++lo;
  }
  while (hi > lo) {
    const u32 c = r[hi - 1];
    if (c >= 0x80) return false;
    if (!ascii_space(c)) break;
    --hi;
  }
  tl = lo; th = hi;
  return true;
}

// Inclusive add-scan over a wave in DPP steps (row shifts 1/2/4/8, then the two row
// broadcasts): no LDS round trips, unlike __shfl_up (ds_bpermute).
__device__ __forceinline__ u32 wave_scan_add(u32 v) {
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}


__device__ __forceinline__ u32 umax(u32 a, u32 b) { return a > b ? a : b; }

// lanes below this one with their bit set in b
__device__ __forceinline__ u32 mbcnt64(u64 b) {
  return __builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u));
}
// inclusive wave scan of small per-lane counts: two ballots and their lane-prefix counts when
// every count is below 4 (a 64-byte word holds at most three '\n' unless lines are under ~21
// bytes), else the DPP scan -- 7 VALU instead of 12
__device__ __forceinline__ u32 wave_scan_add_small(u32 c) {
  if (__ballot(c > 3u) == 0) {
    const u64 b1 = __ballot(c & 1u), b2 = __ballot(c & 2u);
    return mbcnt64(b1) + 2u * mbcnt64(b2) + c;
  }
  return wave_scan_add(c);
}

// FastaMonoid::combine on 32-bit aggregates (a wave's count of '>' fits 13 bits)
__device__ __forceinline__ u32 fa_comb32(u32 a, u32 b) {
  const u32 af = a & 3u, bf = b & 3u;
  const u32 bd = (b >> 2) & 1u;
  const u32 cnt = (a >> 3) + (b >> 3) + ((af == 2u) ? bd : 0u);
  const u32 d = af == 0u ? bd : (a >> 2) & 1u;
  const u32 f = bf == 0u ? af : bf;
  return (cnt << 3) | (d << 2) | f;
}
// wave-inclusive scans over DPP row shifts / broadcasts (no LDS round trips; identity 0 fills
// the lanes a shift leaves without a source, as in wave_scan_add)
#define SIDX_DPP_SCAN(v, OP)                                                                   \
  do {                                                                                         \
    v = OP((u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false), v);            \
    v = OP((u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false), v);            \
    v = OP((u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false), v);            \
    v = OP((u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false), v);            \
    v = OP((u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false), v);            \
    v = OP((u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false), v);            \
  } while (0)
__device__ __forceinline__ u32 wave_scan_fa32(u32 v) { SIDX_DPP_SCAN(v, fa_comb32); return v; }
__device__ __forceinline__ u32 wave_scan_max(u32 v) { SIDX_DPP_SCAN(v, umax); return v; }

// bytes that differ between raw[a, a+4) and raw[b, b+4) (only the first n if n < 4);
// aligned dword LDS reads + v_alignbyte (raw is 4-aligned)
__device__ __forceinline__ u32 lds_diff4(const uint8_t *raw, u32 a, u32 b, u32 n) {
  const u32 *w = reinterpret_cast<const u32 *>(raw);
  const u32 wa = __builtin_amdgcn_alignbyte(w[(a >> 2) + 1], w[a >> 2], a & 3);
  const u32 wb = __builtin_amdgcn_alignbyte(w[(b >> 2) + 1], w[b >> 2], b & 3);
  const u32 m = n >= 4 ? ~0u : ((1u << (8 * n)) - 1u);
  return (wa ^ wb) & m;
}


// fastq.go:134-213 certifies the record [s, e3] valid (the common case) when its TrimSpace
// edges are printable ASCII, LF or CRLF line ends: branch-free over the 13 edge bytes (one
// LDS round).  Anything else -- an error, a blank or space-padded line, a byte >= 0x80 at an
// edge -- returns false and the record goes to k_fixup, whose general validator reports
// exactly what Go reports.  A plus line that carries an ID comes back with cn = the ID length:
// r[s+1, s+1+cn) must then equal r[cb, cb+cn) (the caller compares).  r: the tile's byte 0.
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"  // the flags below are combined branch-free
__device__ __forceinline__ bool fq_ok(const uint8_t *r, u32 s, u32 e0, u32 e1, u32 e2, u32 e3, u32 &cn, u32 &cb,
                                      u32 &crs, bool &idclean) {
  const u32 cs = r[s], ci1 = r[s + 1], cs1 = r[e0 + 1], cp = r[e1 + 1], cq1 = r[e2 + 1];
  const u32 a0 = r[e0 - 1], a1 = r[e1 - 1], a2 = r[e2 - 1], a3 = r[e3 - 1];
  const u32 b0 = r[e0 - 2], b1 = r[e1 - 2], b2 = r[e2 - 2], b3 = r[e3 - 2];
  // a '\r' before the '\n' is trimmed too: z = the end of the line's trimmed content
  const u32 c0 = a0 == '\r', c1 = a1 == '\r', c2 = a2 == '\r', c3 = a3 == '\r';
  const u32 z0 = e0 - c0, z1 = e1 - c1, z2 = e2 - c2, z3 = e3 - c3;
  const u32 l0 = c0 ? b0 : a0, l1 = c1 ? b1 : a1, l2 = c2 ? b2 : a2, l3 = c3 ? b3 : a3;
  const bool pluslong = z2 > e1 + 2;  // TrimSpace(plus) longer than "+": the ID must match
  const bool ok = (e0 > s + 1) & (cs == '@') & (cp == '+') &                   // :164-169, :191
                  (z1 > e0 + 1) & ascii_nonspace(cs1) & ascii_nonspace(l1) &   // seq content
                  (z3 > e2 + 1) & ascii_nonspace(cq1) & ascii_nonspace(l3) &   // qual content
                  (z1 - e0 == z3 - e2) &                                       // :202-207
                  ascii_nonspace(l2) &                                         // plus edge
                  (!pluslong | (ascii_nonspace(ci1) & ascii_nonspace(l0) & (z0 - s == z2 - e1 - 1)));
  cn = (ok && pluslong) ? z0 - s - 1 : 0u;  // :195-199 ID bytes r[s+1..] vs r[e1+2..]
  cb = e1 + 2;
  crs = c0 | (c1 << 1) | (c3 << 2);  // (filters) the '\r' before the ID / sequence / quality line ends
  idclean = ascii_nonspace(ci1) & ascii_nonspace(l0) & (z0 > s + 1);  // TrimSpace(ID) drops only the line end
  return ok;
}

// FASTQ phase read off the tile: the first newline c (of the first 16) after which an
// '@' line, a sequence line, a '+' line and an equal-length quality line follow.
__device__ __forceinline__ u32 fq_guess_at(const uint8_t *raw, const uint16_t *nlpos, u32 TT, int lane) {
  // branch-free: every lane reads (clamped indices, values ignored where not valid), so the
  // two LDS rounds are not serialised behind branches
  const u32 c = (u32)lane & 15u;
  const u32 a = nlpos[c], b1 = nlpos[c + 1], b2 = nlpos[c + 2], b3 = nlpos[c + 3], b4 = nlpos[c + 4];
  const u32 x = raw[FRONT + a + 1], y = raw[FRONT + b2 + 1];
  const bool ok = ((u32)lane < 16) & (c + 4 < TT) & (x == '@') & (y == '+') & (b2 - b1 > 1) & ((b2 - b1) == (b4 - b3));
  const u64 m = __ballot(ok);
  return m ? (ctz64(m) & 3u) : GUESS_NONE;
}

// Device-scope atomics and stores through address-space-1 pointers: a generic (flat) access
// inside the streaming loop would make the compiler drain every outstanding load, the tile
// DMA included, before the next LDS access (a flat access may touch LDS).
typedef __attribute__((address_space(1))) u32 gu32;
__device__ __forceinline__ u32 g_add(u32 *p, u32 v) {
  return __hip_atomic_fetch_add((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_or(u32 *p, u32 v) {
  (void)__hip_atomic_fetch_or((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_min64(u64 *p, u64 v) {
  (void)__hip_atomic_fetch_min((__attribute__((address_space(1))) u64 *)p, v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void push_fix(const SlabParams &p, u64 start, u64 g, u32 tile) {
  const u32 i = g_add(&p.counters[2], 1u);
  if (i < p.fixcap) {
    __attribute__((address_space(1))) u64 *f = (__attribute__((address_space(1))) u64 *)(p.fix + 3 * (u64)i);
    f[0] = start; f[1] = g; f[2] = tile;  // FixRec {start, g, tile, pad}
  } else {
    g_or(&p.counters[3], 1u);  // overflow: the host re-runs the build on the general kernel
  }
  if (start == ~0ull) (void)g_add(&p.counters[3], 2u);  // whole-tile items (diagnostic), bits 1..
}


// ====================================================================================
// LDS-DMA tile staging shared by the tile passes: a 256-thread workgroup stages one 16 KiB
// tile (+ the 16 bytes in front of it and a 1 KiB halo) into its LDS slot by buffer_load ...
// lds (1 KiB per wave-instruction, no VGPR destination), waits with vmcnt and classifies its
// own 64 bytes per thread into one '\n' mask word.
// ====================================================================================
constexpr int SNT = TILE / 64;                // threads per workgroup: one 64-byte '\n' mask word each
constexpr int SNW = SNT / 64;
static_assert(HALO % 256 == 0, "256-byte halo DMA pieces");
constexpr int SHPW = (HALO / 256 + SNW - 1) / SNW;  // halo pieces per wave (the last waves may have fewer)
constexpr int SSLOT = FRONT + TILE + HALO;    // LDS slot: [16 bytes before | tile | halo]
static_assert(SSLOT % 16 == 0, "16-byte aligned slots");
constexpr int SPER = TILE / 1024 / SNW;       // 1 KiB DMA wave-instructions per wave per tile
#ifndef SIDX_SNLCAP_DIV
#define SIDX_SNLCAP_DIV 16
#endif
constexpr int SNLCAP = TILE / SIDX_SNLCAP_DIV;  // '\n' positions kept (lines >= 16 B on average)
constexpr int SHW = HALO / 64;                // halo mask words (classified by the last wave)
static_assert(SHW <= 64, "halo words fit one wave");



constexpr int SHALO = HALO - FRONT;           // halo bytes past the tile read into a slot
typedef __attribute__((address_space(3))) uint8_t lds_u8;
// cache policy of the DMA: SIDX_DMA_NT bit 0 = the tile body non-temporal (read once), bit 1 =
// the 256-byte pieces (halo, front) too -- the halo is the next tile's first KiB, which the
// neighbouring workgroup on the same XCD reads, so it keeps the default policy.  Round 4, input
// in contiguous HBM, interleaved A/B on one box: k_fq_tiles 1.910 -> 1.874 ms with the body nt
// (bit 1 as well: slower); FASTA and line tiles take the nt body always (dma_piece16_nt)
#ifndef SIDX_DMA_NT
#define SIDX_DMA_NT 1
#endif
#if SIDX_DMA_NT & 1
#define SIDX_POL16 "nt "
#else
#define SIDX_POL16 ""
#endif
#if SIDX_DMA_NT & 2
#define SIDX_POL4 "nt "
#else
#define SIDX_POL4 ""
#endif
__device__ __forceinline__ void dma_piece16(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen " SIDX_POL16 "lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
// The tile body non-temporal: FASTA and line tiles (no halo read by a neighbour) -- A/B on one
// box, 10 GiB: k_fa_tiles 2.21 -> 2.15 ms, k_line_tiles 2.24 -> 2.06 ms; FASTQ unchanged, so it
// keeps the default policy (its halo is the next tile's first KiB, read through L2)
__device__ __forceinline__ void dma_piece16_nt(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen nt lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ void dma_piece4(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  lds = (u32)__builtin_amdgcn_readfirstlane((int)lds);  // uniform by construction (M0)
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %1, %3, 0 offen " SIDX_POL4 "lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
// P0: DMA of tile tn into the slot `dst` ([16 bytes in front | tile | halo], slot byte o = file
// byte tlo - FRONT + o).  Wave w stages the tile bytes [4096 w, 4096 (w + 1)) -- exactly the
// 64-byte words its own threads classify first -- as 4 pieces of 1 KiB (16 bytes per lane), so
// each wave starts on its masks after its own covering vmcnt, with no barrier: an LDS-DMA is
// ordered for the issuing wave's reads by its vmcnt alone (MI355X_MICROARCH.md, co-residence
// item 7), and other waves read those bytes only after a later barrier.  kFq: also the 16
// bytes in front (wave 0, 4 lanes of 4 bytes) and the halo (one 256-byte piece per wave), both
// read only after a barrier.  The buffer range [., min(., end)) is checked per dword: nothing
// past the slab's readable end is read (those dwords land as zeros).  For the file's first tile
// (no bytes in front) the base is the tile itself and the front piece's lanes fall out of range.
// The DMA is inline asm the compiler does not track: its waits are counted by hand, and no
// compiler-visible load is live across it in the loop.
// A wave's 4 KiB of the tile body as four pieces under one M0 (the instruction offset advances
// the global and the LDS address together) instead of one M0 save / set / restore per piece:
// A/B on one box (profiles/r04/ab_m0once.txt) k_fq_tiles 1.876 -> 1.855 ms, k_fa_tiles
// 2.134 -> 2.095 ms -- the tile passes issue a third of their instructions on the scalar unit.
// (Folding the FASTQ halo piece into the same statement measured the same: ab_halofold_fastq.txt.)
#ifndef SIDX_DMA_M0ONCE
#define SIDX_DMA_M0ONCE 1
#endif
template <bool kNt>
__device__ __forceinline__ void dma_body4(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  if (kNt)
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen nt lds\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen offset:1024 nt lds\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen offset:2048 nt lds\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen offset:3072 nt lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
  else
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen offset:1024 lds\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen offset:2048 lds\n\t"
                 "buffer_load_dwordx4 %1, %3, 0 offen offset:3072 lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
template <bool kFq>
__device__ __forceinline__ void stage_tile(const SlabParams &p, u64 tn, u32 dst, int wid, int lane) {
  const u64 tlo = tn * TILE;
  const bool shifted = tlo >= FRONT || p.front >= FRONT;
  const u64 ba = (u64)(p.data + tlo) - (shifted ? FRONT : 0);
  const u64 lim = (tlo + TILE + SHALO < p.end) ? tlo + TILE + SHALO : p.end;
  const u32 nrec = (u32)(lim - tlo) + (shifted ? FRONT : 0);
  const uint8_t *sbase = (const uint8_t *)(((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)ba)) |
                                           ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)(ba >> 32)) << 32));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)sbase, (short)0,
                                                    (int)__builtin_amdgcn_readfirstlane((int)nrec), 0x00020000);
  const u32 adj = shifted ? 0u : (u32)FRONT;  // unshifted: slot offsets are 16 bytes ahead of the base
  const u32 w0 = (u32)FRONT + (u32)(wid * SPER) * 1024u;
  if (SIDX_DMA_M0ONCE && SPER == 4) {
    dma_body4<!kFq || (SIDX_DMA_NT & 1)>(w0 + (u32)lane * 16u - adj, dst + w0, rs);
  } else {
#pragma unroll
    for (int i = 0; i < SPER; ++i) {
      if (kFq) dma_piece16(w0 + (u32)i * 1024u + (u32)lane * 16u - adj, dst + w0 + (u32)i * 1024u, rs);
      else dma_piece16_nt(w0 + (u32)i * 1024u + (u32)lane * 16u - adj, dst + w0 + (u32)i * 1024u, rs);
    }
  }
  if (!kFq) return;
  if (wid == 0 && lane < FRONT / 4) dma_piece4((u32)lane * 4u - adj, dst, rs);
#pragma unroll
  for (int h = 0; h < SHPW; ++h) {
    const int piece = wid * SHPW + h;
    const u32 h0 = (u32)(FRONT + TILE) + (u32)piece * 256u;
    if (piece < HALO / 256) dma_piece4(h0 + (u32)lane * 4u - adj, dst + h0, rs);
  }
}

// ====================================================================================
// FASTQ tile pass: k_fq_tiles -> exclusive scan of the tile newline counts -> k_fq_place.
// LDS-DMA staging, '\n' masks, newline positions, the phase read off the tile, lane
// validation with fq_ok -- and no cross-workgroup dependency at all: each tile's valid records go to a provisional row table (start |
// length << 16, indexed by the tile-local record number) and its newline count to agg[t].
// Once every count is known, a device-wide scan gives each tile's true newline rank j0, and
// k_fq_place writes the final rows at their global record numbers (or queues the tile for
// k_fixup when the phase guess was wrong).  Extra traffic: 4 bytes per record
// written and read back (about 2 % of the input for short-read FASTQ).
// ====================================================================================
// Per-tile results.  Every byte this pass writes is expensive next to the bytes it streams in
// (tools/streambench.hip: 32 bytes per 16 KiB tile cost 4 % of the pass, 228 bytes 10 %), so a
// tile writes one u64 (fq_agg[t], packed below; the scan reads its newline count) and one u16
// per record (its start, bit 15 = not certified) plus the end of the last record -- a record's
// length is the next one's start minus its own (the records of a tile are back to back).
// Deferred records (dl[], ds[]: 2 * MAX_DEFER words per tile) are written only when a tile
// defers.
// (nrec: 9 bits -- a tile keeps at most RCAP records' starts, more makes it slow and nrec unused)
constexpr u32 FQW_T = 0, FQW_GI = 16, FQW_NREC = 19, FQW_SLOW = 28, FQW_NDEF = 29;
constexpr u32 FQW_NRECM = 0x1FF;
constexpr u64 FQW_TMASK = 0xFFFF;  // the newline count: what the scan folds
__device__ __forceinline__ u64 fq_word(u32 T, u32 gi0, u32 nrec, bool slow, u32 ndefer) {
  return ((u64)T << FQW_T) | ((u64)(gi0 & 7u) << FQW_GI) | ((u64)(nrec < FQW_NRECM ? nrec : FQW_NRECM) << FQW_NREC) |
         ((u64)(slow || nrec > (u32)RCAP) << FQW_SLOW) | ((u64)ndefer << FQW_NDEF);
}
// Where a tile's u16 starts are (round 6): tile t's first FQ_LINE_E entries in one 128-byte line
// at entry FQ_LINE_E t of fq_stage -- a dense, tile-indexed array that advances with the read
// stream, one full-line store per tile -- and entries FQ_LINE_E.. (tiles of more than 63
// records; C2 has ~47 per tile) in an overflow slot of FQ_OVF entries per tile behind the lines.
// History: a fixed 1 KiB slot per tile (round 3-4) left a partial line per tile;
// round 5 appended each workgroup's arrays to a region of its own through an LDS ring flushed in
// whole lines, packed at any entry (the offset in the tile word).  Both run the same as this
// layout on an input buffer the box places well and ~0.2 ms slower on one it places badly
// (profiles/r06/calls/a: 1.866-1.871 against 1.874-1.882 ms on three fast copies, 2.086 against
// 2.102 on the slow one; whole builds 2.005-2.013 against 2.000-2.008, 2.227 against 2.228) --
// this one needs no ring, no regions and no offset field.  Round 5 also dropped: a tile's stores
// issued after the next tile's DMA, two LDS slots per workgroup (4 workgroups per CU), fewer
// records certified per wave, temporal row-start stores (all slower or within noise).
constexpr u32 FQ_LINE_E = 64;                                // u16 entries per line
constexpr u32 FQ_OVF = ((RCAP + 1 - FQ_LINE_E) + 7u) & ~7u;  // overflow entries per tile (16-byte multiple)
__device__ __forceinline__ u64 fq_ovf(const SlabParams &p, u64 t) { return (u64)p.ntiles * FQ_LINE_E + t * FQ_OVF; }
// entry L of tile t (L <= nrec: entry nrec is the end of the tile's last record)
__device__ __forceinline__ u32 fq_start(const SlabParams &p, u64 t, u32 L) {
  const uint16_t *s = reinterpret_cast<const uint16_t *>(p.fq_stage);
  return L < FQ_LINE_E ? s[t * FQ_LINE_E + L] : s[fq_ovf(p, t) + (L - FQ_LINE_E)];
}
constexpr u32 FQ_UNCERT = 0x8000;  // row entry: the record is not certified here
__device__ __forceinline__ u32 *fq_defer(const SlabParams &p, u64 t) { return p.fq_tiles + t * (2 * MAX_DEFER); }

// A workgroup keeps the lines and tile words of FQ_BLK consecutive tiles in LDS, so they leave as
// one 2 KiB burst of lines and one 128-byte line of words per FQ_BLK tiles (profiles/r06/calls/e:
// the kernel 1.872 -> 1.855 ms and the build 1.998 -> 1.982 on each of four input copies, against
// one tile per burst).  The tiles come in batches of FQ_RR consecutive tiles dealt round-robin to
// the workgroups (k_fq_tiles).
constexpr u32 FQ_BLK = 16;
constexpr u64 FQ_RR = 32;
static_assert(FQ_RR % FQ_BLK == 0, "a batch holds whole bursts");
struct __align__(16) TilesSmem {
  uint16_t nlpos[SNLCAP + 8];        // + 8: the certifier reads aligned 8-entry windows
  uint16_t line[FQ_BLK][FQ_LINE_E];  // the batch's lines: a tile's first FQ_LINE_E entries each
  u64 words[FQ_BLK];                 // the batch's tile words
  u32 wtot[SNW];
  u32 nh, ndefer, slow, pad;
};

// entry L of the tile being certified (batch slot j): its line in LDS, or the overflow slot
__device__ __forceinline__ void fq_put(const SlabParams &p, TilesSmem &S, u64 t, u32 j, u32 L, uint16_t v) {
  if (L < FQ_LINE_E) S.line[j][L] = v;
  else __builtin_nontemporal_store(v, reinterpret_cast<uint16_t *>(p.fq_stage) + fq_ovf(p, t) + (L - FQ_LINE_E));
}

template <bool kSpans>
__device__ __forceinline__ void tiles_iter(const SlabParams &p, TilesSmem &S, uint8_t *raw, u64 t, int tid, int lane,
                                           int wid, u64 *tacc, u32 j, bool flush) {
  // diagnostic phase stamps (SIDX_DIAG builds with SHOCKIDX_TIMING; tacc == nullptr otherwise):
  // lane 0 of waves 0 (the certifying wave) and 1 accumulate the cycles of each phase
  u64 tprev = tacc ? stamp() : 0;
#define TILES_STAMP(i)              \
  if (tacc) {                       \
    const u64 tn_ = stamp();        \
    tacc[i] += tn_ - tprev;         \
    tprev = tn_;                    \
  }
  // ---- P0 / P1: DMA of this tile; each wave waits for its own pieces ------------------------
  // wave priorities: a tile's DMA is issued ahead of other workgroups' compute, and a tile's
  // record certification (one wave, the tile's critical path while its other waves wait at the
  // barrier) ahead of other workgroups' mask / position phases -- each workgroup then returns
  // its slot to the DMA sooner (10 GiB: 2.24-2.31 -> 2.09 ms)
  __builtin_amdgcn_s_setprio(3);
  stage_tile<true>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TILES_STAMP(0);
  // the last wave also collects the newlines past the tile: the straggler at the next barrier,
  // so it goes first
  if (wid == SNW - 1) __builtin_amdgcn_s_setprio(1);
  const u64 tlo = t * TILE;
  const u64 thi = (tlo + TILE < p.n) ? tlo + TILE : p.n;
  const u32 tlen = (u32)(thi - tlo);
  const u32 llen = (u32)(((tlo + TILE + SHALO < p.end) ? tlo + TILE + SHALO : p.end) - tlo);
  if (llen < (u32)(TILE + SHALO) || (t == 0 && p.front < FRONT)) {  // slab end / file start: zero-fill
    lds_barrier();  // (every wave's DMA landed: the fill may touch any part of the slot)
    for (u32 c = (u32)tid; c < (u32)((TILE + SHALO) / 16); c += SNT) {
      const u32 o = c * 16;
      if (o + 16 <= llen) continue;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (o < llen) {
        v = keep_bytes(*reinterpret_cast<const uint4 *>(raw + FRONT + o), llen - o);
        if (llen & 3u) {
          u32 ll;
          const auto rs = tile_rsrc(p, t, ll);
          patch_tail(v, o, llen, tail_dword(rs, llen));
        }
      }
      *reinterpret_cast<uint4 *>(raw + FRONT + o) = v;
    }
    if (t == 0 && p.front < FRONT && tid == 0) *reinterpret_cast<uint4 *>(raw) = make_uint4(0, 0, 0, 0);
    lds_barrier();
  }
  // ---- P2: '\n' mask word per thread (swizzled 16-byte reads), block count ----------------
  u64 m = 0;  // 3-op equality flags; the rare suspect word ("\n\v") is re-checked exactly
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
    const uint4 v = *reinterpret_cast<const uint4 *>(raw + FRONT + tid * 64 + 16 * cj);
    m |= (u64)eq16x(v, '\n') << (16 * cj);
  }
  if (eq_suspect(m)) {
    m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) m |= (u64)eq16(*reinterpret_cast<const uint4 *>(raw + FRONT + tid * 64 + 16 * j), '\n') << (16 * j);
  }
  const u32 rl = tlen > (u32)tid * 64 ? tlen - (u32)tid * 64 : 0u;
  const u64 mown = m & lowmask(rl);
  const u32 c = popc64(mown);
  // (fewer VALU instructions per tile -- the pass issues VALU about two thirds of its time: a
  // ballot scan of the small per-lane counts, the wave totals read as scalars, a word's first two
  // positions without the loop, the halo words by the 3-op equality flags; round 5, within noise)
  const u32 incl = wave_scan_add_small(c);
  if (lane == 63) S.wtot[wid] = incl;
  if (tid == 0) { S.ndefer = 0; S.slow = 0; }
  lds_barrier();
  TILES_STAMP(1);
  static_assert(SNW == 4, "the wave totals: one uniform 16-byte LDS read");
  const uint4 w4 = *reinterpret_cast<const uint4 *>(S.wtot);
  const u32 t0 = (u32)__builtin_amdgcn_readfirstlane((int)w4.x), t1 = (u32)__builtin_amdgcn_readfirstlane((int)w4.y),
            t2 = (u32)__builtin_amdgcn_readfirstlane((int)w4.z), t3 = (u32)__builtin_amdgcn_readfirstlane((int)w4.w);
  const u32 T = t0 + t1 + t2 + t3;
  const u32 wpre = (wid > 0 ? t0 : 0u) + (wid > 1 ? t1 : 0u) + (wid > 2 ? t2 : 0u);
  // ---- P3: newline positions (tile + the first NLHALO past it), phase, validation -----------
  const bool use_arr = T + NLHALO <= (u32)SNLCAP;
  if (use_arr) {
    u32 o = wpre + incl - c;
    u64 mm = mown;
    const u64 m1 = mm & (mm - 1);  // a word's first two '\n' without the loop
    if (c >= 1) S.nlpos[o] = (uint16_t)((u32)tid * 64 + ctz64(mm));
    if (c >= 2) S.nlpos[o + 1] = (uint16_t)((u32)tid * 64 + ctz64(m1));
    mm = m1 & (m1 - 1);
    o += 2;
    while (mm) {
      S.nlpos[o++] = (uint16_t)((u32)tid * 64 + ctz64(mm));
      mm &= mm - 1;
    }
    if (wid == SNW - 1) {
      const u32 wb = tlen >> 6;
      u32 hc = 0;
      u64 hm = 0;
      const u32 wd = wb + (u32)lane;
      if (wd * 64 < llen) {
        // this lane's word past the tile's last byte, classified here from the slot (the halo
        // DMA was other waves'; no mask words are kept in LDS)
#pragma unroll
        for (int j = 0; j < 4; ++j) hm |= (u64)eq16x(*reinterpret_cast<const uint4 *>(raw + FRONT + wd * 64 + 16 * j), '\n') << (16 * j);
        if (eq_suspect(hm)) {
          hm = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            hm |= (u64)eq16(*reinterpret_cast<const uint4 *>(raw + FRONT + wd * 64 + 16 * j), '\n') << (16 * j);
        }
        if (wd == wb) hm &= ~lowmask(tlen & 63);
        if (wd * 64 + 64 > llen) hm &= lowmask(llen - wd * 64);
        hc = popc64(hm);
      }
      const u32 hpre = wave_scan_add_small(hc);
      u32 o2 = hpre - hc;
      while (hm && o2 < (u32)NLHALO) {
        S.nlpos[T + o2] = (uint16_t)(wd * 64 + ctz64(hm));
        ++o2;
        hm &= hm - 1;
      }
      if (lane == 63) S.nh = hpre < (u32)NLHALO ? hpre : (u32)NLHALO;
    }
  }
  lds_barrier();
  TILES_STAMP(2);
  const bool fs = p.file_start && t == 0;
  const u32 TT = use_arr ? T + S.nh : 0;
  u32 gi0;
  if (t == 0) gi0 = (u32)((3 - (p.state_in & 3)) & 3);  // slab start: rank known
  else if (use_arr && (wid == 0 || (T + 3) / 4 + 1 > 64u * (u32)wid)) gi0 = fq_guess_at(raw, S.nlpos, TT, lane);
  else gi0 = GUESS_NONE;  // (or this wave has no records to certify: only wave 0's gi0 is kept)
  const u32 ng = gi0 < T ? (T - gi0 + 3) / 4 : 0;
  const u32 nrec = ng + (fs ? 1u : 0u);
  const bool slow = !use_arr || gi0 == GUESS_NONE || nrec > (u32)RCAP;
  u32 *tdef = fq_defer(p, t);
  __builtin_amdgcn_s_setprio(2);
  if (!slow) {
    // record q = 64 w + lane (a tile's ~50 records fit one wave); one LDS round per step
    const uint8_t *r = raw + FRONT;
    for (u32 qb = (u32)wid * 64u; qb < ng + 1; qb += SNW * 64u) {
      const u32 q = qb + (u32)lane;
      const bool inr = q < ng;
      const bool act = inr || (q == ng && fs);
      const u32 d = inr ? gi0 + 4 * q : 0u;
      const u32 i = inr ? d + 1 : 0u;
      const u32 L = inr ? q + (fs ? 1u : 0u) : 0u;
      const bool known = act && i + 3 < TT;
      u32 s0, e0, e1, e2, e3;
      if (!fs) {
        // nlpos[d .. d+4] from two aligned 8-byte reads: d & 3 = gi0 & 3 is the same in every lane
        const u32 db = inr ? (d & ~3u) : 0u;  // s0 is needed even when the record runs past the halo (k_fixup)
        const uint2 wa = *reinterpret_cast<const uint2 *>(&S.nlpos[db]);
        const uint2 wb = *reinterpret_cast<const uint2 *>(&S.nlpos[db + 4]);
        const u32 sh2 = (gi0 & 1u) * 2u;   // byte shift inside a dword
        const bool hiw = (gi0 & 2u) != 0u;  // start in the second dword
        const u32 x0 = hiw ? wa.y : wa.x, x1 = hiw ? wb.x : wa.y, x2 = hiw ? wb.y : wb.x, x3 = hiw ? 0u : wb.y;
        const u32 p01 = __builtin_amdgcn_alignbyte(x1, x0, sh2), p23 = __builtin_amdgcn_alignbyte(x2, x1, sh2),
                  p4 = __builtin_amdgcn_alignbyte(x3, x2, sh2);
        s0 = inr ? (p01 & 0xFFFFu) + 1u : 0u;
        e0 = known ? p01 >> 16 : 0u;
        e1 = known ? p23 & 0xFFFFu : 0u;
        e2 = known ? p23 >> 16 : 0u;
        e3 = known ? p4 & 0xFFFFu : 0u;
      } else {  // the file's first tile: record 0 starts at offset 0, its line ends are entries 0..3
        const u32 ic = known ? i : 0u;
        e0 = S.nlpos[ic]; e1 = S.nlpos[ic + 1]; e2 = S.nlpos[ic + 2]; e3 = S.nlpos[ic + 3];
        s0 = inr ? S.nlpos[d] + 1u : 0u;
      }
      u32 cn = 0, cb = 0, crs = 0;
      bool idclean = false;
      const bool ok = fq_ok(r, s0, e0, e1, e2, e3, cn, cb, crs, idclean) && known;
      bool good = ok;
      const u32 ca = FRONT + s0 + 1;
      cb += FRONT;
      const bool need = ok && cn != 0;
      bool idmis = false;
      {  // plus-line IDs: per lane up to 64 bytes, longer ones by the whole wave
        if (__ballot(need && cn <= 64)) {
          u32 diff = 0;
          const u32 nn = (need && cn <= 64) ? cn : 0u;
          for (u32 o = 0; o < nn; o += 16) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const u32 oo = o + 4 * (u32)j;
              if (oo < nn) diff |= lds_diff4(raw, ca + oo, cb + oo, nn - oo);
            }
          }
          idmis = diff != 0;
        }
        u64 mc = __ballot(need && cn > 64);
        while (mc) {
          const int Lc = (int)ctz64(mc);
          mc &= mc - 1;
          const u32 xa = (u32)__shfl((int)ca, Lc, 64), xb = (u32)__shfl((int)cb, Lc, 64);
          const u32 xn = (u32)__shfl((int)cn, Lc, 64);
          u32 diff = 0;
          for (u32 o = (u32)lane * 4; o < xn; o += 256) diff |= lds_diff4(raw, xa + o, xb + o, xn - o);
          const bool any = __ballot(diff != 0) != 0;
          if (lane == Lc) idmis = any;
        }
      }
      if (idmis) good = false;
      // a blank group right after four '\n' follows a group that already ended the records
      // (fastq.go:143-163 and fastq_record's DONTCARE rule): nothing to validate there
      const bool dontcare = known && !good && e0 == s0 && r[s0 - 1] == '\n' && r[s0 - 2] == '\n' &&
                            r[s0 - 3] == '\n' && r[s0 - 4] == '\n';
      if (!act) continue;
      fq_put(p, S, t, j, L, (uint16_t)(s0 | (good ? 0u : FQ_UNCERT)));
      if (kSpans && good) {  // the record's inner line ends for the filters' spans (0xFFFF: trim the ID globally)
        uint16_t *ln = p.fq_lines + t * (3 * RCAP) + 3 * L;
        ln[0] = (uint16_t)(idclean ? (e0 | ((crs & 1u) << 15)) : 0xFFFFu);
        ln[1] = (uint16_t)(e1 | ((crs & 2u) << 14));
        ln[2] = (uint16_t)(e2 | ((crs & 4u) << 13));
      }
      if (L + 1 == nrec && known) fq_put(p, S, t, j, nrec, (uint16_t)(e3 + 1));  // the end of the tile's last record
      if (!good && !dontcare) {  // anything but a certified record: k_fixup validates it from global memory
        const u32 slot = atomicAdd(&S.ndefer, 1u);
        if (slot < (u32)MAX_DEFER) { tdef[slot] = L; tdef[MAX_DEFER + slot] = s0; }
        else S.slow = 1;
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
  TILES_STAMP(3);
  lds_barrier();  // S.ndefer / S.slow / S.line final; the slot and the newline arrays are reused next
  TILES_STAMP(4);
  const u64 word = fq_word(T, gi0, nrec, slow || S.slow, S.ndefer < (u32)MAX_DEFER ? S.ndefer : (u32)MAX_DEFER);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  {
    // the batch's lines and words leave together after its last tile, from wave 0 (the next
    // batch writes slot 0 only after two more barriers); the lines are read once, by k_fq_place:
    // non-temporal.  (A slow or empty tile's line is never read.)
    if (tid == 0) S.words[j] = word;
    if (flush && wid == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const u64 t0 = t - j;
      for (u32 c = (u32)lane; c < (j + 1) * (FQ_LINE_E / 8); c += 64) {
        const v4u v = *reinterpret_cast<const v4u *>(&S.line[0][0] + 8 * c);
        __builtin_nontemporal_store(v, (__attribute__((address_space(1))) v4u *)(reinterpret_cast<uint16_t *>(p.fq_stage) +
                                                                                 t0 * FQ_LINE_E + 8 * c));
      }
      if ((u32)lane * 2 < j + 1) {  // the words, 16 bytes per lane (a last odd word alone)
        if ((u32)lane * 2 + 1 < j + 1) {
          const v4u v = *reinterpret_cast<const v4u *>(&S.words[2 * lane]);
          *(__attribute__((address_space(1))) v4u *)(p.fq_agg + t0 + 2 * lane) = v;
        } else {
          p.fq_agg[t0 + 2 * lane] = S.words[2 * lane];
        }
      }
    }
  }
  TILES_STAMP(5);
#undef TILES_STAMP
}

// Persistent grid-stride over batches of tiles, one LDS slot per workgroup (each tile is staged,
// certified and stored before the next is DMA'd; 7 workgroups per CU keep the DMA busy); no waits
// on other workgroups, so the grid need not be co-resident.
#ifndef SIDX_TILES_WGS
#define SIDX_TILES_WGS 7  // 19.5 KiB of LDS: 8 would fit, but at <= 64 VGPRs (41 SGPR spills) it ran 1.6 % slower
#endif
template <bool kSpans>
__global__ __launch_bounds__(SNT, SIDX_TILES_WGS) void k_fq_tiles(const SlabParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[SSLOT];
  __shared__ TilesSmem S;
  if (gated_off(p)) return;  // format speculation failed: the host re-runs with the detected format
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 G = p.pgrid;
  u64 tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 *tacc = (tmg(p) && (tid == 0 || tid == 64)) ? tacc_ : nullptr;
  u64 ntl = 0;
  // batches of FQ_RR consecutive tiles dealt round-robin to the workgroups (a tile's halo, the
  // first KiB of the next tile, is read again by the same workgroup through its own L2 except at a
  // batch's end).  Where the workgroups' concurrent streams sit in the input decides how fast
  // they run together: in one process over the C2 input (profiles/r06/calls/j/ab_fq_rr*.json, every
  // table hashed and equal) batches of 32 ran 1.834-2.034 ms where a contiguous block of 368
  // tiles per workgroup (round 6 before) ran 1.987-2.118, faster on each of eight input copies
  // over three boxes; batches of 8, 16, 24, 48 or 64, or a last round split evenly, all ran slower than 32
  const u64 nbat = (p.ntiles + FQ_RR - 1) / FQ_RR;
  for (u64 c = blockIdx.x; c < nbat; c += G) {
    const u64 tb = c * FQ_RR, te = tb + FQ_RR < p.ntiles ? tb + FQ_RR : p.ntiles;
    for (u64 t = tb; t < te; ++t) {
      const u32 j = (u32)(t - tb) & (FQ_BLK - 1);  // (bursts start at even tiles: the words leave 16 bytes per lane)
      tiles_iter<kSpans>(p, S, raw, t, tid, lane, wid, tacc, j, j == FQ_BLK - 1 || t + 1 == te);
      ++ntl;
    }
  }
  if (tacc) {  // per workgroup: wave 0's phases in slots 0-5, wave 1's in the next 9-slot record
    u64 *o = tmg(p) + ((u64)blockIdx.x * 2 + (tid ? 1 : 0)) * 9;
    for (int i = 0; i < 8; ++i) o[i] = tacc[i];
    o[8] = ntl;
  }
}

// ====================================================================================
// Line index tile pass (line.go:37-45 + index/line.go:33-85, single-slab builds): every '\n'
// ends a row, so a tile needs only its line-number base (scan of the tile counts) and the
// last '\n' before it (a max scan).  k_line_tiles reads the input once: per tile the count,
// the last '\n' and the tile-relative '\n' positions (u16, up to LCAP per tile); k_line_place
// writes the rows (one wave per tile; a tile with more than LCAP lines -- lines under 16 B on
// average -- is rescanned from global memory); k_line_final the last row (the bytes after the
// last '\n', possibly empty: Create always emits it).
// ====================================================================================
constexpr u32 LCAP = TILE / 16;
// Where a tile's positions go: each workgroup of the persistent grid appends its tiles' position
// arrays back to back (16-byte aligned) into its own region of the stage buffer, so the stores of
// consecutive tiles fill whole cache lines; fq_agg[t] = count | the array's offset (16-byte
// units) << 32.  (Fixed 2 KiB slots per tile left a partial line per tile: ablating the stores
// took 0.23-0.37 ms off the kernel, profiles/r04/ab_line_tiles_ablations.txt.)  The region of the
// workgroup whose first tile is t0 starts where t0's would in tile order, t0 * q + min(t0, r)
// tiles in (ntiles = q G + r), and holds LCAP entries per tile it processes.
constexpr u64 LOFF_SHIFT = 32, LCOUNT = (1ull << LOFF_SHIFT) - 1;
#ifndef SIDX_LINE_WGS
#define SIDX_LINE_WGS 7  // workgroups per CU (the slot holds no halo: up to 9 fit the LDS)
#endif
__global__ __launch_bounds__(SNT, SIDX_LINE_WGS) void k_line_tiles(const SlabParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[FRONT + TILE];
  __shared__ __attribute__((aligned(16))) uint16_t sp[LCAP];  // the tile's '\n' positions, stored out whole
  __shared__ u32 wtot[SNW], wlast[SNW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 G = p.pgrid;
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  uint4 *stage16 = reinterpret_cast<uint4 *>(p.fq_stage);
  u64 wofs = (t * (p.ntiles / G) + (t < p.ntiles % G ? t : p.ntiles % G)) * (LCAP / 8);  // 16-byte units
  // A tile's stores leave after the next tile's DMA is issued: vmcnt counts a wave's stores as
  // well as its loads, in issue order, so stores issued before the DMA would be waited for with it
  // (1.768 against 1.778 ms with the stores first, on each of 4 input copies, profiles/r05/calls/r05n)
  u64 pt = ~0ull, pword = 0, ppcnt = 0, pwofs = 0;
  u32 pT = 0;
  auto flush_pending = [&]() -> u32 {  // this wave's store instructions (uniform per wave)
    if (pt == ~0ull) return 0u;
    u32 n = 0;
    if (wid == 0) {
      if (tid == 0) {
        p.fq_agg[pt] = pword;
        p.pcnt[pt] = ppcnt;
      }
      n = 2;
    }
    if (pT <= LCAP && (u32)wid * 512u < pT) {  // (lanes tid * 8 < pT)
      if ((u32)tid * 8 < pT) {
        typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
        const uint4 x = *reinterpret_cast<const uint4 *>(&sp[8 * tid]);
        *reinterpret_cast<v4u_t *>(stage16 + pwofs + (u64)tid) = (v4u_t){x.x, x.y, x.z, x.w};
      }
      ++n;
    }
    pt = ~0ull;
    return n;
  };
  for (; t < p.ntiles; t += G) {
    __builtin_amdgcn_s_setprio(3);
    stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);
    __builtin_amdgcn_s_setprio(0);
    {  // a wave reads only the bytes it staged: wait for its DMA, not for the stores behind it
      const u32 nst = flush_pending();
      if (nst == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (nst == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else if (nst == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    }
    const u64 tlo = t * TILE;
    const u32 tlen = (u32)(((tlo + TILE < p.n) ? tlo + TILE : p.n) - tlo);
    u64 m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
      m |= (u64)eq16x(*reinterpret_cast<const uint4 *>(raw + FRONT + tid * 64 + 16 * cj), '\n') << (16 * cj);
    }
    if (eq_suspect(m)) {  // "\n\v" inside a dword: the exact mask
      m = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) m |= (u64)eq16(*reinterpret_cast<const uint4 *>(raw + FRONT + tid * 64 + 16 * j), '\n') << (16 * j);
    }
    const u32 rl = tlen > (u32)tid * 64 ? tlen - (u32)tid * 64 : 0u;
    m &= lowmask(rl);  // bytes past the slab end were zero-filled or are not this tile's
    // the DMA range check is per dword: a partial last dword of the input came back as zeros
    if (tlen < (u32)TILE && (tlen & 3u) && (u32)tid == ((tlen - 1) >> 6))
      for (u32 i = tlen & ~3u; i < tlen; ++i) m |= (u64)(p.data[tlo + i] == '\n') << (i - (u32)tid * 64);
    const u32 c = popc64(m);
    const u32 incl = wave_scan_add(c);
    const u32 last = m ? (u32)tid * 64 + 64 - clz64(m) : 0u;  // tile-relative '\n' + 1
    const u64 lb = __ballot(m != 0);
    const u32 lmx = lb ? (u32)__builtin_amdgcn_readlane((int)last, 63 - (int)clz64(lb)) : 0u;  // the wave's last
    if (lane == 63) { wtot[wid] = incl; wlast[wid] = lmx; }
    lds_barrier();
    u32 wpre = 0, T = 0, L = 0;
#pragma unroll
    for (int w = 0; w < SNW; ++w) {
      const u32 x = wtot[w];
      if (w < wid) wpre += x;
      T += x;
      L = L > wlast[w] ? L : wlast[w];
    }
    // the positions go through LDS and leave as whole 16-byte stores (scattered 2-byte global
    // stores cost several times their bytes next to the stream); raw is not read past the
    // barrier above, wtot / sp are rewritten only after the next tile's first barrier
    if (T <= LCAP) {
      u32 o = wpre + incl - c;
      u64 mm = m;
      while (mm) {
        sp[o++] = (uint16_t)((u32)tid * 64 + ctz64(mm));
        mm &= mm - 1;
      }
    }
    pt = t;
    pword = (u64)T | (wofs << LOFF_SHIFT);
    ppcnt = L ? tlo + L : (u64)0;  // last '\n' + 1 (absolute), 0: none in the tile
    pwofs = wofs;
    pT = T;
    lds_barrier();
    if (T <= LCAP) wofs += (T + 7) / 8;
  }
  (void)flush_pending();  // the last tile's
}

// The rows of the '\n's in [a, a + 64 * 64) of the tile (wave; lanes take 64-byte words in
// order): line k ends at its '\n', starts after the previous one (`carry` = previous '\n' + 1
// before the range).  Returns the new carry and advances k.
__device__ u64 line_rows_wave(const SlabParams &p, u64 a, u64 hi, u64 carry, u64 &k, int lane) {
  const u64 w = a + 64ull * (u64)lane;
  u64 m = 0;
  if (w < hi) {
    const u64 lim = hi - w < 64 ? hi - w : 64;
    if (lim == 64) {
#pragma unroll
      for (int j = 0; j < 4; ++j) m |= (u64)eq16(load16(p.data + w + 16 * j), '\n') << (16 * j);
    } else {
      for (u64 i = 0; i < lim; ++i) m |= (u64)(p.data[w + i] == '\n') << i;
    }
  }
  const u32 c = popc64(m);
  const u32 incl = wave_scan_add(c);
  const u64 lst = m ? w + 64 - clz64(m) : 0;
  u64 pm = lst;
  for (int d = 1; d < 64; d <<= 1) {
    const u64 y = __shfl_up(pm, d, 64);
    if (lane >= d) pm = pm > y ? pm : y;
  }
  u64 before = __shfl_up(pm, 1, 64);
  if (lane == 0) before = 0;
  u64 start = before > carry ? before : carry;
  u64 kk = k + incl - c;
  while (m) {
    const u64 pos = w + ctz64(m);
    m &= m - 1;
    put_row(p, kk++, start, pos + 1 - start);
    start = pos + 1;
  }
  const u64 tot = (u64)__shfl((int)incl, 63, 64);
  const u64 newc = __shfl(pm, 63, 64);
  k += tot;
  return newc > carry ? newc : carry;
}

// k_line_place: 32 consecutive tiles per workgroup (round 3: one wave per tile, two dependent
// global round trips per wave).  Wave 0 reads the tiles' counts, row bases and carried line
// starts and scans the rows and 16-byte chunks of '\n' positions of the tiles that kept them;
// all lanes stage those chunks in LDS, all in flight together; thread r then writes row r of the
// workgroup's run (its tile by a two-level search of the row prefixes), so the row stores are
// 4 KiB per instruction.  Dense tiles (more than LCAP lines) are rescanned from global memory,
// one wave each; a batch whose positions do not fit LPLACE_ECAP entries places its tiles one
// per wave from global memory.
// SAM (F == F_SAM, k_sam_tiles): the staged positions are the tile's terminator '\n's, the
// first one possibly not a terminator (settled by k_sam_resolve: fq_tiles bit 30); rows end at
// terminators, the row base is the SamMonoid count before the tile, dense tiles re-run two-pass.
constexpr int LPLACE_TILES = 32;
constexpr u32 LPLACE_ECAP = 12288;  // u16 '\n' positions staged per workgroup (24 KiB)
constexpr u32 SAM_HASNL = 1u << 31, SAM_FIRST_TERM = 1u << 30, SAM_DMASK = SAM_FIRST_TERM - 1;
template <int F>
__global__ __launch_bounds__(256) void k_line_place(const SlabParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t ent[LPLACE_ECAP];
  __shared__ __attribute__((aligned(16))) uint16_t sR[LPLACE_TILES + 8];  // first row of each tile in the run
  __shared__ __attribute__((aligned(16))) uint16_t sC[8];                 // sR[8 j]
  __shared__ u32 sE[LPLACE_TILES + 1];
  __shared__ u64 sB[LPLACE_TILES], sCar[LPLACE_TILES];
  __shared__ uint8_t sO[LPLACE_TILES];  // SAM: 1 when the tile's first staged '\n' is not a terminator
  __shared__ u64 sOff[LPLACE_TILES];    // the tile's position array in the stage buffer (16-byte units)
  __shared__ u32 sDense, sTot;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint16_t *stage = reinterpret_cast<const uint16_t *>(p.fq_stage);
  for (u64 t0 = (u64)blockIdx.x * LPLACE_TILES; t0 < p.ntiles; t0 += (u64)gridDim.x * LPLACE_TILES) {
    if (wid == 0) {
      const u64 t = t0 + (u64)lane;
      const bool valid = lane < LPLACE_TILES && t < p.ntiles;
      u32 rows = 0, chunks = 0;
      bool dense = false;
      if (valid && F == F_SAM) {
        const u32 w = p.fq_tiles[t], D = w & SAM_DMASK;
        const u32 o = ((w & SAM_HASNL) && !(w & SAM_FIRST_TERM)) ? 1u : 0u;
        sB[lane] = SamMonoid::apply(p.state_in, p.tile_excl[t]) >> 2;
        sCar[lane] = p.ppre[t];
        sO[lane] = (uint8_t)o;
        sOff[lane] = t * (LCAP / 8);  // (k_sam_tiles: one fixed slot per tile)
        if (D <= LCAP) {  // (dense tiles: the build re-runs two-pass, k_sam_tiles flagged it)
          rows = D - o;
          chunks = (D + 7) / 8;
        }
      } else if (valid) {
        const u64 w = p.fq_agg[t], T = w & LCOUNT;
        sOff[lane] = w >> LOFF_SHIFT;
        // row k ends at '\n' number k (rows before the slab: state_in); a slab after the first
        // drops the row open at its start through row_base (put_row)
        sB[lane] = p.state_in + p.tile_excl[t];
        sCar[lane] = p.ppre[t];
        sO[lane] = 0;
        dense = T > LCAP;
        rows = dense ? 0u : (u32)T;
        chunks = (rows + 7) / 8;
      }
      const u32 ri = wave_scan_add(rows), ci = wave_scan_add(chunks);
      const u64 db = __ballot(dense);
      if (lane <= LPLACE_TILES) {
        sR[lane] = (uint16_t)(ri - rows);
        sE[lane] = 8u * (ci - chunks);
        if ((lane & 7) == 0 && lane < LPLACE_TILES) sC[lane >> 3] = (uint16_t)(ri - rows);
      }
      if (lane == 0) sDense = (u32)db;
      if (lane == LPLACE_TILES - 1) sTot = ri;
    }
    __syncthreads();
    const u32 R = sTot, E = sE[LPLACE_TILES];
    if (E <= LPLACE_ECAP) {
      // 8 lanes per tile: chunks c, c + 8, ... of its positions, two loads in flight per step
      const int k = tid >> 3;
      const u32 e0 = sE[k], nch = (sE[k + 1] - e0) >> 3;
      const uint4 *src = reinterpret_cast<const uint4 *>(stage) + sOff[k];
      u32 c = (u32)(tid & 7);
      for (; c + 8 < nch; c += 16) {
        const uint4 a = src[c], b = src[c + 8];
        *reinterpret_cast<uint4 *>(&ent[e0 + 8 * c]) = a;
        *reinterpret_cast<uint4 *>(&ent[e0 + 8 * (c + 8)]) = b;
      }
      if (c < nch) *reinterpret_cast<uint4 *>(&ent[e0 + 8 * c]) = src[c];
      __syncthreads();
      const uint2 cw = *reinterpret_cast<const uint2 *>(sC);
      const u32 c1 = cw.x >> 16, c2 = cw.y & 0xFFFFu, c3 = cw.y >> 16;
      for (u32 r = (u32)tid; r < R; r += 256) {
        const u32 g = (c1 <= r ? 1u : 0u) + (c2 <= r ? 1u : 0u) + (c3 <= r ? 1u : 0u);
        const uint4 fw = *reinterpret_cast<const uint4 *>(&sR[8 * g]);
        const u32 fv[8] = {fw.x & 0xFFFFu, fw.x >> 16, fw.y & 0xFFFFu, fw.y >> 16,
                           fw.z & 0xFFFFu, fw.z >> 16, fw.w & 0xFFFFu, fw.w >> 16};
        u32 kk = 8 * g;
#pragma unroll
        for (int j = 1; j < 8; ++j) kk += (8 * g + (u32)j < (u32)LPLACE_TILES && fv[j] <= r) ? 1u : 0u;
        const u32 L = r - (u32)sR[kk];
        const u32 e = sE[kk] + (u32)sO[kk] + L;
        const u64 tlo = (t0 + kk) * TILE;
        const u32 pos = ent[e];
        const u64 start = L ? tlo + ent[e - 1] + 1 : sCar[kk];
        put_row(p, sB[kk] + L, start, tlo + pos + 1 - start);
      }
    } else {
      for (int k = wid; k < LPLACE_TILES; k += 4) {
        const u32 T = (u32)sR[k + 1] - (u32)sR[k];
        if (!T) continue;
        const uint16_t *st = stage + sOff[k] * 8 + sO[k];
        const u64 tlo = (t0 + k) * TILE;
        for (u32 L = (u32)lane; L < T; L += 64) {
          const u64 start = L ? tlo + st[L - 1] + 1 : sCar[k];
          put_row(p, sB[k] + L, start, tlo + st[L] + 1 - start);
        }
      }
    }
    // dense tiles: rescanned from global memory, one wave each
    for (u32 dm = F == F_LINE ? sDense : 0u; dm; dm &= dm - 1) {
      const int k = (int)__builtin_ctz(dm);
      if ((k & 3) != wid) continue;
      const u64 tlo = (t0 + k) * TILE;
      const u64 hi = (tlo + TILE < p.n) ? tlo + TILE : p.n;
      u64 kr = sB[k], cr = sCar[k];
      for (u64 a = tlo; a < hi; a += 64 * 64) cr = line_rows_wave(p, a, hi, cr, kr, lane);
    }
    __syncthreads();
  }
}

// ppre = exclusive max scan of pcnt (done by the caller): the last row, after the last '\n'
// (index/line.go:33-85 emits it even when empty).  A slab with a halo closes it at the first
// '\n' of the halo (one wave, 1 KiB per step), else at EOF; a halo that ends neither the row
// nor the file is ST_NEEDMORE.  A slab
// with no '\n' at all holds no row of its own (its bytes belong to the row of an earlier slab).
__global__ void k_line_final(const SlabParams p) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x >= 64 || blockIdx.x) return;
  const u64 t = p.ntiles - 1;
  const u64 c = p.pcnt[t] > p.ppre[t] ? p.pcnt[t] : p.ppre[t];  // last '\n' + 1 of the slab
  const u64 k = p.state_in + p.tile_excl[t] + (p.fq_agg[t] & LCOUNT);
  if (c == 0 && !p.file_start) return;
  for (u64 c0 = p.n & ~15ull; c0 < p.end; c0 += 1024) {  // a slab with a halo: its first '\n'
    const u64 a = c0 + 16ull * (u64)lane;
    u32 m = 0;
    if (a < p.end) {
      m = eq16((a + 16 <= p.end) ? load16(p.data + a) : load16_partial(p.data, a, p.end), '\n');
      if (a < p.n) m &= ~((1u << (u32)(p.n - a)) - 1u);
    }
    const u64 hb = __ballot(m != 0);
    if (hb) {
      const int L = (int)ctz64(hb);
      const u64 q = c0 + 16ull * (u64)L + (u32)__shfl((int)(m ? (u32)__builtin_ctz(m) : 0u), L, 64);
      if (lane == 0) put_row(p, k, c, q + 1 - c);
      return;
    }
  }
  if (p.eof) {  // the bytes after the last '\n' of the file
    if (lane == 0) put_row(p, k, c, p.end - c);
    return;
  }
  if (lane == 0) g_min64(p.badkey, (k << KEY_REC_SHIFT) | ((u64)(t & ((1u << KEY_TILE_BITS) - 1)) << 4) | ST_NEEDMORE);
}

// ====================================================================================
// SAM tile pass (sam.go:83-98 GetReadOffset, single-slab builds): a record ends at the '\n' of
// a "terminator" line -- longer than the '\n' alone, first byte not '@' -- and the next record
// starts after it; header and blank lines belong to the record that follows them.  One read of
// the input, as the line pass:
//   k_sam_tiles    per tile the SamMonoid aggregate (the two-pass build's tile aggregate), the
//                  tile's first '\n' and every later terminator '\n' (u16, a line that starts in
//                  the tile is classed from LDS), the last of those + 1
//   SamMonoid scan -> each tile's incoming state: terminators before it, open-line class
//   k_sam_resolve  the first '\n' of a tile: a terminator iff the open line is a data line, or
//                  the tile starts a line whose first byte is neither '\n' nor '@'
//   max scan       of the last terminator + 1 -> each tile's first row start
//   k_line_place<F_SAM>, k_sam_final (the bytes after the last terminator, a row when not empty;
//                  else no record: ST_ABSENT, as sam_record at EOF)
// A tile with more than LCAP '\n's (lines under 16 bytes on average) makes the build re-run
// two-pass (counters[3] bit 0, as a k_fixup overflow).
// ====================================================================================
__global__ __launch_bounds__(SNT, SIDX_LINE_WGS) void k_sam_tiles(const SlabParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[FRONT + TILE];
  __shared__ __attribute__((aligned(16))) uint16_t sp[LCAP];
  __shared__ u32 wlast[SNW], wtot[SNW], wkeep[SNW];
  __shared__ u64 wagg[SNW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 G = p.pgrid;
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  uint16_t *stage = reinterpret_cast<uint16_t *>(p.fq_stage);
  for (; t < p.ntiles; t += G) {
    __builtin_amdgcn_s_setprio(3);
    stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a wave reads only the bytes it staged
    const u64 tlo = t * TILE;
    const u32 tlen = (u32)(((tlo + TILE < p.n) ? tlo + TILE : p.n) - tlo);
    const uint8_t *b = raw + FRONT;
    u64 m = 0, at = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = *reinterpret_cast<const uint4 *>(b + tid * 64 + 16 * j);
      m |= (u64)eq16(v, '\n') << (16 * j);
      at |= (u64)eq16(v, '@') << (16 * j);
    }
    const u32 rl = tlen > (u32)tid * 64 ? tlen - (u32)tid * 64 : 0u;
    // the DMA range check is per dword: a partial last dword of the input came back as zeros
    if (tlen < (u32)TILE && (tlen & 3u) && (u32)tid == ((tlen - 1) >> 6))
      for (u32 i = tlen & ~3u; i < tlen; ++i) {
        const uint8_t c = p.data[tlo + i];
        m |= (u64)(c == '\n') << (i - (u32)tid * 64);
        at |= (u64)(c == '@') << (i - (u32)tid * 64);
      }
    m &= lowmask(rl);
    at &= lowmask(rl);
    const u32 len = rl < 64 ? rl : 64u;
    const u64 wi = wave_incl_scan<SamMonoid>(SamMonoid::seg(m, at, len), lane);
    // previous '\n' + 1 before this thread's word, inside the tile (0: none)
    const u32 last = m ? (u32)tid * 64 + 64 - clz64(m) : 0u;
    u32 pm = last;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = (u32)__shfl_up((int)pm, d, 64);
      if (lane >= d) pm = pm > y ? pm : y;
    }
    u32 before = (u32)__shfl_up((int)pm, 1, 64);
    if (lane == 0) before = 0;
    if (lane == 63) { wlast[wid] = pm; wagg[wid] = wi; }
    lds_barrier();
    for (int w = 0; w < wid; ++w) before = before > wlast[w] ? before : wlast[w];
    // the thread's kept '\n's: the tile's first one (settled later) and every terminator whose
    // line starts in the tile
    u64 keep = 0;
    u32 lk = 0;  // last terminator + 1 (tile-relative), the first '\n' excluded
    {
      u32 pp = before;
      for (u64 mm = m; mm; mm &= mm - 1) {
        const u32 q = (u32)tid * 64 + ctz64(mm);
        if (!pp) {
          keep |= 1ull << (q & 63);
        } else if (pp < q && b[pp] != '@') {
          keep |= 1ull << (q & 63);
          lk = q + 1;
        }
        pp = q + 1;
      }
    }
    const u32 c = popc64(keep);
    const u32 incl = wave_scan_add(c);
    const u64 kb = __ballot(lk != 0);
    const u32 lkw = kb ? (u32)__builtin_amdgcn_readlane((int)lk, 63 - (int)clz64(kb)) : 0u;
    if (lane == 63) { wtot[wid] = incl; wkeep[wid] = lkw; }
    lds_barrier();
    u32 wpre = 0, D = 0, LK = 0, anynl = 0;
    u64 agg = SamMonoid::identity();
#pragma unroll
    for (int w = 0; w < SNW; ++w) {
      const u32 x = wtot[w];
      if (w < wid) wpre += x;
      D += x;
      LK = LK > wkeep[w] ? LK : wkeep[w];
      anynl |= wlast[w];
      agg = SamMonoid::combine(agg, wagg[w]);
    }
    if (D <= LCAP) {
      u32 o = wpre + incl - c;
      for (u64 kk = keep; kk; kk &= kk - 1) sp[o++] = (uint16_t)((u32)tid * 64 + ctz64(kk));
    }
    if (tid == 0) {
      p.fq_agg[t] = agg;
      p.pcnt[t] = LK ? tlo + LK : 0;
      p.fq_tiles[t] = D | (anynl ? SAM_HASNL : 0u);
      if (D > LCAP) atomicOr(&p.counters[3], 1u);  // dense tile: re-run two-pass
    }
    lds_barrier();
    if (D <= LCAP && (u32)tid * 8 < D)
      reinterpret_cast<uint4 *>(stage + t * LCAP)[tid] = *reinterpret_cast<const uint4 *>(&sp[8 * tid]);
  }
}

// The first '\n' of every tile: a terminator iff the line open at the tile start is a data line
// (SamMonoid state 1), or the tile starts a line (state 0) whose first byte is neither '\n' nor
// '@' (the monoid's dF).  A tile whose only terminator it is takes its end as its last one.
__global__ void k_sam_resolve(const SlabParams p) {
  const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.ntiles) return;
  const u32 w = p.fq_tiles[t];
  if (!(w & SAM_HASNL) || (w & SAM_DMASK) > LCAP) return;
  const u32 st = (u32)(SamMonoid::apply(p.state_in, p.tile_excl[t]) & 3);
  const u64 tlo = t * TILE;
  const u32 b0 = p.data[tlo];
  if (!(st == 1 || (st == 0 && b0 != '\n' && b0 != '@'))) return;
  p.fq_tiles[t] = w | SAM_FIRST_TERM;
  if (!p.pcnt[t]) p.pcnt[t] = tlo + reinterpret_cast<const uint16_t *>(p.fq_stage)[t * LCAP] + 1;
}

// The record after the last terminator: the rest of the file, or none when nothing is left
// (sam_record at EOF: ST_ABSENT, so the count is the number of terminators).
__global__ void k_sam_final(const SlabParams p) {
  if (threadIdx.x || blockIdx.x) return;
  const u64 t = p.ntiles - 1;
  const u64 c = p.pcnt[t] > p.ppre[t] ? p.pcnt[t] : p.ppre[t];  // last terminator + 1 (0: none)
  const u64 k = SamMonoid::apply(p.state_in, SamMonoid::combine(p.tile_excl[t], p.fq_agg[t])) >> 2;
  if (p.end > c) put_row(p, k, c, p.end - c);
  else g_min64(p.badkey, (k << KEY_REC_SHIFT) | ((u64)(t & ((1u << KEY_TILE_BITS) - 1)) << 4) | ST_ABSENT);
}

// k_fq_place: 64 consecutive tiles per workgroup, in three steps with one global round trip
// each (round 3 placed a tile per wave at a time, two dependent u16 loads before every row
// store: 16 serial load latencies per wave, 0.17 ms at C2).
//  1. wave 0, lane k = tile t0 + k: the tile's word and scan prefix decide it -- its rows when
//     the phase read off the tile was right, else the whole tile to k_fixup; a wave scan of the
//     placed tiles' record counts gives each tile its first row in the workgroup's run, a scan of
//     their 16-byte chunks of u16 starts its place in LDS;
//  2. every lane loads 16-byte chunks of the tiles' start arrays into LDS, all in flight together;
//  3. thread r writes row r of the workgroup's run (its tile by a two-level search of the row
//     prefixes: one 16-byte LDS read of every 8th prefix, one of the 8 in that group), so each
//     store instruction writes 4 KiB of consecutive rows.
// A batch whose starts do not fit PLACE_ECAP entries (records under ~140 bytes) places its tiles
// one per wave from global memory instead.
constexpr int PLACE_TILES = 64;
constexpr u32 PLACE_ECAP = 8192;  // u16 starts staged per workgroup (16 KiB)
__global__ __launch_bounds__(256) void k_fq_place(const SlabParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t ent[PLACE_ECAP];
  __shared__ __attribute__((aligned(16))) uint16_t sR[PLACE_TILES + 8];  // first row of each tile (+ total)
  __shared__ __attribute__((aligned(16))) uint16_t sC[8];                // sR[8 j]
  __shared__ u32 sE[PLACE_TILES + 1];                                    // first LDS entry of each tile
  __shared__ u64 sG[PLACE_TILES];                                        // global number of local record 0
  if (gated_off(p)) return;  // format speculation failed: the host re-runs with the detected format
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (u64 t0 = (u64)blockIdx.x * PLACE_TILES; t0 < p.ntiles; t0 += (u64)gridDim.x * PLACE_TILES) {
    if (wid == 0) {
      const u64 t = t0 + (u64)lane;
      u32 rows = 0, chunks = 0;
      u64 gbase = 0;
      if (t < p.ntiles) {
        const u64 w = p.fq_agg[t];
        const u32 Te = (u32)(w >> FQW_T) & 0xFFFFu;
        const u32 gi = (u32)(w >> FQW_GI) & 7u;
        const u32 i0 = gi == 7u ? GUESS_NONE : gi;
        const u32 nrec = (u32)(w >> FQW_NREC) & FQW_NRECM;
        const u32 nd = (u32)(w >> FQW_NDEF) & 0x1Fu;
        const u64 j0 = p.state_in + p.tile_excl[t];
        const u32 ti0 = (u32)((3 - (j0 & 3)) & 3);
        const bool fs = p.file_start && t == 0;
        const u32 ngt = ti0 < Te ? (Te - ti0 + 3) / 4 : 0;
        const u32 ngg = i0 < Te ? (Te - i0 + 3) / 4 : 0;
        const bool redo = ((w >> FQW_SLOW) & 1u) || (i0 != ti0 && (ngt | ngg) != 0);
        if (!redo) {
          gbase = ((j0 + ti0 + 1) >> 2) - (fs ? 1u : 0u);
          rows = nrec;
          // starts 0..nrec (entry nrec: the last record's end): the tile's line, then its overflow
          chunks = nrec ? (nrec + 8) / 8 : 0u;
          if (nd) {
            const u32 *tdef = fq_defer(p, t);
            for (u32 i = 0; i < nd; ++i) push_fix(p, t * TILE + tdef[MAX_DEFER + i], gbase + tdef[i], (u32)t);
          }
        } else {
          push_fix(p, ~0ull, j0, (u32)t);  // whole tile, true rank j0
        }
      }
      const u32 ri = wave_scan_add(rows), ci = wave_scan_add(chunks);
      sR[lane] = (uint16_t)(ri - rows);
      sE[lane] = 8u * (ci - chunks);  // the tile's entry 0 (its chunks staged from there)
      sG[lane] = gbase;
      if ((lane & 7) == 0) sC[lane >> 3] = (uint16_t)(ri - rows);
      if (lane == 63) { sR[PLACE_TILES] = (uint16_t)ri; sE[PLACE_TILES] = 8u * ci; }
    }
    __syncthreads();
    const u32 R = sR[PLACE_TILES], E = sE[PLACE_TILES];
    if (E <= PLACE_ECAP) {
      // step 2: lanes 4 k' .. 4 k' + 3 of wave w stage tile 16 w + k' (chunks c, c + 4, ...)
      const int k = wid * 16 + (lane >> 2);
      const u32 e0 = sE[k], nch = (sE[k + 1] - e0) >> 3;
      const u64 tk = t0 + (u64)k;
      // chunks 0..7: the tile's line; 8..: its overflow slot (two loads in flight per step)
      const uint4 *ln = reinterpret_cast<const uint4 *>(reinterpret_cast<const uint16_t *>(p.fq_stage) + tk * FQ_LINE_E);
      const uint4 *ov = reinterpret_cast<const uint4 *>(reinterpret_cast<const uint16_t *>(p.fq_stage) + fq_ovf(p, tk)) -
                        FQ_LINE_E / 8;
      u32 c = (u32)(lane & 3);
      for (; c + 4 < nch; c += 8) {
        const uint4 a = c < FQ_LINE_E / 8 ? ln[c] : ov[c], b = c + 4 < FQ_LINE_E / 8 ? ln[c + 4] : ov[c + 4];
        *reinterpret_cast<uint4 *>(&ent[e0 + 8 * c]) = a;
        *reinterpret_cast<uint4 *>(&ent[e0 + 8 * (c + 4)]) = b;
      }
      if (c < nch) *reinterpret_cast<uint4 *>(&ent[e0 + 8 * c]) = c < FQ_LINE_E / 8 ? ln[c] : ov[c];
      __syncthreads();
      // step 3: row r of the run
      const uint4 cw = *reinterpret_cast<const uint4 *>(sC);
      const u32 cv[8] = {cw.x & 0xFFFFu, cw.x >> 16, cw.y & 0xFFFFu, cw.y >> 16,
                         cw.z & 0xFFFFu, cw.z >> 16, cw.w & 0xFFFFu, cw.w >> 16};
      for (u32 r = (u32)tid; r < R; r += 256) {
        u32 g = 0;
#pragma unroll
        for (int j = 1; j < 8; ++j) g += cv[j] <= r ? 1u : 0u;
        const uint4 fw = *reinterpret_cast<const uint4 *>(&sR[8 * g]);
        const u32 fv[8] = {fw.x & 0xFFFFu, fw.x >> 16, fw.y & 0xFFFFu, fw.y >> 16,
                           fw.z & 0xFFFFu, fw.z >> 16, fw.w & 0xFFFFu, fw.w >> 16};
        u32 kk = 8 * g;
#pragma unroll
        for (int j = 1; j < 8; ++j) kk += fv[j] <= r ? 1u : 0u;
        const u32 L = r - (u32)sR[kk];
        const u32 e = sE[kk] + L;
        const u32 rv = ent[e], nx = ent[e + 1];
        if (!(rv & FQ_UNCERT)) put_row(p, sG[kk] + L, (t0 + kk) * TILE + rv, (nx & ~FQ_UNCERT) - rv);
      }
    } else {
      for (int k = wid; k < PLACE_TILES; k += 4) {
        const u32 rows = (u32)sR[k + 1] - (u32)sR[k];
        const u64 tk = t0 + (u64)k;
        for (u32 L = (u32)lane; L < rows; L += 64) {
          const u32 rv = fq_start(p, tk, L);
          if (!(rv & FQ_UNCERT)) put_row(p, sG[k] + L, tk * TILE + rv, (fq_start(p, tk, L + 1) & ~FQ_UNCERT) - rv);
        }
      }
    }
    __syncthreads();
  }
}

// (download filters, sidx_filter.hip) The ID / sequence / quality spans of every record the
// FASTQ tile pass certified, from the line ends it kept (k_fq_tiles<true>: no re-read of the
// section): sidx_filter's layout, 6 u32 per record relative to its start, and the record's output
// length with bit 63 set ("done").  Records it did not certify, IDs whose TrimSpace is more than
// the line end, and whole tiles sent to k_fixup are left to k_fq_spans (their outlen stays 0).
// One wave per tile.
__device__ __forceinline__ u32 ndigits10(u64 v) {
  u32 d = 1;
  u64 q = 10;
#pragma unroll
  for (int k = 1; k < 20; ++k) {
    d += v >= q ? 1u : 0u;
    q *= 10;
  }
  return d;
}
__global__ __launch_bounds__(256) void k_fq_spans_place(const SlabParams p, u32 *spans, u64 *outlen, u64 K, int kind) {
  const int lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * 4;
  for (u64 t = (u64)blockIdx.x * 4 + (threadIdx.x >> 6); t < p.ntiles; t += nw) {
    const u64 w = p.fq_agg[t];
    const u32 Te = (u32)(w >> FQW_T) & 0xFFFFu;
    const u32 gi = (u32)(w >> FQW_GI) & 7u;
    const u32 i0 = gi == 7u ? GUESS_NONE : gi;
    const u32 nrec = (u32)(w >> FQW_NREC) & FQW_NRECM;
    const u64 j0 = p.state_in + p.tile_excl[t];
    const u32 ti0 = (u32)((3 - (j0 & 3)) & 3);
    const u32 ngt = ti0 < Te ? (Te - ti0 + 3) / 4 : 0;
    const u32 ngg = i0 < Te ? (Te - i0 + 3) / 4 : 0;
    if (((w >> FQW_SLOW) & 1u) || (i0 != ti0 && (ngt | ngg) != 0)) continue;  // the whole tile went to k_fixup
    const u64 gbase = ((j0 + ti0 + 1) >> 2) - ((p.file_start && t == 0) ? 1u : 0u);
    const uint16_t *ln = p.fq_lines + t * (3 * RCAP);
    for (u32 L = (u32)lane; L < nrec; L += 64) {
      const u64 g = gbase + L;
      const u32 rv = fq_start(p, t, L);
      if (g < p.row_base || g - p.row_base >= K || (rv & FQ_UNCERT)) continue;
      const u32 x0 = ln[3 * L];
      if (x0 == 0xFFFFu) continue;
      const u32 x1 = ln[3 * L + 1], x2 = ln[3 * L + 2], nx = fq_start(p, t, L + 1) & ~FQ_UNCERT;
      const u32 e0 = x0 & 0x7FFFu, e1 = x1 & 0x7FFFu, e2 = x2 & 0x7FFFu, e3 = nx - 1;
      const u32 z0 = e0 - (x0 >> 15), z1 = e1 - (x1 >> 15), z3 = e3 - (x2 >> 15);
      const u32 il = z0 - rv - 1, sl = z1 - e0 - 1, ql = z3 - e2 - 1;
      const u64 i = g - p.row_base;
      u32 *sp = spans + 6 * i;
      sp[0] = 1u; sp[1] = il;
      sp[2] = e0 + 1 - rv; sp[3] = sl;
      sp[4] = e2 + 1 - rv; sp[5] = ql;
      const u64 len = kind == 1 ? (u64)il + sl + 3 : (u64)ndigits10(i + 1) + sl + ql + 6;
      outlen[i] = len | (1ull << 63);
    }
  }
}

// Record starting at s validated from global memory by the whole wave.
__device__ __forceinline__ void fix_record(const SlabParams &p, u64 s, u64 g, u32 tile, int lane) {
  WaveAcc wa;
  wa.g = p.data; wa.end = p.end; wa.eof = p.eof; wa.lane = lane; wa.front = p.front;
  u64 len = 0, epos = 0, elen = 0;
  const u32 st = run_record_cold<F_FASTQ>(wa, s, 0, len, epos, elen);
  if (lane == 0) {
    if (st == ST_OK) put_row(p, g, s, len);
    else atomicMin(p.badkey, (g << KEY_REC_SHIFT) | ((u64)(tile & ((1u << KEY_TILE_BITS) - 1)) << 4) | st);
  }
}

// k_fixup: the records and tiles k_fq_tiles / k_fq_place queued, one wave per item.  A tile is re-indexed
// with its true newline rank j0: every '\n' of rank 3 mod 4 starts a record.  Its last workgroup to
// finish (a ticket in counters[7]) then runs k_finalize's body: one launch less per build.
struct DevResult;
__device__ __forceinline__ void finalize_body(const SlabParams &p, int fmt, DevResult *res);
__device__ __forceinline__ void last_block_finalize(const SlabParams &p, int fmt, DevResult *res) {
  // every storing wave's stores (rows, FASTA detail slots) complete, then one release per
  // workgroup before its ticket; the last workgroup acquires (MI355X_MICROARCH.md, valid forms)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32 k = __hip_atomic_fetch_add(&p.counters[7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      finalize_body(p, fmt, res);
    }
  }
}
__global__ __launch_bounds__(256) void k_fixup(const SlabParams p, DevResult *res) {
  if (gated_off(p)) {
    if (res) last_block_finalize(p, F_FASTQ, res);
    return;
  }
  const int lane = threadIdx.x & 63;
  const u32 nw = gridDim.x * (blockDim.x / 64);
  const u32 wv = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const u32 n = p.counters[2] < p.fixcap ? p.counters[2] : (u32)p.fixcap;
  for (u32 i = wv; i < n; i += nw) {
    const FixRec f = reinterpret_cast<const FixRec *>(p.fix)[i];
    if (f.start != ~0ull) {
      fix_record(p, f.start, f.g, f.tile, lane);
      continue;
    }
    const u32 tile = f.tile;
    const u64 tlo = (u64)tile * TILE;
    const u64 thi = (tlo + TILE < p.n) ? tlo + TILE : p.n;
    if (p.file_start && tile == 0) fix_record(p, 0, 0, tile, lane);
    u64 rank = f.g;
    for (u64 b = tlo; b < thi; b += 1024) {
      const u64 a = b + (u64)lane * 16;
      u32 m = 0;
      if (a < thi) m = eq16((a + 16 <= thi) ? load16(p.data + a) : load16_partial(p.data, a, thi), '\n');
      const u32 c = __popc(m);
      u32 incl = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      u64 cand = __ballot(m != 0);
      while (cand) {
        const int L = (int)ctz64(cand);
        cand &= cand - 1;
        u32 mL = (u32)__shfl((int)m, L, 64);
        u64 rr = rank + (u32)__shfl((int)(incl - c), L, 64);
        while (mL) {
          const u32 bit = (u32)__builtin_ctz(mL);
          mL &= mL - 1;
          if ((rr & 3) == 3) fix_record(p, b + 16 * (u64)L + bit + 1, (rr + 1) >> 2, tile, lane);
          ++rr;
        }
      }
      rank += (u32)__shfl((int)incl, 63, 64);
    }
  }
  if (res) last_block_finalize(p, F_FASTQ, res);
}

// ====================================================================================
// FASTA tile pass: k_fa_tiles -> scan of the tile aggregates (FastaMonoid) -> k_fa_place ->
// k_fa_fixup.  The input is read once.
//
// fasta.go:93-140 restated per tile: a '>' is a record boundary iff a '\n' occurred since the
// previous '>' (the FastaMonoid).  Inside a tile every '>' but possibly the first is decided
// locally; the tile's first '>' with no '\n' before it in the tile is "conditional" -- a
// boundary iff the tile is entered armed, known after the scan.  The candidates (the
// boundaries plus the conditional '>') go to a provisional table as tile-relative positions.
//
// Validation is owned by the END of a record: the piece that closes a record is the bytes
// since the previous '>' (fasta.go:111-121, TrimSpace must leave a '\n' inside), so the tile
// holding the closing '>' checks it from LDS.  A piece that starts in an earlier tile is
// certified from its part in this tile when that part alone shows a '\n' between two ASCII
// non-space bytes; anything undecidable here (such pieces otherwise, non-ASCII bytes at a
// trimmed edge, the conditional '>') goes to k_fa_fixup, which re-checks it from global
// memory.  Rows are owned by the START of a record: k_fa_place writes the row of the record
// opened by each boundary, its end being the next candidate of the tile or, for the tile's
// last boundary, the first boundary of a later tile (read off the tile words).
// ====================================================================================
constexpr u32 FA_OK = 0, FA_INV = 1, FA_DEFER = 2, FA_SKIP = 3;  // SKIP: owned by the previous slab
// Measured choices (round 5, one-process A/B tables under profiles/r05/calls/): the tile
// certificate's '\n' lookup over two mask words in one LDS round; fa_check's fast path looks at
// FA_NLW = 2 mask words (2.12 -> 1.99 ms, r05fa); a word's candidate count by carries instead of a
// loop over its '>' (1.976 -> 1.929 and 2.050 -> 2.021 ms on two input copies, r05fg).  Dropped:
// the tile's stores issued after the next tile's DMA (2.26 against 2.12 ms, r05n).
constexpr int FA_NLW = 2;
constexpr u32 FA_NONE = ~0u;
constexpr int FAW = 8;  // rare tile words: -, -, -, -, finv, inv_lo (a tile with an invalid piece), eof_st, eof_lo (the last tile)
// The per-tile word (fq_agg[t]): the FastaMonoid aggregate in bits 0-17 (what the scan folds),
// the candidate count, slow / conditional-first flags, the first conditional and the first
// definite boundary (15 bits each, 0x7FFF: none) and whether tw[4..5] hold an invalid piece --
// one u64 store per tile instead of a 32-byte record (the k_fq_tiles note on stores).
constexpr u64 FAW_AMASK = 0x3FFFF;
__device__ __forceinline__ u64 fa_word(u64 A, u32 ncand, bool slow, u32 delta, u32 fc, u32 fd, bool hasinv,
                                       bool tcert) {
  const u32 nc = ncand < 0xFFFu ? ncand : 0xFFFu;  // more than RCAP means slow anyway
  return (A & FAW_AMASK) | ((u64)nc << 18) | ((u64)tcert << 30) | ((u64)slow << 31) | ((u64)(delta & 1u) << 32) |
         ((u64)(fc & 0x7FFFu) << 33) | ((u64)(fd & 0x7FFFu) << 48) | ((u64)hasinv << 63);
}
// bit 30: the piece open at the tile's end (from its last '>', or from before the tile) holds a
// '\n' between two ASCII non-space bytes inside this tile -- whatever the rest of the piece is,
// TrimSpace keeps that '\n' inside, so the piece passes fasta.go:111-121 (the next tile's first
// piece, undecidable from its own part, is then settled without k_fa_fixup)
__device__ __forceinline__ bool fa_w_tcert(u64 w) { return (w >> 30) & 1u; }
__device__ __forceinline__ u32 fa_w_none(u32 x) { return x == 0x7FFFu ? FA_NONE : x; }
__device__ __forceinline__ u32 fa_w_flags(u64 w) { return (u32)((w >> 31) & 1u) | ((u32)((w >> 32) & 1u) << 1); }
__device__ __forceinline__ u32 fa_w_fc(u64 w) { return fa_w_none((u32)(w >> 33) & 0x7FFFu); }
__device__ __forceinline__ u32 fa_w_fd(u64 w) { return fa_w_none((u32)(w >> 48) & 0x7FFFu); }

struct __align__(16) FaSmem {
  u64 mnl[TILE / 64];
  u32 cand[RCAP];  // candidate: tile-relative '>' | (previous '>' + 1, 0: none in the tile) << 14
  u64 wagg[SNW];   // per wave: candidates | conditional << 20
  u32 wlast[SNW];  // per wave: last '>' + 1
  u32 wnl[SNW];    // per wave: last '\n' + 1
  u32 finv, tcert, pad[2];
};
static_assert(TILE <= (1 << 14), "candidate packing: 14-bit positions");

// first '\n' in [a, b) of the tile (mask words), b if none
__device__ __forceinline__ u32 fa_find_nl(const u64 *mnl, u32 a, u32 b) {
  if (a >= b) return b;
  u32 w = a >> 6;
  const u32 wl = (b - 1) >> 6;
  u64 m = mnl[w] & (~0ull << (a & 63));
  for (;;) {
    if (m) {
      const u32 q = (w << 6) + ctz64(m);
      return q < b ? q : b;
    }
    if (w == wl) return b;
    m = mnl[++w];
  }
}

// fasta.go:111-121 on the piece [lo, g) of the tile: TrimSpace leaves a '\n' inside.  ASCII
// edges only; an edge byte >= 0x80 (unicode.IsSpace may trim it) is left to the fixup.
// `part`: the piece starts before the tile, [lo, g) is only its tail -- then a '\n' between
// two ASCII non-space bytes certifies it and anything else is undecided.
__device__ __forceinline__ u32 fa_check(const uint8_t *r, const u64 *mnl, u32 lo, u32 g, bool part) {
  // the common piece in one LDS round: its first byte and the byte before its closing "\n>"
  // are printable ASCII (TrimSpace keeps [lo, g - 1)) and the '\n' ending its first line is
  // in the mask word of lo -- that '\n' is then the first one fa_find_nl would return
  if (g >= lo + 3) {
    // the first '\n' from lo within FA_NLW mask words, all read in one LDS round: with one
    // word, a header line running past lo's 64 bytes (about half of C3's records) took the loops
    // below -- 2.12 -> 1.99 ms for k_fa_tiles with two words (profiles/r05/calls/r05fa)
    const u32 c0 = r[lo], c1 = r[g - 1], c2 = r[g - 2];
    const u32 wi = lo >> 6;
    u64 w[FA_NLW];
#pragma unroll
    for (int k = 0; k < FA_NLW; ++k) w[k] = wi + k < (u32)(TILE / 64) ? mnl[wi + k] : 0ull;
    w[0] &= ~0ull << (lo & 63);
    u32 q = ~0u;
#pragma unroll
    for (int k = FA_NLW - 1; k >= 0; --k)
      if (w[k]) q = ((wi + (u32)k) << 6) + ctz64(w[k]);
    if (ascii_nonspace(c0) && c1 == '\n' && ascii_nonspace(c2) && q < g - 1) return FA_OK;
  }
  u32 f = lo;
  while (f < g && ascii_space(r[f])) ++f;
  if (f == g) return part ? FA_DEFER : FA_INV;
  u32 e = g;
  while (ascii_space(r[e - 1])) --e;  // stops at f + 1 at the latest
  if (r[f] >= 0x80 || r[e - 1] >= 0x80) return FA_DEFER;
  if (fa_find_nl(mnl, f, e) < e) return FA_OK;
  return part ? FA_DEFER : FA_INV;
}

__device__ __forceinline__ void fa_iter(const SlabParams &p, FaSmem &S, uint8_t *raw, u64 t, int tid, int lane,
                                        int wid) {
  __builtin_amdgcn_s_setprio(3);  // as k_fq_tiles: DMA issue, then the certification, first
  stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);  // the tile alone: no halo, no front
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a wave classifies only the bytes it staged
  if (tid == 0) S.finv = FA_NONE;
  const u64 tlo = t * TILE;
  const u32 tlen = (u32)(((tlo + TILE < p.n) ? tlo + TILE : p.n) - tlo);
  const u32 llen = (u32)(((tlo + TILE + SHALO < p.end) ? tlo + TILE + SHALO : p.end) - tlo);
  if (llen < (u32)TILE && (llen & 3u)) {  // slab end: the partial last dword came back as zeros
    lds_barrier();
    if (tid == 0) {
      const u32 o = llen & ~15u;
      uint4 v = keep_bytes(*reinterpret_cast<const uint4 *>(raw + FRONT + o), llen - o);
      u32 ll;
      const auto rs = tile_rsrc(p, t, ll);
      patch_tail(v, o, llen, tail_dword(rs, llen));
      *reinterpret_cast<uint4 *>(raw + FRONT + o) = v;
    }
    lds_barrier();
  }
  const uint8_t *r = raw + FRONT;
  // ---- '\n' / '>' mask words, the candidates -----------------------------------------------
  // A '>' at j is a candidate (fasta.go:100-138) iff a '\n' occurred since the previous '>':
  // with pg / pn = the last '>' / '\n' before j (+ 1, 0: none in the tile), iff pn > pg, or
  // pg == 0 (the tile's first '>': a boundary if pn > 0, else conditional on the state the
  // tile is entered in).  Inside a wave, pg and pn come from two max scans; only a wave's first
  // '>' with no '\n' before it in the wave depends on the earlier waves, and is settled after
  // the barrier by a fold over the four wave summaries.
  u64 nl = 0, gt = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
    const uint4 v = *reinterpret_cast<const uint4 *>(r + tid * 64 + 16 * cj);
    nl |= (u64)eq16x(v, '\n') << (16 * cj);
    gt |= (u64)eq16x(v, '>') << (16 * cj);
  }
  if (eq_suspect(nl) || eq_suspect(gt)) {  // two flags of one kind side by side in a dword ("\n\v", ">?"): exact masks
    nl = gt = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = *reinterpret_cast<const uint4 *>(r + tid * 64 + 16 * j);
      nl |= (u64)eq16(v, '\n') << (16 * j);
      gt |= (u64)eq16(v, '>') << (16 * j);
    }
  }
  const u32 rl0 = tlen > (u32)tid * 64 ? tlen - (u32)tid * 64 : 0u;
  const u32 rl = rl0 < 64 ? rl0 : 64u;
  nl &= lowmask(rl);
  gt &= lowmask(rl);
  S.mnl[tid] = nl;
  const u32 base = (u32)tid * 64;
  const u32 ln = nl ? base + 64 - clz64(nl) : 0u;  // last '\n' + 1
  const u32 lg = gt ? base + 64 - clz64(gt) : 0u;  // last '>' + 1
  const u32 NLi = wave_scan_max(ln), GTi = wave_scan_max(lg);
  // the previous lane's two values by one DPP wave shift (lane 0 reads 0); positions + 1 <= 2^14
  const u32 pk = (u32)__builtin_amdgcn_update_dpp(0, (int)((NLi << 16) | GTi), 0x138, 0xF, 0xF, false);
  const u32 NLx = pk >> 16, GTx = pk & 0xFFFFu;  // before this word, in the wave
  // a '>' is a candidate iff the marker ('>' or '\n') nearest below it is a '\n': one carry per
  // '\n' (and one at bit 0 when the word is entered after a '\n') runs up through the non-marker
  // bits of ~u and lands on the next marker; the wave's first '>' with no marker below it at all
  // is the conditional one
  const u64 u = nl | gt;
  const u32 c = popc64(gt & (~u + (nl << 1) + (NLx > GTx ? 1ull : 0ull)));
  const u32 cond = (GTx == 0 && NLx == 0 && (u & (0ull - u) & gt)) ? 1u : 0u;
  const u32 incl = wave_scan_add(c);
  const bool wcond = __ballot(cond) != 0;
  if (lane == 63) {
    S.wagg[wid] = incl | (wcond ? 1u << 20 : 0u);
    S.wlast[wid] = GTi;
    S.wnl[wid] = NLi;
  }
  lds_barrier();
  // fold of the wave summaries in order: candidates before this wave, its first '>' settled
  u32 PN = 0, PG = 0, cnt = 0, delta = 0, myPG = 0, mybase = 0, mycond = 0;
#pragma unroll
  for (int w = 0; w < SNW; ++w) {
    // uniform values: the fold runs on the scalar unit
    const u32 a = (u32)__builtin_amdgcn_readfirstlane((int)(u32)S.wagg[w]);
    const u32 gw = (u32)__builtin_amdgcn_readfirstlane((int)S.wlast[w]);
    const u32 nw = (u32)__builtin_amdgcn_readfirstlane((int)S.wnl[w]);
    if (w == wid) { myPG = PG; mybase = cnt; }
    u32 cw = 0;
    if (a >> 20) {
      if (PG == 0 && PN == 0) { delta = 1; cw = 1; }  // the tile's first '>', conditional
      else if (PG == 0 || PN > PG) cw = 1;
    }
    if (w == wid) mycond = cw;
    cnt += cw + (a & 0xFFFFFu);
    PN = umax(PN, nw);
    PG = umax(PG, gw);
  }
  const u32 ncand = cnt;
  const u32 alast = PG;
  const u64 A = FastaMonoid::mk(cnt - delta, delta, (PN | PG) == 0 ? 0u : (PN > PG ? 2u : 1u));
  // ---- candidates of this word, in order ----------------------------------------------------
  if (gt) {
    u32 idx = mybase + mycond + incl - c;
    u32 pg = GTx, pga = GTx ? GTx : myPG;  // previous '>' + 1: in the wave / in the tile
    for (u64 m = gt; m;) {
      const u32 j = ctz64(m);
      m &= m - 1;
      const u64 nb = nl & lowmask(j);
      const u32 pn = nb ? base + 64 - clz64(nb) : NLx;
      u32 slot = FA_NONE;
      if (pg == 0 && pn == 0) slot = mycond ? mybase : FA_NONE;
      else if (pg == 0 || pn > pg) slot = idx++;
      if (slot < (u32)RCAP) S.cand[slot] = (base + j) | (pga << 14);
      pg = pga = base + j + 1;
    }
  }
  lds_barrier();
  // ---- validation of the pieces that close at the candidates -------------------------------
  __builtin_amdgcn_s_setprio(2);
  const bool slow = ncand > (u32)RCAP;
  uint16_t *stage = reinterpret_cast<uint16_t *>(p.fq_stage + t * RCAP);  // position | status << 14
  // A slab after the file's first: its first tile's first boundary (the incoming state is known
  // there) closes the record open at the slab start, which the previous slab owns and checks
  // through its halo; any other piece starting before data[0] is checked as a part (never INV).
  const bool own0 = p.file_start || t != 0;
  const u32 skip0 = own0 ? ~0u : ((delta && !(p.state_in & 1)) ? 1u : 0u);
  if (!slow) {
    for (u32 i = (u32)tid; i < ncand; i += SNT) {
      const u32 c = S.cand[i];
      const u32 g = c & 0x3FFFu, lo = c >> 14;
      u32 st;
      if (i == skip0) st = FA_SKIP;
      else if (i == 0 && delta) st = FA_DEFER;  // conditional: its piece has no '\n' in this tile
      else st = fa_check(r, S.mnl, lo, g, lo == 0 && (t != 0 || !p.file_start));
      stage[i] = (uint16_t)(g | (st << 14));
      if (st == FA_INV) atomicMin(&S.finv, i);
    }
  }
  u32 *tw = p.fq_tiles + t * FAW;
  if (tid == SNT - 1) {  // the certificate of the piece open at the tile's end (fa_w_tcert)
    // (the first '\n' after the last '>': two mask words in one LDS round, the loop beyond)
    const u32 wi = alast >> 6;
    const u64 w0 = wi < (u32)(TILE / 64) ? S.mnl[wi] & (~0ull << (alast & 63)) : 0ull;
    const u64 w1 = wi + 1 < (u32)(TILE / 64) ? S.mnl[wi + 1] : 0ull;
    u32 q = w0 ? (wi << 6) + ctz64(w0) : (w1 ? ((wi + 1) << 6) + ctz64(w1) : fa_find_nl(S.mnl, alast, tlen));
    if (q > tlen) q = tlen;
    S.tcert = (q > alast && q + 1 < tlen && ascii_nonspace(r[q - 1]) && ascii_nonspace(r[q + 1])) ? 1u : 0u;
  }
  if (t == p.ntiles - 1 && tid == SNT - 1) {  // EOF piece [last '>' + 1, n), fasta.go:111 + :123-125
    u32 est = FA_OK;  // a slab with a halo: its last record is closed there (k_fa_fixup)
    const u32 lo = alast;
    if (p.end > p.n || !p.eof) {
    } else if (lo != 0 || (t == 0 && p.file_start)) {
      if (tlen > lo + 1 && fa_find_nl(S.mnl, lo, tlen) < tlen) est = fa_check(r, S.mnl, lo, tlen, false);
    } else {
      est = fa_check(r, S.mnl, 0, tlen, true);
    }
    tw[6] = est;
    tw[7] = lo;
  }
  __builtin_amdgcn_s_setprio(0);
  lds_barrier();  // S.finv final; the slot and S are reused next
  {  // one packed word per tile (fa_word); the first invalid piece in tw[] (rare)
    const u32 finv = S.finv;
    const u64 word = fa_word(A, ncand, slow, delta, delta ? (S.cand[0] & 0x3FFFu) : FA_NONE,
                             (A >> 3) ? (S.cand[delta] & 0x3FFFu) : FA_NONE, finv != FA_NONE, S.tcert != 0);
    if (tid == 0) p.fq_agg[t] = word;
    if (tid == 0 && finv != FA_NONE) {
      tw[4] = finv;
      tw[5] = S.cand[finv] >> 14;
    }
  }
}

// one LDS slot, batches of FA_RR consecutive tiles dealt round-robin to the workgroups (as
// k_fq_tiles): in one process over three copies of the C3 input (profiles/r06/calls/j/ab_fa_rr32.json)
// 1.858-1.994 ms against 1.896-2.020 for single tiles in XCD-major grid-stride order (round 5)
constexpr u64 FA_RR = 32;
#ifndef SIDX_FA_WGS
#define SIDX_FA_WGS 7  // 19.1 KiB of LDS (no halo in the slot); 8 per CU (<= 64 VGPRs) measured the same
#endif
__global__ __launch_bounds__(SNT, SIDX_FA_WGS) void k_fa_tiles(const SlabParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[FRONT + TILE];
  __shared__ FaSmem S;
  if (gated_off(p)) return;  // format speculation failed: the host re-runs with the detected format
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 G = p.pgrid;
  const u64 nbat = (p.ntiles + FA_RR - 1) / FA_RR;
  for (u64 c = blockIdx.x; c < nbat; c += G) {
    const u64 tb = c * FA_RR, te = tb + FA_RR < p.ntiles ? tb + FA_RR : p.ntiles;
    for (u64 t = tb; t < te; ++t) fa_iter(p, S, raw, t, tid, lane, wid);
  }
}

__device__ __forceinline__ u64 fa_key(u64 k, u32 slot, u32 st) {
  return (k << KEY_REC_SHIFT) | ((u64)(slot & ((1u << KEY_TILE_BITS) - 1)) << 4) | st;
}
// first boundary of tile u given its words and entering state: the conditional '>' when the
// tile is entered armed, else its first definite boundary (FA_NONE: none)
__device__ __forceinline__ u32 fa_first(u32 flags, u32 fc, u32 fd, u64 st) {
  return ((flags & 2) && (st & 1)) ? fc : fd;
}
// first boundary in tiles >= u (the whole wave, 64 tiles per step), n if none
__device__ u64 fa_next_global(const SlabParams &p, u64 u, int lane) {
  for (; u < p.ntiles; u += 64) {
    const u64 v = u + (u64)lane;
    u32 f = FA_NONE;
    if (v < p.ntiles) {
      const u64 w = p.fq_agg[v];
      f = fa_first(fa_w_flags(w), fa_w_fc(w), fa_w_fd(w), FastaMonoid::apply(p.state_in, p.tile_excl[v]));
    }
    const u64 bal = __ballot(f != FA_NONE);
    if (bal) {
      const int L = (int)ctz64(bal);
      return (u + (u64)L) * TILE + (u32)__shfl((int)f, L, 64);
    }
  }
  return p.n;
}

// k_fa_place: 64 consecutive tiles per workgroup, their words and entering states in LDS
// (plus the next tile's, for the row that crosses the group's end); a wave per tile.
__global__ __launch_bounds__(256) void k_fa_place(const SlabParams p) {
  __shared__ uint4 sw[PLACE_TILES + 1][2];
  __shared__ u64 sS[PLACE_TILES + 1];
  __shared__ u32 sC[PLACE_TILES];  // sC[k]: tile t0 + k - 1 certified the piece open at its end
  if (gated_off(p)) return;  // format speculation failed: the host re-runs with the detected format
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (u64 t0 = (u64)blockIdx.x * PLACE_TILES; t0 < p.ntiles; t0 += (u64)gridDim.x * PLACE_TILES) {
    if (tid >= 128 && tid < 128 + PLACE_TILES) {
      const u64 u = t0 + (u64)(tid - 128);  // the tile before t0 + (tid - 128), plus one
      sC[tid - 128] = (u >= 1 && u - 1 < p.ntiles) ? (u32)fa_w_tcert(p.fq_agg[u - 1]) : 0u;
    }
    if (tid <= PLACE_TILES && t0 + tid < p.ntiles) {
      const u64 w = p.fq_agg[t0 + tid];
      const u32 *tw = p.fq_tiles + (t0 + tid) * FAW;
      const bool last = t0 + tid == p.ntiles - 1;
      sw[tid][0] = make_uint4((u32)(w >> 18) & 0xFFFu, fa_w_flags(w), fa_w_fc(w), fa_w_fd(w));
      sw[tid][1] = make_uint4((w >> 63) ? tw[4] : FA_NONE, (w >> 63) ? tw[5] : 0u, last ? tw[6] : FA_OK,
                              last ? tw[7] : 0u);
      sS[tid] = FastaMonoid::apply(p.state_in, p.tile_excl[t0 + tid]);
    }
    __syncthreads();
    // four tiles per wave, 16 lanes each (a FASTA tile has ~10 boundaries): the tiles' stage
    // reads and row writes are in flight together instead of one tile's after another's
    const int sub = lane >> 4, sl = lane & 15;
    for (int kb = wid * 4; kb < PLACE_TILES; kb += 16) {
      const int k = kb + sub;  // <= PLACE_TILES - 1: sw[k + 1] is loaded
      const u64 t = t0 + k;
      const bool live = t < p.ntiles;
      if (!__ballot(live)) break;
      const uint4 w0 = sw[k][0], w1 = sw[k][1];
      const u32 ncand = w0.x, flags = w0.y, finv = w1.x, invlo = w1.y, est = w1.z, elo = w1.w;
      const u64 st = sS[k];
      const u64 cnt = st >> 1;
      const u64 tlo = t * TILE;
      if (p.n == 0) {  // no record at all: (0, EOF) on record 0
        if (lane == 0 && p.file_start) g_min64(p.badkey, fa_key(0, 0, ST_ABSENT));
        continue;
      }
      // too many candidates for the table: the whole tile from global memory
      if (live && (flags & 1) && sl == 0) push_fix(p, ~0ull, st, (u32)t);
      const bool go = live && !(flags & 1);
      const u32 skip = ((flags & 2) && !(st & 1)) ? 1u : 0u;
      const u32 nb = go ? ncand - skip : 0u;
      // end of the record open at the tile's end: the first boundary of a later tile
      u64 nxt = p.n;
      const bool wantn = go && (nb || t == 0) && t + 1 < p.ntiles;
      u32 f = FA_NONE;
      if (wantn) {
        const uint4 x = sw[k + 1][0];
        f = fa_first(x.y, x.z, x.w, sS[k + 1]);
        if (f != FA_NONE) nxt = (t + 1) * TILE + f;
      }
      // a later tile's first boundary: the whole wave searches, one group at a time
      u64 far = __ballot(wantn && f == FA_NONE && sl == 0);
      while (far) {
        const int L = (int)ctz64(far);
        far &= far - 1;
        const u64 tt = t0 + (u64)(kb + (L >> 4));
        const u64 r = fa_next_global(p, tt + 2, lane);
        if (sub == (L >> 4)) nxt = r;
      }
      const uint16_t *stage = reinterpret_cast<const uint16_t *>(p.fq_stage + t * RCAP);
      // the record open at a slab's start (number s0) is the previous slab's: no report of the
      // piece that closes it; if that was the tile's first invalid piece, the later invalid
      // ones of the tile go to k_fa_fixup (their piece starts are not kept)
      const u64 s0 = p.file_start ? ~0ull : (p.state_in >> 1);
      const bool finv_gone = finv != FA_NONE && finv >= skip && cnt + (finv - skip) == s0;
      for (u32 i = (u32)sl; i < nb; i += 16) {
        const u32 idx = i + skip;
        const u32 v = stage[idx];
        const u32 g = v & 0x3FFFu, vs = (v >> 14) & 3u;
        const u64 k2 = cnt + i;  // the record this '>' closes
        if (k2 == s0) {
        } else if (vs == FA_DEFER && idx == 0 && sC[k]) {
          // the tile's first '>' closes a piece that began before the tile: the previous tile
          // found a '\n' between two ASCII non-space bytes inside it (fa_w_tcert), so it is valid
        } else if (vs == FA_DEFER || (vs == FA_INV && finv_gone)) {
          push_fix(p, tlo + g, k2, (u32)t);
        } else if (vs == FA_INV && idx == finv) {  // the tile's first invalid piece
          p.detail[2 * t] = p.base + tlo + invlo;  // file offsets (slabs: base)
          p.detail[2 * t + 1] = g + 1 - invlo;  // the piece includes its '>'
          g_min64(p.badkey, fa_key(k2, (u32)t, ST_FA_INVALID));
        }
        const u64 e = (i + 1 < nb) ? tlo + (stage[idx + 1] & 0x3FFFu) : nxt;
        if (e == p.n && p.end > p.n) push_fix(p, tlo + g, k2 + 1, (u32)t | FIX_HALO);  // ends past the slab
        else put_row(p, k2 + 1, tlo + g, e - tlo - g);
      }
      if (go && t == 0 && sl == 0 && p.file_start) {  // record 0 starts at file offset 0
        const u64 e0 = nb ? (stage[skip] & 0x3FFFu) : nxt;
        if (e0 == p.n && p.end > p.n) push_fix(p, 0, 0, FIX_HALO);
        else put_row(p, 0, 0, e0);
      }
      if (go && p.eof && p.end == p.n && t == p.ntiles - 1 && sl == 0 && cnt + nb != s0) {  // closed by EOF
        const u64 k2 = cnt + nb;
        if (est == FA_INV) {
          const u32 slot = p.ntiles;
          p.detail[2 * (u64)slot] = p.base + tlo + elo;
          p.detail[2 * (u64)slot + 1] = p.n - tlo - elo;
          g_min64(p.badkey, fa_key(k2, slot, ST_FA_INVALID));
        } else if (est == FA_DEFER) {
          push_fix(p, p.n, k2, (u32)t);
        }
      }
    }
    __syncthreads();
  }
}

// position + 1 of the last '>' in [0, pos), 0 if none (the whole wave, 1 KiB per step)
__device__ u64 fa_prev_gt(const SlabParams &p, u64 pos, int lane) {
  if (pos == 0) return 0;
  u64 top = (pos - 1) & ~15ull;  // the chunk holding byte pos - 1
  const u64 off = 16ull * (u64)(63 - lane);
  for (;;) {
    u32 m = 0;
    u64 a = 0;
    if (top >= off) {
      a = top - off;
      const uint4 v = (a + 16 <= p.end) ? load16(p.data + a) : load16_partial(p.data, a, p.end);
      m = eq16(v, '>');
      if (a + 16 > pos) m &= (1u << (u32)(pos - a)) - 1u;
    }
    const u64 bal = __ballot(m != 0);
    if (bal) {
      const int L = 63 - (int)clz64(bal);
      const u64 q = m ? a + 31 - (u64)__builtin_clz(m) : 0ull;
      return __shfl(q, L, 64) + 1;
    }
    if (top < 1024) return 0;
    top -= 1024;
  }
}

__device__ __forceinline__ void fa_report(const SlabParams &p, u64 k, u32 slot, u64 epos, u64 elen, int lane) {
  if (lane == 0) {
    p.detail[2 * (u64)slot] = p.base + epos;  // file offset
    p.detail[2 * (u64)slot + 1] = elen;
    g_min64(p.badkey, fa_key(k, slot, ST_FA_INVALID));
  }
}

// FASTA slab with a halo (end > n): the record opened at b (number k) ends at the first
// boundary at or after n -- a '>' with a '\n' since the '>' before it -- found in the halo
// [n, end) from the slab's final armed bit, 1 KiB per step (per lane: the first boundary of its
// 16 bytes given the armed bit it is entered with, which is the last '\n' / '>' event of the
// lanes before it).  Its closing piece is validated and its row written here; a halo without a
// boundary that does not reach EOF is ST_NEEDMORE (the slab protocol's "halo exhausted").
__device__ void fa_halo_close(const SlabParams &p, u64 b, u64 k, u32 slot, int lane) {
  const u64 nt = p.ntiles;
  u32 armed = (u32)(FastaMonoid::apply(FastaMonoid::apply(p.state_in, p.tile_excl[nt - 1]), p.fq_agg[nt - 1] & FAW_AMASK) & 1);
  WaveAcc wa;
  wa.g = p.data; wa.end = p.end; wa.eof = p.eof; wa.lane = lane; wa.front = p.front;
  u64 g = ~0ull;
  for (u64 c0 = p.n & ~15ull; c0 < p.end && g == ~0ull; c0 += 1024) {
    const u64 a = c0 + 16ull * (u64)lane;
    u32 nl = 0, gt = 0;
    if (a < p.end) {
      const uint4 v = (a + 16 <= p.end) ? load16(p.data + a) : load16_partial(p.data, a, p.end);
      const u32 keep = a < p.n ? ~((1u << (u32)(p.n - a)) - 1u) & 0xFFFFu : 0xFFFFu;  // bytes >= n only
      nl = eq16(v, '\n') & keep;
      gt = eq16(v, '>') & keep;
    }
    // the lane's effect on the armed bit: 0 none, 1 clears ('>' last), 2 sets ('\n' last)
    const u32 hi_nl = nl ? 32 - __builtin_clz(nl) : 0u, hi_gt = gt ? 32 - __builtin_clz(gt) : 0u;
    const u32 eff = (nl | gt) ? (hi_nl > hi_gt ? 2u : 1u) : 0u;
    // armed bit entering the lane: the effect of the nearest lane below with one, else `armed`
    const u32 key = eff ? ((u32)lane + 1) * 4 + eff : 0u;
    u32 mx = key;
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = (u32)__shfl_up((int)mx, d, 64);
      if (lane >= d && y > mx) mx = y;
    }
    u32 below = (u32)__shfl_up((int)mx, 1, 64);
    if (lane == 0) below = 0;
    u32 in = below ? ((below & 3u) == 2u) : armed;
    u32 hit = 16;
    for (u32 m = gt; m; m &= m - 1) {
      const u32 j = (u32)__builtin_ctz(m);
      const u32 prevgt = gt & ((1u << j) - 1u);
      const u32 since = prevgt ? (nl & ~((2u << (31 - __builtin_clz(prevgt))) - 1u)) : nl;
      if ((since & ((1u << j) - 1u)) || (!prevgt && in)) { hit = j; break; }
    }
    const u64 hb = __ballot(hit < 16);
    if (hb) {
      const int L = (int)ctz64(hb);
      g = c0 + 16ull * (u64)L + (u32)__shfl((int)hit, L, 64);
    } else {
      const u32 last = (u32)__shfl((int)mx, 63, 64);
      if (last) armed = (last & 3u) == 2u;
    }
  }
  if (g == ~0ull && !p.eof) {
    if (lane == 0) g_min64(p.badkey, fa_key(k, slot, ST_NEEDMORE));
    return;
  }
  const u64 e = g == ~0ull ? p.end : g;
  const u64 lo = fa_prev_gt(p, e, lane);
  bool ok = true;
  u64 q;
  if (g != ~0ull) fasta_piece_ok(wa, lo, g, ok);
  else if (p.end - lo > 1 && wa.find(C_NL, lo, p.end, q) == FR_FOUND) fasta_piece_ok(wa, lo, p.end, ok);
  if (lane == 0) put_row(p, k, b, e - b);
  if (!ok) fa_report(p, k, slot, lo, g == ~0ull ? p.end - lo : g + 1 - lo, lane);
}

// k_fa_fixup: one wave per queued item.  A piece closing record k at b (b == n: the EOF
// piece) re-checked with the general validator; or a whole tile (start == ~0, g = its
// entering state) walked '>' by '>' from global memory.  Each item reports into a detail
// slot of its own (tiles: the tile; pieces: fixcap + item), so the first-bad record's text
// is never overwritten by another report.
__global__ __launch_bounds__(256) void k_fa_fixup(const SlabParams p, DevResult *res) {
  if (gated_off(p)) {
    if (res) last_block_finalize(p, F_FASTA, res);
    return;
  }
  const int lane = threadIdx.x & 63;
  const u32 nw = gridDim.x * (blockDim.x / 64);
  const u32 wv = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const u32 nq = p.counters[2] < p.fixcap ? p.counters[2] : (u32)p.fixcap;
  WaveAcc wa;
  wa.g = p.data; wa.end = p.end; wa.eof = p.eof; wa.lane = lane; wa.front = p.front;
  const u64 s0 = p.file_start ? ~0ull : (p.state_in >> 1);  // the previous slab's record (see k_fa_place)
  for (u32 i = wv; i < nq; i += nw) {
    const FixRec f = reinterpret_cast<const FixRec *>(p.fix)[i];
    if (f.tile & FIX_HALO) {
      fa_halo_close(p, f.start, f.g, p.fixcap + i, lane);
      continue;
    }
    if (f.start != ~0ull) {
      if (f.g == s0) continue;
      const u64 b = f.start;
      const u64 lo = fa_prev_gt(p, b, lane);
      bool ok = true;
      u64 elen = 0;
      if (b == p.n) {  // EOF piece: validated iff longer than 1 byte and holding a '\n'
        u64 q;
        if (p.n - lo > 1 && wa.find(C_NL, lo, p.n, q) == FR_FOUND) fasta_piece_ok(wa, lo, p.n, ok);
        elen = p.n - lo;
      } else {
        fasta_piece_ok(wa, lo, b, ok);
        elen = b + 1 - lo;
      }
      if (!ok) fa_report(p, f.g, p.fixcap + i, lo, elen, lane);
      continue;
    }
    const u64 t = f.tile;
    u64 cnt = f.g >> 1;
    bool armed = f.g & 1;
    const u64 tlo = t * TILE, thi = (tlo + TILE < p.n) ? tlo + TILE : p.n;
    u64 lo = fa_prev_gt(p, tlo, lane);
    u64 pend = (t == 0 && p.file_start) ? 0 : ~0ull, pk = 0;  // the open row (start, record number)
    u64 pos = tlo;
    bool bad = false;
    for (;;) {
      u64 g, q;
      if (wa.find(C_X, pos, thi, g) != FR_FOUND) break;
      if (!armed) armed = wa.find(C_NL, pos, g, q) == FR_FOUND;
      if (armed) {
        bool ok = true;
        if (cnt != s0) fasta_piece_ok(wa, lo, g, ok);
        if (!ok) {
          fa_report(p, cnt, (u32)t, lo, g + 1 - lo, lane);
          bad = true;
          break;
        }
        if (pend != ~0ull && lane == 0) put_row(p, pk, pend, g - pend);
        ++cnt;
        pend = g;
        pk = cnt;
        armed = false;
      }
      lo = g + 1;
      pos = g + 1;
    }
    if (bad) continue;  // later records are past the first bad one
    if (pend != ~0ull) {
      const u64 e = fa_next_global(p, t + 1, lane);
      if (e == p.n && p.end > p.n) fa_halo_close(p, pend, pk, p.fixcap + i, lane);
      else if (lane == 0) put_row(p, pk, pend, e - pend);
    }
    if (t == p.ntiles - 1 && p.eof && p.end == p.n && cnt != s0) {
      bool ok = true;
      u64 q;
      if (p.n - lo > 1 && wa.find(C_NL, lo, p.n, q) == FR_FOUND) fasta_piece_ok(wa, lo, p.n, ok);
      if (!ok) fa_report(p, cnt, (u32)t, lo, p.n - lo, lane);
    }
  }
  if (res) last_block_finalize(p, F_FASTA, res);
}

// ====================================================================================
// k_finalize: slab result; resets the other build's first-bad slot and counters
// ====================================================================================
template <class M>
__device__ __forceinline__ u64 apply_fmt(u64 s, u64 a) { return M::apply(s, a); }

__device__ __forceinline__ void finalize_body(const SlabParams &p, int fmt, DevResult *res);
__global__ void k_finalize(const SlabParams p, int fmt, DevResult *res) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  finalize_body(p, fmt, res);
}
// k_finalize's body (thread 0 of one workgroup): also run by the last workgroup of k_fixup
__device__ __forceinline__ void finalize_body(const SlabParams &p, int fmt, DevResult *res) {
  if (gated_off(p)) {  // the speculated format was wrong: nothing ran; the host re-runs
    DevResult r = {};
    r.flags = 16;
    r.fmt = (u32)fmt;
    r.detected = (u32)*p.gate;
    *res = r;
    *p.badkey_next = KEY_NONE;
    for (int i = 0; i < NCOUNTERS; ++i) p.counters_next[i] = 0;
    return;
  }
  const u64 w = ((volatile u64 *)p.status)[p.ntiles - 1];
  const u64 agg = w & PAYLOAD_MASK;  // slab aggregate
  u64 fin;
  // (k_fixup's last workgroup: the other workgroups' first-bad keys are device-scope atomics)
  if (fmt == F_FASTA) fin = apply_fmt<FastaMonoid>(p.state_in, agg);
  else if (fmt == F_SAM) fin = apply_fmt<SamMonoid>(p.state_in, agg);
  else fin = apply_fmt<CountMonoid>(p.state_in, agg);
  const u64 key = __hip_atomic_load(p.badkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DevResult r;
  r.state_out = fin;
  r.slab_agg = agg;
  r.err_pos = 0;
  r.err_len = 0;
  r.flags = 0;
  r.path = 0;
  r.fixups = p.counters[2];
  r.fix_tiles = p.counters[3] >> 1;
  r.fmt = (u32)fmt;
  r.detected = p.gate ? (u32)*p.gate : 0u;
  r.pad = 0;
  r.key = key;
  if ((w >> 62) != 2 || (((u32)(w >> EPOCH_SHIFT)) & EPOCH_MASK) != p.epoch) r.flags |= 2;  // no final INC
  u64 krec = key >> KEY_REC_SHIFT;
  u32 kst = (u32)(key & 15);
  const u32 ktile = (u32)((key >> 4) & ((1u << KEY_TILE_BITS) - 1));
  u64 natural;  // count when no record terminates the sequence early
  if (fmt == F_FASTQ) natural = (fin >> 2) + 1;          // groups 0..T/4 all valid
  else if (fmt == F_FASTA) natural = (fin >> 1) + 1;     // records 0..B
  else if (fmt == F_SAM) natural = (fin >> 2) + 1;       // records 0..Tterm
  else natural = fin + 1;                                // lines 0..T
  r.natural = natural;
  if (key == KEY_NONE) {
    r.count = natural;
    r.code = ST_OK;
  } else {
    r.count = krec;
    r.code = kst;
    if (kst == ST_FA_INVALID) {
      r.err_pos = p.detail[2 * (u64)ktile];
      r.err_len = p.detail[2 * (u64)ktile + 1];
    }
    if (kst == ST_DONTCARE) r.flags |= 2;
    if (kst == ST_NEEDMORE) r.flags |= 4;
  }
  if (p.counters[1]) r.flags |= 2;
  if (p.counters[3] & 1) r.flags |= 8;  // k_fixup queue overflow: re-run on the general kernel
  if (p.inject & 1) r.count = r.count ? r.count - 1 : 0;  // test hook: a short count
  const u64 nrows = r.count > p.row_base ? r.count - p.row_base : 0;
  if (nrows > p.row_cap) r.flags |= 1;
  // End-of-build invariants of a whole-file build (record.go:51-83: row i + 1 starts where row i
  // ends, the first at 0).  A successful FASTA / SAM / line build consumes every byte, so its last
  // row ends at the file end; a FASTQ build only skips trailing blank lines after its last record
  // (fastq.go:141-156).  A build whose count or rows came out of stale device state fails here
  // and reports an internal error instead of a short table.
  if (p.file_start && p.eof && p.end == p.n && !(r.flags & 9) && nrows && p.rows) {  // (p.end > p.n: a slab's halo)
    const u64 *rw = p.rows;
    bool bad = rw[0] != p.base;
    if (r.code == ST_OK || r.code == ST_END || r.code == ST_ABSENT) {
      const u64 e = rw[2 * (nrows - 1)] + rw[2 * (nrows - 1) + 1], fe = p.base + p.n;
      if (fmt == F_FASTQ) bad |= e > fe || (e < fe && (p.data[e - p.base] != '\n' || p.data[p.n - 1] != '\n'));
      else bad |= e != fe;
      // the line index's last row is the bytes after the last '\n' (line.go:37-45, possibly none)
      if (fmt == F_LINE) bad |= rw[2 * (nrows - 1) + 1] != 0 && p.n && p.data[p.n - 1] == '\n';
    }
    if (bad) r.flags |= 2;
  }
  *res = r;
  if (p.summary) {
    SlabSummary *o = reinterpret_cast<SlabSummary *>(p.summary);
    o->agg = agg; o->state_in = p.state_in; o->key = key; o->natural = natural;
    o->row_base = p.row_base; o->err_pos = r.err_pos; o->err_len = r.err_len;
    o->fmt = (uint16_t)fmt; o->flags = (uint16_t)r.flags; o->seq = p.seq;
  }
  *p.badkey_next = KEY_NONE;
  for (int i = 0; i < NCOUNTERS; ++i) p.counters_next[i] = 0;
}

// ====================================================================================
// Multi-GPU slabs: guess a slab's incoming state, fold the gathered summaries
// ====================================================================================
// FASTQ: the first line of the slab that looks like a record start ('@' line, '+' two
// lines later, sequence and quality lines of equal length) fixes the line phase.
// FASTA: '\n' vs '>' closest before the slab start (armed bit).  SAM: class of the line
// open at the slab start.  LINE: nothing to guess.  One wave; verified after the exchange.
__global__ void k_slab_guess(const uint8_t *data, u64 n, u64 front, int fmt, u64 *out) {
  __shared__ u32 nlp[256];
  __shared__ u32 cnt;
  const int lane = threadIdx.x;
  u64 guess = 0;
  if (fmt == F_FASTQ) {
    const u64 lim = n < 4096 ? n : 4096;
    if (lane == 0) cnt = 0;
    __syncthreads();
    for (u64 b = 0; b < lim; b += 1024) {  // '\n' positions of the first 4 KiB, in order
      const u64 a = b + (u64)lane * 16;
      u32 m = 0;
      if (a < lim) m = eq16((a + 16 <= lim) ? load16(data + a) : load16_partial(data, a, lim), '\n');
      const u32 c = __popc(m);
      u32 pre = c;
      for (int d = 1; d < 64; d <<= 1) { const u32 y = __shfl_up(pre, d, 64); if (lane >= d) pre += y; }
      const u32 base = cnt;
      u32 o = base + pre - c;
      while (m) { if (o < 256) nlp[o] = (u32)(a + __builtin_ctz(m)); ++o; m &= m - 1; }
      __syncthreads();
      if (lane == 63) cnt = base + pre;
      __syncthreads();
    }
    const u32 N = cnt < 256 ? cnt : 256;
    // candidate i: record starts after '\n' #i (local rank i): lines (i,i+1],(i+1,i+2]...
    bool ok = false;
    for (u32 i0 = 0; i0 + 4 < N; i0 += 64) {
      const u32 i = i0 + lane;
      ok = false;
      if (i + 4 < N) {
        const u32 s = nlp[i] + 1, e0 = nlp[i + 1], e1 = nlp[i + 2], e2 = nlp[i + 3], e3 = nlp[i + 4];
        ok = data[s] == '@' && e0 > s + 1 && data[e1 + 1] == '+' && (e1 - e0) == (e3 - e2) && e1 > e0 + 1;
      }
      const u64 bal = __ballot(ok);
      if (bal) { const u32 L = ctz64(bal); guess = (3u - ((i0 + L) & 3)) & 3; break; }
    }
  } else if (fmt == F_FASTA || fmt == F_SAM) {
    // closest '\n' / '>' before data[0] within `front` bytes (scan backwards 1 KiB per step)
    const u64 lim = front < 65536 ? front : 65536;
    i64 best = -1;
    u32 bestc = 0;
    for (u64 b = 0; b < lim && best < 0; b += 1024) {
      // window [-(b+1024), -b): lane k holds bytes [-(b+16k+16), -(b+16k))
      const u64 hi = b + (u64)lane * 16;  // distance of this chunk's end before data[0]
      u32 nlm = 0, gtm = 0;
      if (hi < lim) {
        const u64 take = (lim - hi) < 16 ? (lim - hi) : 16;
        const uint8_t *q = data - hi - take;
        const uint4 v = load16_partial(q, 0, take);
        nlm = eq16(v, '\n');
        gtm = fmt == F_FASTA ? eq16(v, '>') : 0u;
        // bit j <-> byte at distance hi + take - j before data[0]
        const u32 m = nlm | gtm;
        if (m) {
          const u32 j = 31 - __builtin_clz(m);           // closest to data[0]
          const u64 dist = hi + take - j;                 // >= 1
          const u64 key = (dist << 1) | ((gtm >> j) & 1);
          (void)key;
        }
      }
      const u32 m = nlm | gtm;
      const u64 bal = __ballot(m != 0);
      if (bal) {
        const int L = (int)ctz64(bal);  // nearest chunk first
        const u32 mm = __shfl(m, L, 64);
        const u32 g = __shfl(gtm, L, 64);
        const u64 hiL = b + (u64)L * 16;
        const u64 takeL = (lim - hiL) < 16 ? (lim - hiL) : 16;
        const u32 j = 31 - __builtin_clz(mm);
        best = (i64)(hiL + takeL - j);
        bestc = (g >> j) & 1;  // 1: the nearest is '>'
      }
    }
    if (fmt == F_FASTA) {
      guess = (best < 0) ? 1 : (bestc ? 0 : 1);  // state = count 0 << 1 | armed
    } else {
      // SAM: byte before data[0] is '\n' -> FRESH; else class of the byte after the nearest '\n'
      if (front == 0 || best == 1) guess = 0;
      else if (best < 0) guess = 1;
      else guess = (data[-(best - 1)] == '@') ? 2 : 1;
    }
  }
  if (lane == 0) *out = guess;
}

template <int F>
__device__ __forceinline__ bool slab_compatible(u64 truth, u64 guess) {
  if (F == F_FASTQ) return (truth & 3) == (guess & 3);
  if (F == F_FASTA) return (truth & 1) == (guess & 1);
  if (F == F_SAM) return (truth & 3) == (guess & 3);
  return true;
}
template <int F>
__device__ __forceinline__ u64 slab_delta(u64 truth, u64 guess) {  // global - local record numbers
  if (F == F_FASTQ) return (truth - (guess & 3)) >> 2;
  if (F == F_FASTA) return (truth >> 1) - (guess >> 1);
  if (F == F_SAM) return (truth >> 2) - (guess >> 2);
  return truth - guess;
}

// The caller's expected build tag of every slab's summary (shockidx_slab_combine's expect_seq).
struct SeqExpect {
  u32 v[32];
  u32 on;
};
template <int F>
__device__ void slab_combine(const SlabSummary *all, int world, int rank, const SeqExpect &ex, SlabPlan *out) {
  typedef typename Traits<F>::M M;
  SlabPlan pl;
  pl.inconsistent = 0; pl.flags = 0; pl.err_rank = -1; pl.err_pos = 0; pl.err_len = 0; pl.code = ST_OK;
  pl.count = 0; pl.state_in = 0; pl.first_record = 0;
  u64 s = 0;  // state before slab 0 (file start)
  bool done = false;
  for (int q = 0; q < world; ++q) {
    const SlabSummary &x = all[q];
    if (ex.on && x.seq != ex.v[q]) pl.flags |= 32;  // a stale summary: never folded into a result
    const bool ok = slab_compatible<F>(s, x.state_in);
    if (!ok) pl.inconsistent |= 1u << q;
    const u64 delta = slab_delta<F>(s, x.state_in);
    if (q == rank) { pl.state_in = s; pl.first_record = delta + x.row_base; }
    pl.flags |= x.flags & ~1u;
    if (!done && ok) {
      if (x.key != KEY_NONE) {
        pl.count = (x.key >> KEY_REC_SHIFT) + delta;
        pl.code = (u32)(x.key & 15);
        if (pl.code == ST_FA_INVALID) { pl.err_rank = q; pl.err_pos = x.err_pos; pl.err_len = x.err_len; }
        done = true;
      } else if (q == world - 1) {
        pl.count = x.natural + delta;
      }
    }
    s = M::apply(s, x.agg);
  }
  *out = pl;
}

__global__ void k_slab_combine(const SlabSummary *all, int world, int rank, int fmt, const SeqExpect ex, SlabPlan *out) {
  if (threadIdx.x || blockIdx.x) return;
  if (fmt == F_FASTQ) slab_combine<F_FASTQ>(all, world, rank, ex, out);
  else if (fmt == F_FASTA) slab_combine<F_FASTA>(all, world, rank, ex, out);
  else if (fmt == F_SAM) slab_combine<F_SAM>(all, world, rank, ex, out);
  else slab_combine<F_LINE>(all, world, rank, ex, out);
}

// ====================================================================================
// k_detect: multi.go:43-62 over the zero-padded first 32768 bytes (fasta, fastq, sam)
// ====================================================================================
struct DetBuf {
  const uint8_t *d;  // the zero-padded 32768-byte head, staged in LDS
  __device__ __forceinline__ u32 at(u64 i) const { return d[i]; }
};
__device__ __forceinline__ bool dS(u32 c) { return !(c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == ' '); }
__device__ __forceinline__ bool dSST(u32 c) { return !(c == '\n' || c == '\f' || c == '\r'); }
__device__ __forceinline__ bool dNR(u32 c) { return c == '\n' || c == '\r'; }
__device__ __forceinline__ bool dAlpha(u32 c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

// The matchers run wave-wide: every "class run" of the regex is skipped 64 bytes at a time
// (one byte per lane, a ballot for the first byte outside the class); single-byte checks are
// uniform LDS reads.  skip(b, i, P): the first j >= i with !P(b[j]), N if none.
template <class P>
__device__ __forceinline__ u64 det_skip(const DetBuf &b, u64 i, P pred) {
  const u64 N = 32768;
  const int lane = threadIdx.x & 63;
  for (u64 base = i; base < N; base += 64) {
    const u64 q = base + (u64)lane;
    const u64 m = __ballot(q < N && !pred(b.at(q)));
    if (m) return base + (u64)__builtin_ctzll(m);
  }
  return N;
}
__device__ __forceinline__ bool dLetDash(u32 c) { return dAlpha(c) || c == '-'; }

// fasta.go:22  ^[\n\r]*>\S+[\S\t ]*[\n\r]+[A-Za-z\- ]+
__device__ bool det_fasta(const DetBuf &b) {
  const u64 N = 32768;
  u64 i = det_skip(b, 0, dNR);
  if (i >= N || b.at(i) != '>') return false;
  ++i;
  if (i >= N || !dS(b.at(i))) return false;
  i = det_skip(b, i + 1, dSST);
  if (i >= N || !dNR(b.at(i))) return false;
  i = det_skip(b, i, dNR);
  if (i >= N) return false;
  const u32 c = b.at(i);
  return dAlpha(c) || c == '-' || c == ' ';
}
// fastq.go:22  ^[\n\r]*@\S+[\S\t ]*[\n\r]+[A-Za-z\-]+[\n\r]+\+[\S\t ]*[\n\r]+\S*[\n\r]+
__device__ bool det_fastq(const DetBuf &b) {
  const u64 N = 32768;
  u64 i = det_skip(b, 0, dNR);
  if (i >= N || b.at(i) != '@') return false;
  ++i;
  if (i >= N || !dS(b.at(i))) return false;
  i = det_skip(b, i + 1, dSST);
  if (i >= N || !dNR(b.at(i))) return false;
  i = det_skip(b, i, dNR);
  if (i >= N || !dLetDash(b.at(i))) return false;
  i = det_skip(b, i, dLetDash);
  if (i >= N || !dNR(b.at(i))) return false;
  i = det_skip(b, i, dNR);
  if (i >= N || b.at(i) != '+') return false;
  i = det_skip(b, i + 1, dSST);
  const u64 k = det_skip(b, i, dNR) - i;
  if (k == 0) return false;
  if (k >= 2) return true;
  i = det_skip(b, i + 1, dS);
  return i < N && dNR(b.at(i));
}
// sam.go:17  ^[\n\r]*[@[A-Z][A-Z][ \t]+[\S \t]+[\n\r]]*
__device__ bool det_sam(const DetBuf &b) {
  const u64 N = 32768;
  u64 i = det_skip(b, 0, dNR);
  if (i >= N) return false;
  u32 c = b.at(i);
  if (!(c == '@' || c == '[' || (c >= 'A' && c <= 'Z'))) return false;
  ++i;
  c = b.at(i);
  if (i >= N || !(c >= 'A' && c <= 'Z')) return false;
  ++i;
  c = b.at(i);
  if (i >= N || !(c == ' ' || c == '\t')) return false;
  ++i;
  const u64 e = det_skip(b, i, dSST);
  return e > i && e < N && dNR(b.at(e));
}

// The head is staged into LDS by the whole workgroup (16 B per lane, every load in flight at
// once), then three waves run the three matchers against LDS.
constexpr int DET_THREADS = 512;
__global__ __launch_bounds__(DET_THREADS) void k_detect(const uint8_t *data, u64 n, int *out) {
  __shared__ __align__(16) uint8_t head[32768];
  const u64 m = n < 32768 ? n : 32768;
  constexpr int PER = 32768 / 16 / DET_THREADS;
  uint4 v[PER];  // every load in flight before the first LDS store
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u64 a = (u64)(threadIdx.x + k * DET_THREADS) * 16;
    v[k] = make_uint4(0, 0, 0, 0);
    if (a + 16 <= m) v[k] = load16(data + a);
    else if (a < m) v[k] = load16_partial(data, a, m);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) *reinterpret_cast<uint4 *>(&head[(u64)(threadIdx.x + k * DET_THREADS) * 16]) = v[k];
  __syncthreads();
  // the three matchers, one per wave (side by side), each wave-wide
  __shared__ int part[3];
  const DetBuf b{head};
  if (threadIdx.x < 192) {
    const int w = threadIdx.x >> 6;
    const int r = w == 0 ? (det_fasta(b) ? 1 : 0) : w == 1 ? (det_fastq(b) ? 2 : 0) : (det_sam(b) ? 4 : 0);
    if ((threadIdx.x & 63) == 0) part[w] = r;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const int mk = part[0] | part[1] | part[2];
  out[0] = (mk & 1) ? F_FASTA : (mk & 2) ? F_FASTQ : (mk & 4) ? F_SAM : F_NONE;
  out[1] = mk;
}

// ====================================================================================
// k_scan_excl<M>: the device-wide exclusive scan of the per-tile monoid aggregates -- the
// parallel form of record.go:76's serial `curr += int64(n)` (the global record number of a
// tile's first record is the fold of everything before it).  Single pass, decoupled
// look-back: 2048 aggregates per workgroup (8 per thread, thread -> wave -> block scans),
// the block's aggregate published as an epoch-tagged status word, then wave 0 folds its
// predecessors' words 64 at a time back to the nearest inclusive one.  Workgroups take their
// block number from a per-build ticket, so a block only ever waits on blocks that were
// already running (no residency assumption).  The block holding the last tile also writes
// the slab aggregate where k_finalize reads it (status[ntiles - 1]).
// ====================================================================================
constexpr int SCAN_T = 256, SCAN_ITEMS = 8, SCAN_BLOCK = SCAN_T * SCAN_ITEMS;

template <class M>
__global__ __launch_bounds__(SCAN_T) void k_scan_excl(const u64 *agg, u64 *excl, u32 n, u64 *look, u32 *ticket,
                                                      u64 *total_word, u32 epoch, u64 in_mask, const int *gate,
                                                      int gate_fmt) {
  __shared__ u64 wtot[SCAN_T / 64];
  __shared__ u64 bpre;
  __shared__ u32 sbid;
  if (gate && *gate != gate_fmt) return;  // format speculation failed (no ticket taken)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) sbid = __hip_atomic_fetch_add((gu32 *)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const u32 bid = sbid;
  const u64 i0 = (u64)bid * SCAN_BLOCK + (u64)tid * SCAN_ITEMS;
  u64 v[SCAN_ITEMS];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) v[k] = (i0 + k < n) ? (agg[i0 + k] & in_mask) : M::identity();
#pragma unroll
  for (int k = 1; k < SCAN_ITEMS; ++k) v[k] = M::combine(v[k - 1], v[k]);
  const u64 tinc = wave_incl_scan<M>(v[SCAN_ITEMS - 1], lane);
  u64 texc = __shfl_up(tinc, 1, 64);
  if (lane == 0) texc = M::identity();
  if (lane == 63) wtot[wid] = tinc;
  __syncthreads();
  u64 wpre = M::identity(), btot = M::identity();
#pragma unroll
  for (int w = 0; w < SCAN_T / 64; ++w) {
    if (w < wid) wpre = M::combine(wpre, wtot[w]);
    btot = M::combine(btot, wtot[w]);
  }
  if (wid == 0) {
    gu64 *lk = (gu64 *)look;
    const u64 tag = (u64)epoch << EPOCH_SHIFT;
    u64 pre = M::identity();
    if (bid == 0) {
      if (lane == 0) st_store(lk, FLAG_INC | tag | btot);
    } else {
      if (lane == 0) st_store(lk + bid, FLAG_AGG | tag | btot);
      u64 acc = M::identity();  // fold of the blocks between the window and this one
      i64 hi = (i64)bid - 1;    // newest block of the window (lane 0)
      for (;;) {
        const i64 idx = hi - lane;
        u64 w = idx >= 0 ? st_load(lk + idx) : (FLAG_INC | tag | M::identity());
        u64 incm, zm;
        for (;;) {
          const u32 f = wflag(w, epoch);
          incm = __ballot(f == 2);
          zm = __ballot(f == 0);
          const u64 need = incm ? lowmask(ctz64(incm)) : ~0ull;  // lanes newer than the INC
          if (!(zm & need)) break;
          __builtin_amdgcn_s_sleep(1);
          if (f == 0) w = st_load(lk + idx);
        }
        const u32 fi = incm ? ctz64(incm) : 64u;
        const u64 x = ((u32)lane <= fi) ? (w & PAYLOAD_MASK) : M::identity();
        const u64 fold = __shfl(wave_fold_newest_first<M>(x, lane), 0, 64);
        acc = M::combine(fold, acc);
        if (incm) break;
        hi -= 64;
      }
      pre = acc;
      if (lane == 0) st_store(lk + bid, FLAG_INC | tag | M::combine(pre, btot));
    }
    if (lane == 0) {
      bpre = pre;
      if ((u64)bid * SCAN_BLOCK < n && (u64)(bid + 1) * SCAN_BLOCK >= n)  // the block of the last tile
        st_store((gu64 *)total_word, FLAG_INC | tag | M::combine(pre, btot));
    }
  }
  __syncthreads();
  const u64 base = M::combine(bpre, M::combine(wpre, texc));
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (i0 + k < n) excl[i0 + k] = k ? M::combine(base, v[k - 1]) : base;
}

}  // namespace sidx

// ====================================================================================
// Host launch wrappers (internal to libshockidx; the C ABI lives in sidx_capi.cpp)
// ====================================================================================
using namespace sidx;

extern "C" hipError_t sidx_launch_detect(const uint8_t *d, u64 n, int *d_out, hipStream_t s) {
  hipLaunchKernelGGL(k_detect, dim3(1), dim3(DET_THREADS), 0, s, d, n, d_out);
  return hipGetLastError();
}

// look-back words of the scans: two arrays of the status block (SlabParams::scan_look)
namespace {
// The persistent grid of a tile kernel: CUs x its own co-resident workgroups (the launch
// parameters' pgrid is sized for k_fq_tiles; a larger grid than fits would leave the extra
// workgroups to start after the others finish their whole tile sequence).
template <class K>
int occupancy(K kern) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, SNT, 0) == hipSuccess && n > 0 ? n : 1;
}
u32 tile_grid(const SlabParams &p, int which) {
  // cached per device and kernel; written from the multi-device slab threads at once, so the
  // cache words are atomics (a repeated query stores the same value)
  static std::atomic<int> occ[4], cus[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::atomic<int> &cu_slot = cus[dev & 63];
  int cu = cu_slot.load(std::memory_order_relaxed);
  if (!cu) {
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
    cu_slot.store(cu, std::memory_order_relaxed);
  }
  int oc = occ[which].load(std::memory_order_relaxed);
  if (!oc) {
    oc = which == 1 ? occupancy(k_fa_tiles) : which == 3 ? occupancy(k_sam_tiles) : occupancy(k_line_tiles);
    occ[which].store(oc, std::memory_order_relaxed);
  }
  const u64 g = (u64)(cu > 0 ? cu : 1) * (u64)(oc > 0 ? oc : 1);
  return (u32)(g < p.ntiles ? g : p.ntiles);
}
template <class M>
hipError_t scan_excl(const SlabParams &p, const u64 *agg, u64 *excl, int which, bool total, hipStream_t s,
                     u64 in_mask = ~0ull) {
  const u32 nb = (p.ntiles + SCAN_BLOCK - 1) / SCAN_BLOCK;
  hipLaunchKernelGGL(k_scan_excl<M>, dim3(nb ? nb : 1), dim3(SCAN_T), 0, s, agg, excl, p.ntiles,
                     p.scan_look[which], p.counters + 4 + which, total ? p.status + (p.ntiles - 1) : p.scan_look[which] + nb,
                     p.epoch, in_mask, p.gate, p.gate_fmt);
  return hipGetLastError();
}
}  // namespace

// Two-pass index (SAM; FASTA and line slabs; the general re-run): pass 1 (tile aggregates,
// their exclusive scan, the slab aggregate) then k_index1 with every tile's incoming state.
extern "C" hipError_t sidx_launch_index(int fmt, const SlabParams *pp, DevResult *d_res, hipStream_t s,
                                        hipEvent_t ek0, hipEvent_t ek1) {
  const SlabParams &p = *pp;
  u64 *agg = p.fq_agg, *excl = (u64 *)p.tile_excl;
  const dim3 g1(p.ntiles), block(NTHREADS);
  if (ek0) (void)hipEventRecord(ek0, s);
  hipError_t e = hipSuccess;
  switch (fmt) {
    case F_FASTQ: hipLaunchKernelGGL(k_tile_agg<F_FASTQ>, g1, block, 0, s, p, agg); e = scan_excl<CountMonoid>(p, agg, excl, 0, true, s); break;
    case F_FASTA: hipLaunchKernelGGL(k_tile_agg<F_FASTA>, g1, block, 0, s, p, agg); e = scan_excl<FastaMonoid>(p, agg, excl, 0, true, s); break;
    case F_SAM: hipLaunchKernelGGL(k_tile_agg<F_SAM>, g1, block, 0, s, p, agg); e = scan_excl<SamMonoid>(p, agg, excl, 0, true, s); break;
    case F_LINE: hipLaunchKernelGGL(k_tile_agg<F_LINE>, g1, block, 0, s, p, agg); e = scan_excl<CountMonoid>(p, agg, excl, 0, true, s); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  switch (fmt) {
    case F_FASTQ: hipLaunchKernelGGL(k_index1<F_FASTQ>, g1, block, 0, s, p); break;
    case F_FASTA: hipLaunchKernelGGL(k_index1<F_FASTA>, g1, block, 0, s, p); break;
    case F_SAM: hipLaunchKernelGGL(k_index1<F_SAM>, g1, block, 0, s, p); break;
    case F_LINE: hipLaunchKernelGGL(k_index1<F_LINE>, g1, block, 0, s, p); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ek1) (void)hipEventRecord(ek1, s);
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, p, fmt, d_res);
  return hipGetLastError();
}

extern "C" hipError_t sidx_launch_slab_guess(const uint8_t *d, u64 n, u64 front, int fmt, u64 *d_out,
                                             hipStream_t s) {
  hipLaunchKernelGGL(k_slab_guess, dim3(1), dim3(64), 0, s, d, n, front, fmt, d_out);
  return hipGetLastError();
}

extern "C" hipError_t sidx_launch_slab_combine(const void *d_all, int world, int rank, int fmt, const uint32_t *expect,
                                               void *d_plan, hipStream_t s) {
  SeqExpect ex;
  memset(&ex, 0, sizeof ex);
  if (expect) {
    ex.on = 1;
    for (int q = 0; q < world && q < 32; ++q) ex.v[q] = expect[q];
  }
  hipLaunchKernelGGL(k_slab_combine, dim3(1), dim3(64), 0, s, (const SlabSummary *)d_all, world, rank, fmt, ex,
                     (SlabPlan *)d_plan);
  return hipGetLastError();
}

// Whole-table check (SHOCKIDX_VERIFY builds, on in the GPU test suite): every row starts where
// the previous one ends (record.go:51-83), over the rows the build reported (DevResult::count,
// read on the device after the pipeline); a violation sets the internal-error flag.
__global__ __launch_bounds__(256) void k_verify_rows(const u64 *rows, u64 row_base, u64 row_cap, DevResult *res) {
  const DevResult r = *res;
  if (r.flags & 17) return;  // a capacity overflow or a failed speculation: re-run anyway
  const u64 nr = r.count > row_base ? r.count - row_base : 0;
  const u64 n = nr < row_cap ? nr : row_cap;
  bool bad = false;
  for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i + 1 < n; i += (u64)gridDim.x * 256) {
    const ulonglong2 a = reinterpret_cast<const ulonglong2 *>(rows)[i];
    bad |= a.x + a.y != rows[2 * (i + 1)];
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&res->flags, 2u);
}
extern "C" hipError_t sidx_launch_verify_rows(const u64 *rows, u64 row_base, u64 row_cap, DevResult *d_res, hipStream_t s) {
  hipLaunchKernelGGL(k_verify_rows, dim3(1024), dim3(256), 0, s, rows, row_base, row_cap, d_res);
  return hipGetLastError();
}

constexpr u32 FIX_GRID = 64;  // k_fixup workgroups: the queue is short on real data (a few items per 10 GiB)
// The FASTQ tile pass: k_fq_tiles, the exclusive scan of the tile newline counts (and the
// slab aggregate), k_fq_place, k_fixup, k_finalize.  index_ms (ek0 -> ek1) covers
// k_fq_tiles alone.
extern "C" hipError_t sidx_launch_fq_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                           hipEvent_t ek1) {
  const SlabParams &p = *pp;
  // ek0 / ek1 time the tile pass alone: recorded by its dispatch packet (hipExtLaunchKernel),
  // not as separate stream packets that would add their own gaps to the build
  if (p.fq_lines) hipExtLaunchKernelGGL(k_fq_tiles<true>, dim3(p.pgrid), dim3(SNT), 0, s, ek0, ek1, 0, p);
  else hipExtLaunchKernelGGL(k_fq_tiles<false>, dim3(p.pgrid), dim3(SNT), 0, s, ek0, ek1, 0, p);
  hipError_t e = scan_excl<CountMonoid>(p, p.fq_agg, (u64 *)p.tile_excl, 0, true, s, FQW_TMASK);
  if (e != hipSuccess) return e;
  // test hook (SHOCKIDX_DEBUG bit 12): fail after the scan, as a launch error there would --
  // the build's ticket / first-bad slot is then left unreset (tests/test_gpu_host.py)
  if (p.debug & 4096u) return hipErrorLaunchFailure;
  const u64 pb = (p.ntiles + PLACE_TILES - 1) / PLACE_TILES;
  hipLaunchKernelGGL(k_fq_place, dim3((u32)(pb < 65536 ? pb : 65536)), dim3(256), 0, s, p);
  hipLaunchKernelGGL(k_fixup, dim3(FIX_GRID), dim3(256), 0, s, p, d_res);  // (finalizes the build)
  return hipGetLastError();
}

extern "C" hipError_t sidx_launch_fq_spans_place(const SlabParams *pp, u32 *spans, u64 *outlen, u64 K, int kind,
                                                hipStream_t s) {
  const SlabParams &p = *pp;
  if (!p.fq_lines || !p.ntiles) return hipSuccess;
  const u64 wb = (p.ntiles + 3) / 4;
  hipLaunchKernelGGL(k_fq_spans_place, dim3((u32)(wb < 65536 ? wb : 65536)), dim3(256), 0, s, p, spans, outlen, K, kind);
  return hipGetLastError();
}

// The line tile pass: k_line_tiles, the count scan (row bases, slab aggregate) and the max
// scan of the last '\n' + 1 (each tile's first row start), k_line_place, k_line_final.
extern "C" hipError_t sidx_launch_line_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                             hipEvent_t ek1) {
  const SlabParams &p = *pp;
  SlabParams q = p;
  q.pgrid = tile_grid(p, 2);
  hipExtLaunchKernelGGL(k_line_tiles, dim3(q.pgrid), dim3(SNT), 0, s, ek0, ek1, 0, q);
  hipError_t e = scan_excl<CountMonoid>(p, p.fq_agg, (u64 *)p.tile_excl, 0, true, s, LCOUNT);
  if (e == hipSuccess) e = scan_excl<MaxMonoid>(p, p.pcnt, p.ppre, 1, false, s);
  if (e != hipSuccess) return e;
  const u64 wb = (p.ntiles + LPLACE_TILES - 1) / LPLACE_TILES;
  hipLaunchKernelGGL(k_line_place<F_LINE>, dim3((u32)(wb < 65536 ? wb : 65536)), dim3(256), 0, s, p);
  hipLaunchKernelGGL(k_line_final, dim3(1), dim3(64), 0, s, p);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, p, F_LINE, d_res);
  return hipGetLastError();
}

// The SAM tile pass (single-slab builds): k_sam_tiles, the SamMonoid scan (incoming states,
// the slab aggregate), k_sam_resolve, the max scan of the last terminator + 1, placement,
// k_sam_final, k_finalize.
extern "C" hipError_t sidx_launch_sam_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                            hipEvent_t ek1) {
  const SlabParams &p = *pp;
  SlabParams q = p;
  q.pgrid = tile_grid(p, 3);
  hipExtLaunchKernelGGL(k_sam_tiles, dim3(q.pgrid), dim3(SNT), 0, s, ek0, ek1, 0, q);
  hipError_t e = scan_excl<SamMonoid>(p, p.fq_agg, (u64 *)p.tile_excl, 0, true, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sam_resolve, dim3((p.ntiles + 255) / 256), dim3(256), 0, s, p);
  e = scan_excl<MaxMonoid>(p, p.pcnt, p.ppre, 1, false, s);
  if (e != hipSuccess) return e;
  const u64 wb = (p.ntiles + LPLACE_TILES - 1) / LPLACE_TILES;
  hipLaunchKernelGGL(k_line_place<F_SAM>, dim3((u32)(wb < 65536 ? wb : 65536)), dim3(256), 0, s, p);
  hipLaunchKernelGGL(k_sam_final, dim3(1), dim3(64), 0, s, p);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, p, F_SAM, d_res);
  return hipGetLastError();
}

// SHOCKIDX_SAM_MODE=two: the two-pass SAM build instead of the tile pass
extern "C" int sidx_sam_tiles() {
  const char *e = getenv("SHOCKIDX_SAM_MODE");
  return (e && (!strcmp(e, "two") || !strcmp(e, "0"))) ? 0 : 1;
}

// SHOCKIDX_LINE_MODE=two: the two-pass line build instead of the tile pass
extern "C" int sidx_line_tiles() {
  const char *e = getenv("SHOCKIDX_LINE_MODE");
  return (e && (!strcmp(e, "two") || !strcmp(e, "0"))) ? 0 : 1;
}

// The FASTA tile pass: k_fa_tiles, the FastaMonoid scan of the tile aggregates, k_fa_place,
// k_fa_fixup, k_finalize.
extern "C" hipError_t sidx_launch_fa_tiles(const SlabParams *pp, DevResult *d_res, hipStream_t s, hipEvent_t ek0,
                                           hipEvent_t ek1) {
  const SlabParams &p = *pp;
  SlabParams q = p;
  q.pgrid = tile_grid(p, 1);
  hipExtLaunchKernelGGL(k_fa_tiles, dim3(q.pgrid), dim3(SNT), 0, s, ek0, ek1, 0, q);
  hipError_t e = scan_excl<FastaMonoid>(p, p.fq_agg, (u64 *)p.tile_excl, 0, true, s, FAW_AMASK);
  if (e != hipSuccess) return e;
  const u64 pb = (p.ntiles + PLACE_TILES - 1) / PLACE_TILES;
  hipLaunchKernelGGL(k_fa_place, dim3((u32)(pb < 65536 ? pb : 65536)), dim3(256), 0, s, p);
  hipLaunchKernelGGL(k_fa_fixup, dim3(FIX_GRID), dim3(256), 0, s, p, d_res);  // (finalizes the build)
  return hipGetLastError();
}

// SHOCKIDX_FA_MODE=two: the two-pass FASTA build (k_tile_agg + k_index1) instead of the tile pass
// (read per build, so one process can compare both)
extern "C" int sidx_fa_tiles() {
  const char *e = getenv("SHOCKIDX_FA_MODE");
  return (e && (!strcmp(e, "two") || !strcmp(e, "0"))) ? 0 : 1;
}

// Co-resident workgroups per CU of the tile passes (persistent grid = CUs x this).
// 1: the FASTQ tile pass appends to per-XCD logs whose cursors the host zeroes before the pass

extern "C" int sidx_tiles_blocks_per_cu() {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fq_tiles<false>, SNT, 0) == hipSuccess ? n : 0;
}
