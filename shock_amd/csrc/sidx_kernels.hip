// sidx_kernels.hip -- gfx950 kernels of the MI355X record indexer.
//
//   k_detect     format detection (multi.go:43-62), one lane, <= 32 KiB inspected
//   k_index<F>   single-pass record index of one slab: coalesced 16 B/lane loads into LDS,
//                SWAR byte classes, ordered block scan of the format monoid, decoupled
//                look-back (62-bit payload + 2-bit flag, one sc1 store), record emission
//                with per-lane validation from LDS and a wave-cooperative global path for
//                records that cross the tile end
//   k_finalize   folds the slab's terminal state + first-bad key into a DevResult
//
// Reference semantics restated (paths relative to /root/reference/shock-server/):
//   record driver  node/file/index/record.go:34-90     line driver node/file/index/line.go:33-85
//   FASTQ          node/file/format/fastq/fastq.go:134-213
//   FASTA          node/file/format/fasta/fasta.go:93-140
//   SAM            node/file/format/sam/sam.go:83-98
//   line           node/file/format/line/line.go:37-45
#include <hip/hip_runtime.h>

#include "sidx_common.hpp"
#include "sidx_device.hpp"

namespace sidx {

constexpr u64 INF = ~0ull;

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
    if (s >= 4 && a.byte(s - 1) == '\n' && a.byte(s - 2) == '\n' && a.byte(s - 3) == '\n' &&
        a.byte(s - 4) == '\n')
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

template <int F>
struct __align__(16) Smem {
  uint8_t raw[TILE];
  u64 mnl[TILE / 64];
  u64 mx[Traits<F>::kX ? TILE / 64 : 1];
  u64 wtot[NWAVES];
  u64 tile_in;
  u64 badkey;
  u64 defer_s[MAX_DEFER];
  u64 defer_k[MAX_DEFER];
  u64 defer_aux[MAX_DEFER];
  u32 ndefer;
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
  const u64 key = (k << 26) | ((u64)(tile & ((1u << KEY_TILE_BITS) - 1)) << 4) | st;
  if (key < b.key) { b.key = key; b.pos = pos; b.len = len; }
}

template <int F, class A>
__device__ __forceinline__ void finish_record(const SlabParams &p, A &a, u32 tile, u64 s, u64 k,
                                              u64 aux, Bad &bad, Smem<F> *sm) {
  u64 len = 0, epos = 0, elen = 0;
  const u32 st = run_record<F>(a, s, aux, len, epos, elen);
  if (st == ST_OK) {
    put_row(p, k, s, len);
  } else if (st == ST_DEFER) {
    const u32 slot = atomicAdd(&sm->ndefer, 1u);
    if (slot < MAX_DEFER) {
      sm->defer_s[slot] = s;
      sm->defer_k[slot] = k;
      sm->defer_aux[slot] = aux;
    } else {
      atomicAdd(&p.counters[1], 1u);  // never silently dropped: finalize flags an error
    }
  } else {
    note_bad(bad, k, tile, st, p.base + epos, elen);
  }
}

// ====================================================================================
// Look-back (wave 0).  Returns the monoid state before `tile`.
// ====================================================================================
template <int F>
__device__ u64 wave_tile_aggregate(const SlabParams &p, u64 tile, int lane) {
  // self-help: aggregate of another tile straight from global memory (rare path)
  typedef typename Traits<F>::M M;
  const u64 lo = tile * TILE;
  const u64 hi = (lo + TILE < p.n) ? lo + TILE : p.n;
  u64 acc = M::identity();
  for (u64 b = lo; b < hi; b += 1024) {
    const u64 a = b + (u64)lane * 16;
    u64 agg = M::identity();
    if (a < hi) {
      const uint4 v = (a + 16 <= hi) ? load16(p.data + a) : load16_partial(p.data, a, hi);
      const u32 nl = eq16(v, '\n');
      const u32 x = Traits<F>::kX ? eq16(v, Traits<F>::xc) : 0u;
      agg = M::seg(nl, x, (u32)((hi - a) < 16 ? hi - a : 16));
    }
    acc = M::combine(acc, wave_total_in_order<M>(agg, lane));
  }
  return acc;
}

template <int F>
__device__ u64 lookback(const SlabParams &p, u64 tile, u64 tile_agg, int lane) {
  typedef typename Traits<F>::M M;
  if (tile == 0) {
    if (lane == 0)
      __hip_atomic_store(&p.status[0], FLAG_INC | M::apply(p.state_in, tile_agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    return p.state_in;
  }
  if (lane == 0)
    __hip_atomic_store(&p.status[tile], FLAG_AGG | tile_agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u64 acc = M::identity();  // aggregate of the tiles between the INC found and `tile`
  i64 hi = (i64)tile - 1;
  for (;;) {
    const i64 idx = hi - lane;
    u64 w = (idx >= 0) ? __hip_atomic_load(&p.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : (FLAG_INC | p.state_in);
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    u32 helped = 0;
    for (;;) {
      const u64 incm = __ballot((w >> 62) == 2);
      const u64 zerom = __ballot((w >> 62) == 0);
      const u32 first_inc = incm ? ctz64(incm) : 64u;
      const u64 need = zerom & lowmask(first_inc);
      if (!need) break;
      // bounded wait, then compute the missing aggregates ourselves (no reliance on
      // workgroup dispatch order for forward progress)
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000ull /* 200 us @ 100 MHz */) {
        const u32 L = ctz64(need);
        const u64 agg = wave_tile_aggregate<F>(p, (u64)(hi - (i64)L), lane);
        if (lane == (int)L) w = FLAG_AGG | agg;
        ++helped;
        continue;
      }
      __builtin_amdgcn_s_sleep(2);
      if ((w >> 62) == 0 && idx >= 0)
        w = __hip_atomic_load(&p.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (helped && lane == 0) atomicAdd(&p.counters[0], helped);
    const u64 incm = __ballot((w >> 62) == 2);
    const u32 first_inc = incm ? ctz64(incm) : 64u;
    const u64 v = ((u32)lane < first_inc) ? (w & PAYLOAD_MASK) : M::identity();
    const u64 win = __shfl(wave_fold_newest_first<M>(v, lane), 0, 64);
    acc = M::combine(win, acc);
    if (first_inc < 64) {
      const u64 st = M::apply(__shfl(w & PAYLOAD_MASK, (int)first_inc, 64), acc);
      if (lane == 0)  // publish the inclusive state so later tiles stop here
        __hip_atomic_store(&p.status[tile], FLAG_INC | M::apply(st, tile_agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      return st;
    }
    hi -= 64;
  }
}

// ====================================================================================
// k_index<F>: one workgroup per 32 KiB tile
// ====================================================================================
template <int F>
__global__ __launch_bounds__(NTHREADS) void k_index(const SlabParams p) {
  typedef typename Traits<F>::M M;
  __shared__ Smem<F> sm;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u32 tile = blockIdx.x;
  const u64 tlo = (u64)tile * TILE;
  const u64 thi = (tlo + TILE < p.n) ? tlo + TILE : p.n;
  const u32 tlen = (u32)(thi - tlo);

  if (tid == 0) { sm.ndefer = 0; sm.badkey = KEY_NONE; }

  // ---- 1. coalesced 16 B/lane loads -> LDS raw copy + per-byte class masks ----------
  {
    uint4 v[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const u32 off = (u32)(k * NTHREADS + tid) * CHUNK;
      if (off + CHUNK <= tlen) v[k] = load16(p.data + tlo + off);
      else if (off < tlen) v[k] = load16_partial(p.data, tlo + off, thi);
      else v[k] = make_uint4(0, 0, 0, 0);
    }
    uint16_t *mnl16 = reinterpret_cast<uint16_t *>(sm.mnl);
    uint16_t *mx16 = reinterpret_cast<uint16_t *>(sm.mx);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const u32 c = (u32)(k * NTHREADS + tid);
      *reinterpret_cast<uint4 *>(&sm.raw[c * CHUNK]) = v[k];
      mnl16[c] = (uint16_t)eq16(v[k], '\n');
      if (Traits<F>::kX) mx16[c] = (uint16_t)eq16(v[k], Traits<F>::xc);
    }
  }
  __syncthreads();

  // ---- 2. region (128 contiguous bytes per thread) aggregates + ordered block scan --
  const u32 rlo = (u32)tid * REGION;
  const u64 nl0 = sm.mnl[2 * tid], nl1 = sm.mnl[2 * tid + 1];
  const u64 x0 = Traits<F>::kX ? sm.mx[2 * tid] : 0, x1 = Traits<F>::kX ? sm.mx[2 * tid + 1] : 0;
  const u32 len0 = tlen > rlo ? (tlen - rlo >= 64 ? 64u : tlen - rlo) : 0u;
  const u32 len1 = tlen > rlo + 64 ? (tlen - rlo - 64 >= 64 ? 64u : tlen - rlo - 64) : 0u;
  const u64 ragg = M::combine(M::seg(nl0, x0, len0), M::seg(nl1, x1, len1));
  const u64 incl = wave_incl_scan<M>(ragg, lane);
  if (lane == 63) sm.wtot[wid] = incl;
  u64 lexcl = __shfl_up(incl, 1, 64);
  if (lane == 0) lexcl = M::identity();
  __syncthreads();
  u64 wpre = M::identity();
  for (int w = 0; w < wid; ++w) wpre = M::combine(wpre, sm.wtot[w]);
  const u64 texcl = M::combine(wpre, lexcl);

  // ---- 3. decoupled look-back by wave 0 ---------------------------------------------
  if (wid == 0) {
    u64 tagg = M::identity();
    for (int w = 0; w < NWAVES; ++w) tagg = M::combine(tagg, sm.wtot[w]);
    const u64 st = lookback<F>(p, tile, tagg, lane);
    if (lane == 0) sm.tile_in = st;
  }
  __syncthreads();
  const u64 tin = M::apply(sm.tile_in, texcl);  // state before this thread's region

  // ---- 4. emission: records owned by this region ------------------------------------
  LaneAcc acc;
  acc.g = p.data; acc.raw = sm.raw; acc.mnl = sm.mnl; acc.mx = sm.mx;
  acc.tlo = tlo; acc.thi = thi; acc.end = p.end; acc.eof = p.eof;
  Bad bad;

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
        if (F == F_LINE) {
          finish_record<F>(p, acc, tile, q + 1, j + 1, 0, bad, &sm);
        } else if ((j & 3) == 3) {
          finish_record<F>(p, acc, tile, q + 1, (j + 1) >> 2, 0, bad, &sm);
        }
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
        const u32 gbit = ctz64(m);
        m &= m - 1;
        const u32 g = 64 * h + gbit;
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
          term = (ls < q) && sm.raw[ls] != '@';
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
  __syncthreads();

  // ---- 5. deferred records: wave-cooperative global-memory path -------------------
  {
    const u32 nd = sm.ndefer < MAX_DEFER ? sm.ndefer : MAX_DEFER;
    WaveAcc wa;
    wa.g = p.data; wa.end = p.end; wa.eof = p.eof; wa.lane = lane;
    for (u32 i = wid; i < nd; i += NWAVES) {
      const u64 s = sm.defer_s[i], k = sm.defer_k[i], aux = sm.defer_aux[i];
      u64 len = 0, epos = 0, elen = 0;
      const u32 st = run_record<F>(wa, s, aux, len, epos, elen);
      if (lane == 0) {
        if (st == ST_OK) put_row(p, k, s, len);
        else note_bad(bad, k, tile, st, p.base + epos, elen);
      }
    }
  }

  // ---- 6. first bad record of the tile -> slab-wide min ------------------------------
  if (bad.key != KEY_NONE) atomicMin(&sm.badkey, bad.key);
  __syncthreads();
  const u64 tkey = sm.badkey;
  if (tkey != KEY_NONE) {
    if (bad.key == tkey) {
      p.detail[2 * (u64)tile] = bad.pos;
      p.detail[2 * (u64)tile + 1] = bad.len;
    }
    if (tid == 0) {
      const u64 cur = __hip_atomic_load(p.badkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tkey < cur) atomicMin(p.badkey, tkey);
    }
  }
}

// ====================================================================================
// k_finalize: slab result
// ====================================================================================
__global__ void k_finalize(const SlabParams p, int fmt, DevResult *res) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const u64 fin = p.status[p.ntiles - 1] & PAYLOAD_MASK;
  const u64 key = *p.badkey;
  DevResult r;
  r.state_out = fin;
  r.err_pos = 0;
  r.err_len = 0;
  r.flags = 0;
  r.selfhelp = p.counters[0];
  r.fmt = (u32)fmt;
  u64 krec = key >> 26;
  u32 kst = (u32)(key & 15);
  const u32 ktile = (u32)((key >> 4) & ((1u << KEY_TILE_BITS) - 1));
  u64 natural;  // count when no record terminates the sequence early
  if (fmt == F_FASTQ) natural = (fin >> 2) + 1;          // groups 0..T/4 all valid
  else if (fmt == F_FASTA) natural = (fin >> 1) + 1;     // records 0..B
  else if (fmt == F_SAM) natural = (fin >> 2) + 1;       // records 0..Tterm
  else natural = fin + 1;                                // lines 0..T
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
  const u64 nrows = r.count > p.row_base ? r.count - p.row_base : 0;
  if (nrows > p.row_cap) r.flags |= 1;
  *res = r;
}

// ====================================================================================
// k_detect: multi.go:43-62 over the zero-padded first 32768 bytes (fasta, fastq, sam)
// ====================================================================================
struct DetBuf {
  const uint8_t *d;
  u64 n;
  __device__ __forceinline__ u32 at(u64 i) const { return i < n ? d[i] : 0u; }  // zero pad
};
__device__ __forceinline__ bool dS(u32 c) { return !(c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == ' '); }
__device__ __forceinline__ bool dSST(u32 c) { return !(c == '\n' || c == '\f' || c == '\r'); }
__device__ __forceinline__ bool dNR(u32 c) { return c == '\n' || c == '\r'; }
__device__ __forceinline__ bool dAlpha(u32 c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

// fasta.go:22  ^[\n\r]*>\S+[\S\t ]*[\n\r]+[A-Za-z\- ]+
__device__ bool det_fasta(const DetBuf &b) {
  const u64 N = 32768;
  u64 i = 0;
  while (i < N && dNR(b.at(i))) ++i;
  if (i >= N || b.at(i) != '>') return false;
  ++i;
  if (i >= N || !dS(b.at(i))) return false;
  ++i;
  while (i < N && dSST(b.at(i))) ++i;
  if (i >= N || !dNR(b.at(i))) return false;
  while (i < N && dNR(b.at(i))) ++i;
  if (i >= N) return false;
  const u32 c = b.at(i);
  return dAlpha(c) || c == '-' || c == ' ';
}
// fastq.go:22  ^[\n\r]*@\S+[\S\t ]*[\n\r]+[A-Za-z\-]+[\n\r]+\+[\S\t ]*[\n\r]+\S*[\n\r]+
__device__ bool det_fastq(const DetBuf &b) {
  const u64 N = 32768;
  u64 i = 0;
  while (i < N && dNR(b.at(i))) ++i;
  if (i >= N || b.at(i) != '@') return false;
  ++i;
  if (i >= N || !dS(b.at(i))) return false;
  ++i;
  while (i < N && dSST(b.at(i))) ++i;
  if (i >= N || !dNR(b.at(i))) return false;
  while (i < N && dNR(b.at(i))) ++i;
  if (i >= N || !(dAlpha(b.at(i)) || b.at(i) == '-')) return false;
  while (i < N && (dAlpha(b.at(i)) || b.at(i) == '-')) ++i;
  if (i >= N || !dNR(b.at(i))) return false;
  while (i < N && dNR(b.at(i))) ++i;
  if (i >= N || b.at(i) != '+') return false;
  ++i;
  while (i < N && dSST(b.at(i))) ++i;
  u64 k = 0;
  while (i + k < N && dNR(b.at(i + k))) ++k;
  if (k == 0) return false;
  if (k >= 2) return true;
  ++i;
  while (i < N && dS(b.at(i))) ++i;
  return i < N && dNR(b.at(i));
}
// sam.go:17  ^[\n\r]*[@[A-Z][A-Z][ \t]+[\S \t]+[\n\r]]*
__device__ bool det_sam(const DetBuf &b) {
  const u64 N = 32768;
  u64 i = 0;
  while (i < N && dNR(b.at(i))) ++i;
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
  u64 run = 0;
  while (i < N && dSST(b.at(i))) { ++i; ++run; }
  return run >= 1 && i < N && dNR(b.at(i));
}

__global__ void k_detect(const uint8_t *data, u64 n, int *out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DetBuf b{data, n < 32768 ? n : 32768};
  const int m = (det_fasta(b) ? 1 : 0) | (det_fastq(b) ? 2 : 0) | (det_sam(b) ? 4 : 0);
  out[0] = (m & 1) ? F_FASTA : (m & 2) ? F_FASTQ : (m & 4) ? F_SAM : F_NONE;
  out[1] = m;
}

}  // namespace sidx

// ====================================================================================
// Host launch wrappers (internal to libshockidx; the C ABI lives in sidx_capi.cpp)
// ====================================================================================
using namespace sidx;

extern "C" hipError_t sidx_launch_detect(const uint8_t *d, u64 n, int *d_out, hipStream_t s) {
  hipLaunchKernelGGL(k_detect, dim3(1), dim3(64), 0, s, d, n, d_out);
  return hipGetLastError();
}

extern "C" hipError_t sidx_launch_index(int fmt, const SlabParams *pp, DevResult *d_res, hipStream_t s) {
  const SlabParams &p = *pp;
  hipError_t e = hipMemsetAsync(p.status, 0, (size_t)p.ntiles * sizeof(u64), s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(p.badkey, 0xFF, sizeof(u64), s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(p.counters, 0, 4 * sizeof(u32), s);
  if (e != hipSuccess) return e;
  const dim3 grid(p.ntiles), block(NTHREADS);
  switch (fmt) {
    case F_FASTQ: hipLaunchKernelGGL(k_index<F_FASTQ>, grid, block, 0, s, p); break;
    case F_FASTA: hipLaunchKernelGGL(k_index<F_FASTA>, grid, block, 0, s, p); break;
    case F_SAM: hipLaunchKernelGGL(k_index<F_SAM>, grid, block, 0, s, p); break;
    case F_LINE: hipLaunchKernelGGL(k_index<F_LINE>, grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, p, fmt, d_res);
  return hipGetLastError();
}
