// sidx_device.hpp -- device-side building blocks for the gfx950 record indexer:
// SWAR byte classification, the per-format look-back monoids, ordered wave scans,
// Go bytes.TrimSpace / utf8 restated for the device, and the two byte accessors
// (lane: LDS tile + masks; wave: cooperative global-memory scan).
#pragma once
#include <hip/hip_runtime.h>

#include "sidx_common.hpp"

namespace sidx {

// ------------------------------------------------------------------------------------
// SWAR: 16 bytes (one dwordx4) -> 16-bit mask of bytes equal to c (bit i = byte i)
// ------------------------------------------------------------------------------------
// bit 7 of each byte set iff that byte differs from the pattern byte (exact: no borrows)
__device__ __forceinline__ u32 ne4(u32 w, u32 pat) {
  const u32 x = w ^ pat;
  return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// The four per-dword flag words are packed with byte dot products (v_dot4_u32_u8): each
// flag byte is 0 or 0x80, so dot4(flags, {1,2,4,8}) = 0x80 * nibble, no carries.
__device__ __forceinline__ u32 eq16(const uint4 v, u32 c) {
  const u32 pat = c * 0x01010101u;
  const u32 lo = __builtin_amdgcn_udot4(ne4(v.y, pat), 0x80402010u,
                                        __builtin_amdgcn_udot4(ne4(v.x, pat), 0x08040201u, 0u, false), false);
  const u32 hi = __builtin_amdgcn_udot4(ne4(v.w, pat), 0x80402010u,
                                        __builtin_amdgcn_udot4(ne4(v.z, pat), 0x08040201u, 0u, false), false);
  return ((lo >> 7) | (hi << 1)) ^ 0xFFFFu;  // lo = 0x80 * (bytes 0-7 mask), hi likewise
}

// Equality flags in 3 VALU per dword (v_xad_u32, v_bitop3, v_dot4): bit 7 of a byte is set
// if the byte equals the pattern byte (< 0x80) -- or if it is pattern ^ 1 directly above a
// flagged byte of the same dword (the borrow of x - 0x01010101 runs up through 0x01 bytes).
// So the 16-bit mask is exact unless two flags sit next to each other inside one dword; the
// caller checks that (eq_suspect) and recomputes such words with eq16.
__device__ __forceinline__ u32 eq4x(u32 w, u32 pat) {
  // (w ^ pat) - 0x01010101 in one v_xad_u32 (the compiler does not fuse two literal operands)
  u32 t;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(t) : "v"(w), "s"(pat), "v"(0xFEFEFEFFu));
  return t & ~w & 0x80808080u;
}
__device__ __forceinline__ u32 eq16x(const uint4 v, u32 c) {
  const u32 pat = c * 0x01010101u;
  const u32 lo = __builtin_amdgcn_udot4(eq4x(v.y, pat), 0x80402010u,
                                        __builtin_amdgcn_udot4(eq4x(v.x, pat), 0x08040201u, 0u, false), false);
  const u32 hi = __builtin_amdgcn_udot4(eq4x(v.w, pat), 0x80402010u,
                                        __builtin_amdgcn_udot4(eq4x(v.z, pat), 0x08040201u, 0u, false), false);
  return (lo >> 7) | (hi << 1);
}
// a 64-bit eq16x mask word may hold a false flag: two adjacent flags inside one dword (nibble)
__device__ __forceinline__ bool eq_suspect(u64 m) { return (m & (m >> 1) & 0x7777777777777777ull) != 0; }

__device__ __forceinline__ u64 lowmask(u32 k) { return k >= 64 ? ~0ull : ((1ull << k) - 1ull); }
__device__ __forceinline__ u32 ctz64(u64 x) { return (u32)__builtin_ctzll(x); }
__device__ __forceinline__ u32 clz64(u64 x) { return (u32)__builtin_clzll(x); }
__device__ __forceinline__ u32 popc64(u64 x) { return (u32)__popcll(x); }

__device__ __forceinline__ uint4 load16(const uint8_t *p) { return *reinterpret_cast<const uint4 *>(p); }

// bytes [a, lim) of the 16-byte chunk at a (lim - a < 16), zero-filled beyond
// (fully unrolled, no indexed local array: a dynamically indexed array would live in scratch)
__device__ __noinline__ uint4 load16_partial(const uint8_t *data, u64 a, u64 lim) {
  u32 w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const u32 b = (a + i < lim) ? (u32)data[a + i] : 0u;
    if (i < 4) w0 |= b << (8 * i);
    else if (i < 8) w1 |= b << (8 * (i - 4));
    else if (i < 12) w2 |= b << (8 * (i - 8));
    else w3 |= b << (8 * (i - 12));
  }
  return make_uint4(w0, w1, w2, w3);
}

// ------------------------------------------------------------------------------------
// Per-format monoids.  An aggregate summarises a byte segment; a state is what the
// sequential Go reader knows at a position.  combine(a, b) = a then b; apply(s, a).
// All packed into 62 bits (look-back payload).
// ------------------------------------------------------------------------------------

// FASTQ / LINE: newline count (fastq.go reads 4 lines per record; line.go 1).
struct CountMonoid {
  static __device__ __forceinline__ u64 identity() { return 0; }
  static __device__ __forceinline__ u64 combine(u64 a, u64 b) { return a + b; }
  static __device__ __forceinline__ u64 apply(u64 s, u64 a) { return s + a; }
  static __device__ __forceinline__ u64 seg(u64 nl, u64 /*x*/, u32 len) { return len ? popc64(nl) : 0; }
};

// Running maximum (the line tile pass: start of each tile's first row = last '\n' + 1
// before it).
struct MaxMonoid {
  static __device__ __forceinline__ u64 identity() { return 0; }
  static __device__ __forceinline__ u64 combine(u64 a, u64 b) { return a > b ? a : b; }
};

// FASTA (fasta.go:100-138): a '>' ends a record iff a '\n' occurred since the previous
// '>' ("armed").  Aggregate = count<<3 | delta<<2 | f, f: 0 identity, 1 const-0, 2 const-1;
// delta = the segment's first '>' has no '\n' before it inside the segment (it is a
// boundary iff the incoming state is armed).  State = count<<1 | armed.
struct FastaMonoid {
  static __device__ __forceinline__ u64 identity() { return 0; }
  static __device__ __forceinline__ u64 mk(u64 cnt, u32 d, u32 f) { return (cnt << 3) | ((u64)d << 2) | f; }
  static __device__ __forceinline__ u64 combine(u64 a, u64 b) {
    const u32 af = a & 3, bf = b & 3;
    if (af == 0) return mk((a >> 3) + (b >> 3), (b >> 2) & 1, bf);
    const u64 cnt = (a >> 3) + (b >> 3) + ((af == 2) ? ((b >> 2) & 1) : 0);
    return mk(cnt, (a >> 2) & 1, bf == 0 ? af : bf);
  }
  static __device__ __forceinline__ u64 apply(u64 s, u64 a) {
    const u32 armed = s & 1, f = a & 3;
    const u64 cnt = (s >> 1) + (a >> 3) + (armed ? ((a >> 2) & 1) : 0);
    const u32 arm2 = f == 0 ? armed : (f == 2 ? 1u : 0u);
    return (cnt << 1) | arm2;
  }
  // nl / gt: masks of a segment of len (<= 64) bytes
  static __device__ __forceinline__ u64 seg(u64 nl, u64 gt, u32 len) {
    if (!len) return 0;
    if (!gt) return mk(0, 0, nl ? 2u : 0u);
    u32 prev = ctz64(gt);
    const u32 delta = (nl & lowmask(prev)) == 0;
    u64 cnt = delta ? 0 : 1;
    u64 rem = gt & (gt - 1);
    while (rem) {
      const u32 g = ctz64(rem);
      if (nl & lowmask(g) & ~lowmask(prev + 1)) ++cnt;
      prev = g;
      rem &= rem - 1;
    }
    const u32 f = (prev < 63 && (nl >> (prev + 1))) ? 2u : 1u;
    return mk(cnt, delta, f);
  }
};

// SAM (sam.go:83-98): a record ends with a "terminator" line (>= 2 bytes, first byte not
// '@').  State of the open line at a segment edge: 0 FRESH (line starts here), 1 T, 2 H.
// Aggregate = count<<8 | dF<<5 | has_nl<<4 | cls0<<2 | c.  State = count<<2 | s.
struct SamMonoid {
  static __device__ __forceinline__ u64 identity() { return 0; }
  static __device__ __forceinline__ u64 mk(u64 cnt, u32 dF, u32 hn, u32 cls0, u32 c) {
    return (cnt << 8) | ((u64)dF << 5) | ((u64)hn << 4) | ((u64)cls0 << 2) | c;
  }
  static __device__ __forceinline__ u64 combine(u64 a, u64 b) {
    const u32 a_hn = (a >> 4) & 1, b_hn = (b >> 4) & 1;
    const u32 a_cls0 = (a >> 2) & 3, b_cls0 = (b >> 2) & 3;
    if (!a_hn) {
      const u32 cls0 = a_cls0 ? a_cls0 : b_cls0;
      if (!b_hn) return mk(0, 0, 0, cls0, 0);
      const u32 dF = a_cls0 ? (a_cls0 == 1) : ((b >> 5) & 1);
      return mk(b >> 8, dF, 1, cls0, b & 3);
    }
    const u32 mid = a & 3;
    if (b_hn) {
      const u64 add = mid == 1 ? 1 : (mid == 0 ? ((b >> 5) & 1) : 0);
      return mk((a >> 8) + (b >> 8) + add, (a >> 5) & 1, 1, a_cls0, b & 3);
    }
    return mk(a >> 8, (a >> 5) & 1, 1, a_cls0, mid == 0 ? b_cls0 : mid);
  }
  static __device__ __forceinline__ u64 apply(u64 s, u64 a) {
    const u32 st = s & 3;
    if (!((a >> 4) & 1)) {
      const u32 cls0 = (a >> 2) & 3;
      return (s & ~3ull) | (st == 0 ? cls0 : st);
    }
    const u64 add = st == 1 ? 1 : (st == 0 ? ((a >> 5) & 1) : 0);
    return ((((s >> 2) + (a >> 8) + add)) << 2) | (a & 3);
  }
  // nl / at masks of a segment of len (<= 64) bytes
  static __device__ __forceinline__ u64 seg(u64 nl, u64 at, u32 len) {
    if (!len) return 0;
    const u32 cls0 = (at & 1) ? 2u : 1u;
    if (!nl) return mk(0, 0, 0, cls0, 0);
    const u32 dF = !(nl & 1) && !(at & 1);
    const u32 L = 63 - clz64(nl);
    const u32 c = (L == len - 1) ? 0u : (((at >> (L + 1)) & 1) ? 2u : 1u);
    const u64 ts = (nl << 1) & ~nl & ~at & lowmask(L);
    return mk(popc64(ts), dF, 1, cls0, c);
  }
};

// ------------------------------------------------------------------------------------
// Wave / block ordered scans over a monoid (64-wide waves; lane order = byte order)
// ------------------------------------------------------------------------------------
template <class M>
__device__ __forceinline__ u64 wave_incl_scan(u64 x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u64 y = __shfl_up(x, d, 64);
    if (lane >= d) x = M::combine(y, x);
  }
  return x;
}

// lanes hold aggregates with lane 0 = NEWEST segment; returns (in lane 0) the fold
// combine(v[63], ..., v[0]).
template <class M>
__device__ __forceinline__ u64 wave_fold_newest_first(u64 v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u64 y = __shfl_down(v, d, 64);
    if (lane + d < 64) v = M::combine(y, v);
  }
  return v;
}

// lanes hold aggregates in byte order (lane 0 = OLDEST); returns the total in every lane
template <class M>
__device__ __forceinline__ u64 wave_total_in_order(u64 v, int lane) {
  const u64 inc = wave_incl_scan<M>(v, lane);
  return __shfl(inc, 63, 64);
}

// ------------------------------------------------------------------------------------
// Go bytes.TrimSpace / utf8 restated over an accessor (exactness on non-ASCII bytes)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool ascii_space(u32 c) {
  return c == 0x20 || (c >= 0x09 && c <= 0x0D);
}
__device__ __forceinline__ bool unicode_space(u32 r) {
  if (r <= 0xFF) return r == 0x20 || (r >= 0x09 && r <= 0x0D) || r == 0x85 || r == 0xA0;
  return r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 ||
         r == 0x202F || r == 0x205F || r == 0x3000;
}

// Byte view for the out-of-line Unicode path: byte(pos) = ptr[pos - base] (ptr may point
// into LDS or global memory; scalar arguments only, so no caller object lives in scratch).
struct Bytes {
  const uint8_t *ptr;
  u64 base;
  __device__ __forceinline__ u32 byte(u64 p) const { return ptr[p - base]; }
};

// unicode/utf8.DecodeRune on [p, lim)
__device__ __forceinline__ u32 decode_rune(const Bytes &a, u64 p, u64 lim, u32 &w) {
  if (p >= lim) { w = 0; return 0xFFFD; }
  const u32 p0 = a.byte(p);
  if (p0 < 0x80) { w = 1; return p0; }
  u32 sz, lo, hi;
  if (p0 >= 0xC2 && p0 <= 0xDF) { sz = 2; lo = 0x80; hi = 0xBF; }
  else if (p0 == 0xE0) { sz = 3; lo = 0xA0; hi = 0xBF; }
  else if ((p0 >= 0xE1 && p0 <= 0xEC) || p0 == 0xEE || p0 == 0xEF) { sz = 3; lo = 0x80; hi = 0xBF; }
  else if (p0 == 0xED) { sz = 3; lo = 0x80; hi = 0x9F; }
  else if (p0 == 0xF0) { sz = 4; lo = 0x90; hi = 0xBF; }
  else if (p0 >= 0xF1 && p0 <= 0xF3) { sz = 4; lo = 0x80; hi = 0xBF; }
  else if (p0 == 0xF4) { sz = 4; lo = 0x80; hi = 0x8F; }
  else { w = 1; return 0xFFFD; }
  if (lim - p < sz) { w = 1; return 0xFFFD; }
  const u32 b1 = a.byte(p + 1);
  if (b1 < lo || b1 > hi) { w = 1; return 0xFFFD; }
  if (sz == 2) { w = 2; return ((p0 & 0x1F) << 6) | (b1 & 0x3F); }
  const u32 b2 = a.byte(p + 2);
  if (b2 < 0x80 || b2 > 0xBF) { w = 1; return 0xFFFD; }
  if (sz == 3) { w = 3; return ((p0 & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F); }
  const u32 b3 = a.byte(p + 3);
  if (b3 < 0x80 || b3 > 0xBF) { w = 1; return 0xFFFD; }
  w = 4;
  return ((p0 & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((b2 & 0x3F) << 6) | (b3 & 0x3F);
}

// unicode/utf8.DecodeLastRune on [lo, end)
__device__ __forceinline__ u32 decode_last_rune(const Bytes &a, u64 lo, u64 end, u32 &w) {
  if (end <= lo) { w = 0; return 0xFFFD; }
  const u32 last = a.byte(end - 1);
  if (last < 0x80) { w = 1; return last; }
  i64 start = (i64)end - 1;
  i64 lim = (i64)end - 4;
  if (lim < (i64)lo) lim = (i64)lo;
  for (start--; start >= lim; start--)
    if ((a.byte((u64)start) & 0xC0) != 0x80) break;
  if (start < (i64)lo) start = (i64)lo;
  u32 size;
  const u32 r = decode_rune(a, (u64)start, end, size);
  if ((u64)start + size != end) { w = 1; return 0xFFFD; }
  w = size;
  return r;
}

// bytes.TrimFunc(s[a:b], unicode.IsSpace) -- the rare non-ASCII path, out of line, returns
// (lo, hi) packed as lo | hi << 32 relative to a (spans are < 4 GiB)
__device__ __noinline__ u64 trim_unicode(const uint8_t *ptr, u64 base, u64 a, u64 b) {
  const Bytes acc{ptr, base};
  u64 i = a;
  u32 w;
  while (i < b) {
    const u32 r = decode_rune(acc, i, b, w);
    if (!unicode_space(r)) break;
    i += w;
  }
  u64 j = b;
  i64 found = -1;
  while (j > i) {
    u32 r = acc.byte(j - 1), size = 1;
    if (r >= 0x80) r = decode_last_rune(acc, i, j, size);
    j -= size;
    if (!unicode_space(r)) { found = (i64)j; break; }
  }
  u64 hi;
  if (found < 0) {
    hi = i;
  } else if (acc.byte((u64)found) >= 0x80) {
    decode_rune(acc, (u64)found, b, w);
    hi = (u64)found + w;
  } else {
    hi = (u64)found + 1;
  }
  return (i - a) | ((hi - a) << 32);
}

// bytes.TrimSpace (Go >= 1.13): ASCII fast path, Unicode fallback at the first byte >= 0x80
template <class A>
__device__ __forceinline__ void trim_space(A &acc, u64 a, u64 b, u64 &tlo, u64 &thi) {
  u64 s = a;
  for (; s < b; ++s) {
    const u32 c = acc.byte(s);
    if (c >= 0x80) {
      const u64 r = trim_unicode(acc.ptr(), acc.base(), s, b);
      tlo = s + (u32)r; thi = s + (r >> 32);
      return;
    }
    if (!ascii_space(c)) break;
  }
  u64 e = b;
  for (; e > s; --e) {
    const u32 c = acc.byte(e - 1);
    if (c >= 0x80) {
      const u64 r = trim_unicode(acc.ptr(), acc.base(), s, e);
      tlo = s + (u32)r; thi = s + (r >> 32);
      return;
    }
    if (!ascii_space(c)) break;
  }
  tlo = s;
  thi = e;
}

// ------------------------------------------------------------------------------------
// Byte accessors
// ------------------------------------------------------------------------------------
enum FindResult : u32 { FR_FOUND = 0, FR_NONE = 1, FR_DEFER = 2, FR_NEEDMORE = 3 };
enum Cls : int { C_NL = 0, C_X = 1, C_NOTNL = 2 };  // C_X = '>' (FASTA) or '@' (SAM)

// Lane accessor: the tile [tlo, thi), a 16-byte front pad and a halo up to lhi are staged in
// LDS (raw bytes + per-byte masks); raw[0] holds byte tlo - FRONT.  Every byte a lane
// validator reads lies in [tlo - FRONT, lhi) by construction, so reads are LDS-only (no
// global load ever waits behind the next tile's prefetch); searches that would leave
// [tlo, lhi) return FR_DEFER (the wave path takes over).
constexpr int FRONT = 16;
struct LaneAcc {
  const uint8_t *raw;   // LDS copy of [tlo - FRONT, lhi)
  const u64 *mnl;       // LDS '\n' mask words (bit i of word w = byte tlo+64w+i)
  const u64 *mx;        // LDS class-X mask words
  u64 tlo, lhi, end;
  int eof;
  u32 dbg = 0;
  u64 front = 0;  // readable bytes before slab offset 0
  const uint16_t *nextx = nullptr;  // FASTA: first '>' at or after each mask word (0xFFFF: none)

  __device__ __forceinline__ u32 byte(u64 p) const { return (u32)raw[p - tlo + FRONT]; }
  __device__ __forceinline__ const uint8_t *ptr() const { return raw; }
  __device__ __forceinline__ u64 base() const { return tlo - FRONT; }
  __device__ __forceinline__ u64 word(int cls, u32 w) const {
    return cls == C_NL ? mnl[w] : (cls == C_X ? mx[w] : ~mnl[w]);
  }
  __device__ u32 find(int cls, u64 p, u64 lim, u64 &out) const {
    const u64 hi = lim < end ? lim : end;
    if (p < tlo) return FR_DEFER;
    const u64 stop = hi < lhi ? hi : lhi;
    if (cls == C_X && nextx && p < stop) {  // O(1): this word, else the suffix table
      const u32 r0 = (u32)(p - tlo), r1 = (u32)(stop - tlo);
      const u32 w = r0 >> 6;
      const u64 m = mx[w] & (~0ull << (r0 & 63));
      const u32 q = m ? (w << 6) + ctz64(m) : (u32)nextx[w + 1];
      if (q < r1) { out = tlo + q; return FR_FOUND; }
      if (stop == hi) return (hi == end && !eof) ? FR_NEEDMORE : FR_NONE;
      return FR_DEFER;
    }
    if (p < stop) {
      const u32 r0 = (u32)(p - tlo), r1 = (u32)(stop - tlo);
      u32 w = r0 >> 6;
      const u32 wl = (r1 - 1) >> 6;
      u64 m = word(cls, w) & (~0ull << (r0 & 63));
      for (;;) {
        if (w == wl && (r1 & 63)) m &= lowmask(r1 & 63);
        if (m) { out = tlo + ((u64)w << 6) + ctz64(m); return FR_FOUND; }
        if (w == wl) break;
        ++w;
        m = word(cls, w);
      }
    }
    if (stop == hi) return (hi == end && !eof) ? FR_NEEDMORE : FR_NONE;
    return FR_DEFER;
  }
};

// Wave accessor: all 64 lanes execute the same validator on the same record and search
// global memory cooperatively, 1 KiB (64 lanes x 16 B) per step, with a ballot.
struct WaveAcc {
  const uint8_t *g;
  u64 end;
  int eof;
  int lane;
  u64 front = 0;

  __device__ __forceinline__ u32 byte(u64 p) const { return g[p]; }
  __device__ __forceinline__ const uint8_t *ptr() const { return g; }
  __device__ __forceinline__ u64 base() const { return 0; }
  __device__ u32 find(int cls, u64 p, u64 lim, u64 &out) const {
    const u64 hi = lim < end ? lim : end;
    const u32 xc = cls == C_X ? (u32)'>' : (u32)'\n';
    for (u64 b = p & ~15ull; b < hi; b += 1024) {
      const u64 a = b + (u64)lane * 16;
      u32 m = 0;
      if (a < hi) {
        const uint4 v = (a + 16 <= end) ? load16(g + a) : load16_partial(g, a, end);
        m = cls == C_X ? eq16(v, xc) : eq16(v, '\n');
        if (cls == C_NOTNL) m = ~m & 0xFFFFu;
        if (a < p) m &= ~0u << (u32)(p - a);
        if (a + 16 > hi) m &= (1u << (u32)(hi - a)) - 1u;
      }
      const u64 bal = __ballot(m != 0);
      if (bal) {
        const int L = (int)ctz64(bal);
        const u64 pos = a + (m ? (u64)__builtin_ctz(m) : 0ull);
        out = __shfl(pos, L, 64);
        return FR_FOUND;
      }
    }
    return (hi == end && !eof) ? FR_NEEDMORE : FR_NONE;
  }
};

// A second class-X character for the wave accessor: SAM needs '@' not '>'.  The wave
// path of SAM never searches class X (only '\n'), FASTA searches '>'; so C_X means '>'
// in WaveAcc.  (LaneAcc reads whichever class mask the format staged.)

}  // namespace sidx
