"""An early-DMA FASTA tile pass as a variant library of the CURRENT sources (the product source
is not touched): one LDS slot per workgroup as in the product, but the next tile's DMA is issued
as soon as the candidates are listed, so it crosses HBM while this tile's pieces are validated
and its word is written.  The validation then reads no tile bytes: the candidate loop captures
the four bytes each piece check needs (its first byte, the three before its closing '>'), the
open piece's certificate moves before the barrier, and what those bytes cannot settle is
deferred to k_fa_fixup.  Links shock_amd/variants/libshockidx_faearly.so (recipe of `make variant`).

  python tools/probes/fa_early_variant.py && python tools/ab_inproc.py base faearly --fmt fasta
"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

PATCHES = [
    # the tile was staged by the previous iteration (or the prologue)
    ("""  __builtin_amdgcn_s_setprio(3);  // as k_fq_tiles: DMA issue, then the certification, first
  stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);  // the tile alone: no halo, no front
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a wave classifies only the bytes it staged""",
     """  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a wave classifies only the bytes it staged"""),
    ("""  u32 finv, tcert, pad[2];
};""", """  u32 finv, tcert, pad[2];
  u32 cb[RCAP];    // the bytes a candidate's piece check reads: r[lo] | r[g-1] << 8 | r[g-2] << 16 | r[g-3] << 24
};"""),
    ("""      if (slot < (u32)RCAP) S.cand[slot] = (base + j) | (pga << 14);""",
     """      if (slot < (u32)RCAP) {
        S.cand[slot] = (base + j) | (pga << 14);
        const int g0 = (int)(base + j);  // (r[-3..-1]: the slot's front bytes, never used then)
        S.cb[slot] = (u32)r[pga] | ((u32)r[g0 - 1] << 8) | ((u32)r[g0 - 2] << 16) | ((u32)r[g0 - 3] << 24);
      }"""),
    ("""__device__ __forceinline__ void fa_iter(const SlabParams &p, FaSmem &S, uint8_t *raw, u64 t, int tid, int lane,
                                        int wid) {""",
     """__device__ __forceinline__ u32 fa_check_cap(u32 cb, const u64 *mnl, u32 lo, u32 g, bool part) {
  const u32 c0 = cb & 0xFFu, c1 = (cb >> 8) & 0xFFu, c2 = (cb >> 16) & 0xFFu, c3 = cb >> 24;
  if (g >= lo + 3) {
    const u32 wi = lo >> 6;
    u64 w[FA_NLW];
#pragma unroll
    for (int k = 0; k < FA_NLW; ++k) w[k] = wi + k < (u32)(TILE / 64) ? mnl[wi + k] : 0ull;
    w[0] &= ~0ull << (lo & 63);
    u32 q = ~0u;
#pragma unroll
    for (int k = FA_NLW - 1; k >= 0; --k)
      if (w[k]) q = ((wi + (u32)k) << 6) + ctz64(w[k]);
    if (ascii_nonspace(c0) && c1 == '\\n' && ascii_nonspace(c2) && q < g - 1) return FA_OK;
  }
  if (g == lo) return part ? FA_DEFER : FA_INV;
  if (c0 >= 0x80 || ascii_space(c0)) return FA_DEFER;  // the leading trim needs more bytes
  u32 e, ce;  // r[lo] is not a space, so the trailing trim stops at lo + 1 at the latest
  if (!ascii_space(c1)) { e = g; ce = c1; }
  else if (!ascii_space(c2)) { e = g - 1; ce = c2; }
  else if (!ascii_space(c3)) { e = g - 2; ce = c3; }
  else return FA_DEFER;
  if (ce >= 0x80) return FA_DEFER;
  if (fa_find_nl(mnl, lo, e) < e) return FA_OK;
  return part ? FA_DEFER : FA_INV;
}

__device__ __forceinline__ void fa_iter(const SlabParams &p, FaSmem &S, uint8_t *raw, u64 t, int tid, int lane,
                                        int wid) {"""),
    ("""      else st = fa_check(r, S.mnl, lo, g, lo == 0 && (t != 0 || !p.file_start));""",
     """      else st = fa_check_cap(S.cb[i], S.mnl, lo, g, lo == 0 && (t != 0 || !p.file_start));"""),
    ("""  for (; t < p.ntiles; t += G) fa_iter(p, S, raw, t, tid, lane, wid);""",
     """  if (t < p.ntiles) stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);
  for (; t < p.ntiles; t += G) fa_iter(p, S, raw, t, tid, lane, wid);"""),
]

TCERT_START = "  u32 *tw = p.fq_tiles + t * FAW;\n  if (tid == SNT - 1) {  // the certificate"
TCERT_END = "    S.tcert = (q > alast && q + 1 < tlen && ascii_nonspace(r[q - 1]) && ascii_nonspace(r[q + 1])) ? 1u : 0u;\n  }\n"
B2 = "  lds_barrier();\n  // ---- validation of the pieces that close at the candidates"
NEXT_DMA = """  lds_barrier();
  if (t + p.pgrid < p.ntiles) {  // every wave is past its last read of the slot: the next tile
    __builtin_amdgcn_s_setprio(3);
    stage_tile<false>(p, t + p.pgrid, (u32)(size_t)(lds_u8 *)raw, wid, lane);
    __builtin_amdgcn_s_setprio(0);
  }
  // ---- validation of the pieces that close at the candidates"""


def main():
    tmp = tempfile.mkdtemp(prefix="faearly_")
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    for old, new in PATCHES:
        assert s.count(old) == 1, "k_fa_tiles moved: update the patch: " + old[:60]
        s = s.replace(old, new)
    # the open piece's certificate (reads the tile) moves before the barrier that frees the slot
    a = s.index(TCERT_START)
    b = s.index(TCERT_END, a) + len(TCERT_END)
    blk = s[a:b]
    s = s[:a] + s[b:]
    assert s.count(B2) == 1
    s = s.replace(B2, blk + NEXT_DMA)
    open(k, "w").write(s)
    os.makedirs(os.path.join(src, "build"), exist_ok=True)
    shutil.copy(os.path.join(CSRC, "build", "sidx_multi.o"), os.path.join(src, "build", "sidx_multi.o"))
    os.makedirs(os.path.join(ROOT, "shock_amd", "variants"), exist_ok=True)
    subprocess.check_call(["make", "-s", "variant", "V=faearly", "VFLAGS=" + os.environ.get("VFLAGS", "")], cwd=src)
    shutil.move(os.path.join(tmp, "pkg", "variants", "libshockidx_faearly.so"),
                os.path.join(ROOT, "shock_amd", "variants", "libshockidx_faearly.so"))
    if os.environ.get("KEEP"):
        print(tmp)
    else:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
