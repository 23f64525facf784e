"""A two-slot FASTA tile pass as a variant library of the CURRENT sources (the product source is
not touched): each workgroup DMAs tile t + G into its second LDS slot before it classifies tile t,
so the next tile crosses HBM while this one is parsed (4 workgroups per CU instead of 7: two 16 KiB
slots each).  Copies shock_amd/csrc to a scratch directory, patches k_fa_tiles there and links
shock_amd/variants/libshockidx_fa2slot.so with the recipe of `make variant`.

  python tools/probes/fa2slot_variant.py && python tools/ab_inproc.py base fa2slot --fmt fasta
"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

OLD_STAGE = """  __builtin_amdgcn_s_setprio(3);  // as k_fq_tiles: DMA issue, then the certification, first
  stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);  // the tile alone: no halo, no front
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a wave classifies only the bytes it staged
  if (tid == 0) S.finv = FA_NONE;"""
NEW_STAGE = """  if (tid == 0) S.finv = FA_NONE;"""

OLD_LOOP = """  __shared__ __attribute__((aligned(16))) uint8_t raw[FRONT + TILE];
  __shared__ FaSmem S;
  if (gated_off(p)) return;  // format speculation failed: the host re-runs with the detected format
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 G = p.pgrid;
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  for (; t < p.ntiles; t += G) fa_iter(p, S, raw, t, tid, lane, wid);"""
NEW_LOOP = """  __shared__ __attribute__((aligned(16))) uint8_t raw2[2][FRONT + TILE];
  __shared__ FaSmem S;
  if (gated_off(p)) return;  // format speculation failed: the host re-runs with the detected format
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 G = p.pgrid;
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (t < p.ntiles) stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw2[0], wid, lane);
  int i = 0;
  for (; t < p.ntiles; t += G, i ^= 1) {
    if (t + G < p.ntiles) {  // the next tile into the other slot (read last by tile t - G, before its final barrier)
      __builtin_amdgcn_s_setprio(3);
      stage_tile<false>(p, t + G, (u32)(size_t)(lds_u8 *)raw2[i ^ 1], wid, lane);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile t's four pieces (loads return in order)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    fa_iter(p, S, raw2[i], t, tid, lane, wid);
  }"""


def main():
    tmp = tempfile.mkdtemp(prefix="fa2slot_")
    src = os.path.join(tmp, "pkg", "csrc")  # (the sources include ../../include/shockidx.h)
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    for old, new in ((OLD_STAGE, NEW_STAGE), (OLD_LOOP, NEW_LOOP)):
        assert s.count(old) == 1, "k_fa_tiles moved: update the patch"
        s = s.replace(old, new)
    open(k, "w").write(s)
    os.makedirs(os.path.join(src, "build"), exist_ok=True)
    shutil.copy(os.path.join(CSRC, "build", "sidx_multi.o"), os.path.join(src, "build", "sidx_multi.o"))
    os.makedirs(os.path.join(ROOT, "shock_amd", "variants"), exist_ok=True)
    vf = "-DSIDX_FA_WGS=4 " + os.environ.get("VFLAGS", "")
    subprocess.check_call(["make", "-s", "variant", "V=fa2slot", "VFLAGS=" + vf], cwd=src)
    shutil.move(os.path.join(tmp, "pkg", "variants", "libshockidx_fa2slot.so"),
                os.path.join(ROOT, "shock_amd", "variants", "libshockidx_fa2slot.so"))
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
