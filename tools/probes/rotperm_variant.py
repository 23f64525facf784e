"""Mask-assembly variant of the CURRENT sources (the product source is not touched): a thread
reads its 64 bytes as four 16-byte chunks in a rotated order (chunk j at byte 16 ((j + k) & 3),
k = (tid >> 2) & 3, against LDS bank conflicts), and the product shifts each chunk's 16-bit mask
into place with a variable 64-bit shift.  Here the four masks are packed in read order with
constant shifts and the 64-bit word is rotated back by 16k bits with two byte permutes
(v_perm_b32, selectors computed once per thread) -- FASTQ's '\\n' mask and FASTA's '\\n' and '>'
masks.  Links shock_amd/variants/libshockidx_rotperm.so.

  python tools/probes/rotperm_variant.py && python tools/ab_inproc.py base rotperm [--fmt fasta]
"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

HELPER = """// chunks e[0..3] (16-bit masks in read order) -> the 64-bit mask in byte order: rotate left by
// 16k bits, k = (tid >> 2) & 3, as two byte permutes of the packed word
__device__ __forceinline__ u64 unrot_mask(u32 e0, u32 e1, u32 e2, u32 e3, int tid) {
  const u32 k2 = (((u32)tid >> 2) & 3u) * 0x02020202u;
  const u32 sel_lo = (0x0B0A0908u - k2) & 0x07070707u, sel_hi = (0x0F0E0D0Cu - k2) & 0x07070707u;
  const u32 lo = e0 | (e1 << 16), hi = e2 | (e3 << 16);
  return ((u64)__builtin_amdgcn_perm(hi, lo, sel_hi) << 32) | __builtin_amdgcn_perm(hi, lo, sel_lo);
}

"""
ANCHOR = "template <bool kFq>\n__device__ __forceinline__ void stage_tile(const SlabParams &p"

PATCHES = [
    ("""  u64 m = 0;  // 3-op equality flags; the rare suspect word ("\\n\\v") is re-checked exactly
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
    const uint4 v = *reinterpret_cast<const uint4 *>(raw + FRONT + tid * 64 + 16 * cj);
    m |= (u64)eq16x(v, '\\n') << (16 * cj);
  }""", """  u32 e[4];  // 3-op equality flags; the rare suspect word ("\\n\\v") is re-checked exactly
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
    e[j] = eq16x(*reinterpret_cast<const uint4 *>(raw + FRONT + tid * 64 + 16 * cj), '\\n');
  }
  u64 m = unrot_mask(e[0], e[1], e[2], e[3], tid);"""),
    ("""  u64 nl = 0, gt = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
    const uint4 v = *reinterpret_cast<const uint4 *>(r + tid * 64 + 16 * cj);
    nl |= (u64)eq16x(v, '\\n') << (16 * cj);
    gt |= (u64)eq16x(v, '>') << (16 * cj);
  }""", """  u32 en[4], eg[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const u32 cj = ((u32)j + ((u32)tid >> 2)) & 3u;
    const uint4 v = *reinterpret_cast<const uint4 *>(r + tid * 64 + 16 * cj);
    en[j] = eq16x(v, '\\n');
    eg[j] = eq16x(v, '>');
  }
  u64 nl = unrot_mask(en[0], en[1], en[2], en[3], tid), gt = unrot_mask(eg[0], eg[1], eg[2], eg[3], tid);"""),
]


def main():
    name = "rotperm"
    tmp = tempfile.mkdtemp(prefix=name + "_")
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    assert s.count(ANCHOR) == 1
    s = s.replace(ANCHOR, HELPER + ANCHOR)
    for old, new in PATCHES:
        assert s.count(old) == 1, "mask loop moved: update the patch: " + old[:50]
        s = s.replace(old, new)
    open(k, "w").write(s)
    os.makedirs(os.path.join(src, "build"), exist_ok=True)
    shutil.copy(os.path.join(CSRC, "build", "sidx_multi.o"), os.path.join(src, "build", "sidx_multi.o"))
    os.makedirs(os.path.join(ROOT, "shock_amd", "variants"), exist_ok=True)
    subprocess.check_call(["make", "-s", "variant", "V=" + name, "VFLAGS=" + os.environ.get("VFLAGS", "")], cwd=src)
    shutil.move(os.path.join(tmp, "pkg", "variants", f"libshockidx_{name}.so"),
                os.path.join(ROOT, "shock_amd", "variants", f"libshockidx_{name}.so"))
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
