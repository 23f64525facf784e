"""Rebuild the round-5 plus-line ID-compare experiment (SIDX_FQ_IDC, removed in 53bbd23) as a
variant library of the CURRENT sources, for the hunt in idc_hunt.py.

The experiment replaced the certifier's lds_diff4 loop with a compare that reads the 9 dwords
covering 32 ID bytes per side once and aligns them with v_alignbyte.  This script copies
shock_amd/csrc to a scratch directory, re-inserts that branch there (the product source is not
touched) and links shock_amd/variants/libshockidx_idc.so with the same recipe as `make variant`.

  python tools/probes/idc_variant.py
"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

OLD = """          for (u32 o = 0; o < nn; o += 16) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const u32 oo = o + 4 * (u32)j;
              if (oo < nn) diff |= lds_diff4(raw, ca + oo, cb + oo, nn - oo);
            }
          }
          idmis = diff != 0;"""
NEW = """          const u32 *wv = reinterpret_cast<const u32 *>(raw);
          for (u32 o = 0; o < nn; o += 32) {
            const u32 ia = (ca + o) >> 2, ib = (cb + o) >> 2, sa = (ca + o) & 3u, sb = (cb + o) & 3u;
            u32 A[9], B[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
              A[k] = wv[ia + k];
              B[k] = wv[ib + k];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const u32 oo = o + 4 * (u32)k;
              if (oo < nn) {
                const u32 rem = nn - oo, m = rem >= 4 ? ~0u : ((1u << (8 * rem)) - 1u);
                diff |= (__builtin_amdgcn_alignbyte(A[k + 1], A[k], sa) ^ __builtin_amdgcn_alignbyte(B[k + 1], B[k], sb)) & m;
              }
            }
          }
          idmis = diff != 0;"""


def main():
    tmp = tempfile.mkdtemp(prefix="idc_")
    src = os.path.join(tmp, "pkg", "csrc")  # (the sources include ../../include/shockidx.h)
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    assert s.count(OLD) == 1, "the certifier's ID-compare loop moved: update OLD"
    open(k, "w").write(s.replace(OLD, NEW))
    os.makedirs(os.path.join(src, "build"), exist_ok=True)
    shutil.copy(os.path.join(CSRC, "build", "sidx_multi.o"), os.path.join(src, "build", "sidx_multi.o"))
    os.makedirs(os.path.join(ROOT, "shock_amd", "variants"), exist_ok=True)
    subprocess.check_call(["make", "-s", "variant", "V=idc", "VFLAGS=" + os.environ.get("VFLAGS", "")], cwd=src)
    shutil.move(os.path.join(tmp, "pkg", "variants", "libshockidx_idc.so"),
                os.path.join(ROOT, "shock_amd", "variants", "libshockidx_idc.so"))
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
