"""Line tile-pass order variant of the CURRENT sources (the product source is not touched): the
product strides over single tiles in XCD-major order; lnrrN deals batches of N consecutive
tiles round-robin to the workgroups (as the FASTQ and FASTA passes now do), each workgroup's
append region sized by the tiles it gets.  Links shock_amd/variants/libshockidx_lnrr32.so.

  python tools/probes/line_rr_variants.py && python tools/ab_inproc.py base lnrr32 --kind line
"""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

PATCHES = [
    ("""  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  uint4 *stage16 = reinterpret_cast<uint4 *>(p.fq_stage);
  u64 wofs = (t * (p.ntiles / G) + (t < p.ntiles % G ? t : p.ntiles % G)) * (LCAP / 8);  // 16-byte units""",
     """  constexpr u64 B = BATCH;
  const u64 nbat = (p.ntiles + B - 1) / B, w = blockIdx.x;
  u64 bc = w, t = bc * B, te = t + B < p.ntiles ? t + B : p.ntiles;
  uint4 *stage16 = reinterpret_cast<uint4 *>(p.fq_stage);
  // the tiles of the workgroups before this one: batches w' + kG, B tiles each but the last batch
  const u64 q = nbat / G, r = nbat % G, vlast = nbat ? (nbat - 1) % G : 0, lastlen = nbat ? p.ntiles - (nbat - 1) * B : 0;
  u64 wofs = (B * (w * q + (w < r ? w : r)) - (nbat && vlast < w ? B - lastlen : 0)) * (LCAP / 8);  // 16-byte units"""),
    ("""    return n;
  };
  for (; t < p.ntiles; t += G) {
    __builtin_amdgcn_s_setprio(3);
    stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);""",
     """    return n;
  };
  for (; bc < nbat;) {
    __builtin_amdgcn_s_setprio(3);
    stage_tile<false>(p, t, (u32)(size_t)(lds_u8 *)raw, wid, lane);"""),
    ("""    if (T <= LCAP) wofs += (T + 7) / 8;
  }
  (void)flush_pending();  // the last tile's""",
     """    if (T <= LCAP) wofs += (T + 7) / 8;
    if (++t == te) {
      bc += G;
      t = bc * B;
      te = t + B < p.ntiles ? t + B : p.ntiles;
    }
  }
  (void)flush_pending();  // the last tile's"""),
]


def main():
    import sys
    for name in sys.argv[1:] or ["lnrr32"]:
        build(name)


def build(name):
    tmp = tempfile.mkdtemp(prefix=name + "_")
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    for old, new in PATCHES:
        assert s.count(old) == 1, "k_line_tiles moved: update the patch: " + old[:50]
        s = s.replace(old, new.replace("BATCH", name[4:]))
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
