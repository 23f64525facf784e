"""FASTQ tile-pass burst-size variants of the CURRENT sources (the product source is not
touched): FQ_BLK tiles' lines leave as one burst from wave 0.  The product rounds each workgroup's
tile block up to a multiple of FQ_BLK (C2: 366 -> 368 tiles); these variants round it to an even
count only and flush a partial batch at the block's end, so FQ_BLK need not divide it:
  fqb8   bursts of  8 tiles (1 KiB)
  fqb16  bursts of 16 tiles (2 KiB, the product's size; isolates the rounding)
  fqb24  bursts of 24 tiles (3 KiB; 22.2 KiB of LDS, still 7 workgroups per CU)
  fqrr16 / fqrr64  batches of 16 / 64 consecutive tiles dealt round-robin to the workgroups
         (grid-stride over batches: every workgroup's reads advance through one window of the
         input together, as in the grid-stride passes; bursts of 16)
  fqrr32t  batches of 32 while every workgroup gets one, then the rest in one batch per
         workgroup (no round in which some workgroups idle)
Links shock_amd/variants/libshockidx_<name>.so with the recipe of `make variant`.

  python tools/probes/fq_blk_variants.py && python tools/ab_inproc.py base fqb8 fqb16 fqb24
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

OLD_BLK = "constexpr u32 FQ_BLK = 16;"
OLD_LOOP = """  u64 P = (p.ntiles + G - 1) / G;
  P = P >= FQ_BLK ? (P + FQ_BLK - 1) / FQ_BLK * FQ_BLK : (P + 1) & ~1ull;
  const u64 tb = (u64)blockIdx.x * P, te = tb + P < p.ntiles ? tb + P : p.ntiles;
  for (u64 t = tb; t < te; ++t) {
    const u32 j = (u32)((t - tb) % FQ_BLK);
    tiles_iter<kSpans>(p, S, raw, t, tid, lane, wid, tacc, j, j == FQ_BLK - 1 || t + 1 == te);
    ++ntl;
  }"""
NEW_LOOP = """  u64 P = (p.ntiles + G - 1) / G;
  P = (P + 1) & ~1ull;
  const u64 tb = (u64)blockIdx.x * P, te = tb + P < p.ntiles ? tb + P : p.ntiles;
  u32 j = 0;
  for (u64 t = tb; t < te; ++t) {
    const bool flush = j == FQ_BLK - 1 || t + 1 == te;
    tiles_iter<kSpans>(p, S, raw, t, tid, lane, wid, tacc, j, flush);
    j = flush ? 0u : j + 1u;
    ++ntl;
  }"""


RR_LOOP = """  constexpr u64 B = FQ_RR;
  const u64 nbat = (p.ntiles + B - 1) / B;
  for (u64 c = blockIdx.x; c < nbat; c += G) {
    const u64 tb = c * B, te = tb + B < p.ntiles ? tb + B : p.ntiles;
    u32 j = 0;
    for (u64 t = tb; t < te; ++t) {
      const bool flush = j == FQ_BLK - 1 || t + 1 == te;
      tiles_iter<kSpans>(p, S, raw, t, tid, lane, wid, tacc, j, flush);
      j = flush ? 0u : j + 1u;
      ++ntl;
    }
  }"""


RRT_LOOP = """  constexpr u64 B = FQ_RR;
  const u64 full = p.ntiles / (B * G);  // rounds in which every workgroup takes a whole batch
  const u64 tfull = full * B * G;
  const u64 bt = ((p.ntiles - tfull + G - 1) / G + 1) & ~1ull;  // the last round's batches: the rest, evenly
  for (u64 r = 0; r <= full; ++r) {
    const u64 tb = r < full ? (r * G + blockIdx.x) * B : tfull + blockIdx.x * bt;
    const u64 tz = tb + (r < full ? B : bt), te = tz < p.ntiles ? tz : p.ntiles;
    u32 j = 0;
    for (u64 t = tb; t < te; ++t) {
      const bool flush = j == FQ_BLK - 1 || t + 1 == te;
      tiles_iter<kSpans>(p, S, raw, t, tid, lane, wid, tacc, j, flush);
      j = flush ? 0u : j + 1u;
      ++ntl;
    }
  }"""


def build(name, blk):
    tmp = tempfile.mkdtemp(prefix=name + "_")
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    rr = name.startswith("fqrr")
    loop = (RRT_LOOP if name.endswith("t") else RR_LOOP).replace("FQ_RR", str(blk)) if rr else NEW_LOOP
    for old, new in ((OLD_BLK, f"constexpr u32 FQ_BLK = {min(16, blk) if rr else blk};"), (OLD_LOOP, loop)):
        assert s.count(old) == 1, "k_fq_tiles moved: update the patch: " + old[:50]
        s = s.replace(old, new)
    open(k, "w").write(s)
    os.makedirs(os.path.join(src, "build"), exist_ok=True)
    shutil.copy(os.path.join(CSRC, "build", "sidx_multi.o"), os.path.join(src, "build", "sidx_multi.o"))
    os.makedirs(os.path.join(ROOT, "shock_amd", "variants"), exist_ok=True)
    subprocess.check_call(["make", "-s", "variant", "V=" + name, "VFLAGS=" + os.environ.get("VFLAGS", "")], cwd=src)
    shutil.move(os.path.join(tmp, "pkg", "variants", f"libshockidx_{name}.so"),
                os.path.join(ROOT, "shock_amd", "variants", f"libshockidx_{name}.so"))
    shutil.rmtree(tmp)


def main():
    names = sys.argv[1:] or ["fqb8", "fqb16", "fqb24"]
    for n in names:
        build(n, int(n[4:].rstrip("t") if n.startswith("fqrr") else n[3:]))


if __name__ == "__main__":
    main()
