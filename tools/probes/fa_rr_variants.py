"""FASTA tile-pass order variants (the product source is not touched).  Round 6 first measured these
against single tiles in XCD-major grid-stride order; the product now takes batches of FA_RR = 32
consecutive tiles round-robin, and these rebuild it with another batch size:
  farrN    batches of N tiles (N = 16, 24, 32, 48, 64 ...)
  farr32t  batches of 32 while every workgroup gets one, then the rest in one batch each
(the round-6 A/B against the grid-stride order patched the grid-stride loop; the product's loop
is patched here)
Links shock_amd/variants/libshockidx_<name>.so with the recipe of `make variant`.

  python tools/probes/fa_rr_variants.py && python tools/ab_inproc.py base farr32 farr32t --fmt fasta
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "shock_amd", "csrc")

OLD = """  const u64 nbat = (p.ntiles + FA_RR - 1) / FA_RR;
  for (u64 c = blockIdx.x; c < nbat; c += G) {
    const u64 tb = c * FA_RR, te = tb + FA_RR < p.ntiles ? tb + FA_RR : p.ntiles;
    for (u64 t = tb; t < te; ++t) fa_iter(p, S, raw, t, tid, lane, wid);
  }"""
RR = """  constexpr u64 B = BATCH;
  const u64 nbat = (p.ntiles + B - 1) / B;
  for (u64 c = blockIdx.x; c < nbat; c += G) {
    const u64 tb = c * B, te = tb + B < p.ntiles ? tb + B : p.ntiles;
    for (u64 t = tb; t < te; ++t) fa_iter(p, S, raw, t, tid, lane, wid);
  }"""
RRT = """  constexpr u64 B = 32;
  const u64 full = p.ntiles / (B * G);
  const u64 tfull = full * B * G;
  const u64 bt = (p.ntiles - tfull + G - 1) / G;
  for (u64 r = 0; r <= full; ++r) {
    const u64 tb = r < full ? (r * G + blockIdx.x) * B : tfull + blockIdx.x * bt;
    const u64 tz = tb + (r < full ? B : bt), te = tz < p.ntiles ? tz : p.ntiles;
    for (u64 t = tb; t < te; ++t) fa_iter(p, S, raw, t, tid, lane, wid);
  }"""


def build(name):
    tmp = tempfile.mkdtemp(prefix=name + "_")
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    k = os.path.join(src, "sidx_kernels.hip")
    s = open(k).read()
    assert s.count(OLD) == 1, "k_fa_tiles moved: update the patch"
    s = s.replace(OLD, RRT if name.endswith("t") else RR.replace("BATCH", name[4:]))
    open(k, "w").write(s)
    os.makedirs(os.path.join(src, "build"), exist_ok=True)
    shutil.copy(os.path.join(CSRC, "build", "sidx_multi.o"), os.path.join(src, "build", "sidx_multi.o"))
    os.makedirs(os.path.join(ROOT, "shock_amd", "variants"), exist_ok=True)
    subprocess.check_call(["make", "-s", "variant", "V=" + name, "VFLAGS=" + os.environ.get("VFLAGS", "")], cwd=src)
    shutil.move(os.path.join(tmp, "pkg", "variants", f"libshockidx_{name}.so"),
                os.path.join(ROOT, "shock_amd", "variants", f"libshockidx_{name}.so"))
    shutil.rmtree(tmp)


def main():
    for n in sys.argv[1:] or ["farr16", "farr64"]:
        build(n)


if __name__ == "__main__":
    main()
