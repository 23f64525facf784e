"""Per-phase cycle breakdown of k_fq_tiles (dev tool; needs the SIDX_DIAG variant:
`make -C shock_amd/csrc variant V=diag VFLAGS=-DSIDX_DIAG=1`, run with SHOCKIDX_VARIANT=diag).

usage: SHOCKIDX_VARIANT=diag python tools/phase_timing.py [size_gib]
Lane 0 of wave 0 (the certifying wave) and of wave 1 accumulate s_memtime ticks per phase
over every tile of their workgroup; printed as ticks per tile, summed over workgroups."""
import ctypes
import os
import sys

import numpy as np

os.environ["SHOCKIDX_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context, _lib  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402

size = int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 10 << 30
ctx = Context(0)
sf = SynthFile(ctx, "fastq", size)
data = sf.window(0, size)
rows = ctx.alloc(16 * (sf.expected_count() + 1024))
for _ in range(3):
    r = ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
L = _lib.lib()
L.shockidx_debug_tiles_grid.restype = ctypes.c_int
L.shockidx_debug_tiles_grid.argtypes = [ctypes.c_void_p]
nwg = L.shockidx_debug_tiles_grid(ctx._h)
out = np.zeros(9 * 2 * nwg, dtype=np.uint64)
L.shockidx_debug_timing(ctx._h, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(2 * nwg))
t = out.reshape(nwg, 2, 9).astype(np.float64)
names = ["dma issue+wait+bar", "mask+count+bar", "positions+bar", "guess+certify", "final barrier", "tile words"]
print(f"size {size} grid {nwg} index_ms {r.timings['index_ms']:.3f} ok {r.ok} count {r.count}")
for w in range(2):
    ntl = t[:, w, 8].sum()
    tot = t[:, w, :6].sum()
    print(f" wave {w}: {int(ntl)} tiles, {tot / ntl:.0f} ticks/tile")
    for k, nme in enumerate(names):
        print(f"   {nme:20s} {t[:, w, k].sum() / ntl:9.0f} ticks/tile  {100 * t[:, w, k].sum() / tot:5.1f}%")
