"""Per-phase cycle breakdown of k_index (SHOCKIDX_TIMING diagnostic build path).  Dev tool."""
import ctypes, os, sys
import numpy as np
os.environ["SHOCKIDX_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context, _lib
from shock_amd.synth import SynthFile
fmt = sys.argv[1] if len(sys.argv) > 1 else "fastq"
size = int(float(sys.argv[2]) * (1 << 30)) if len(sys.argv) > 2 else 1 << 30
ctx = Context(0)
sf = SynthFile(ctx, fmt, size)
data = sf.window(0, size)
rows = ctx.alloc(16 * (sf.expected_count() + 1024))
for _ in range(3):
    r = ctx.build_buffer(data, size, rows, kind="record", fmt=fmt)
L = _lib.lib()
L.shockidx_debug_grid.restype = ctypes.c_int
nwg = L.shockidx_debug_grid(ctx._h, {"fasta": 1, "fastq": 2}[fmt])
if fmt == "fastq" and os.environ.get("SHOCKIDX_NO_PIPE", "0") != "1":
    L.shockidx_debug_pipe_grid.restype = ctypes.c_int
    nwg = L.shockidx_debug_pipe_grid(ctx._h)
    names = ["stage", "scan+publish", "nlpos", "validate", "prefix wait", "rows", "iter barrier", "-"]
    if os.environ.get("SHOCKIDX_KERNEL", "stream") != "pipe":
        names = ["dma wait+bar", "classify+count", "nlpos+halo", "guess+validate", "fold+j0+bar", "emission", "end barrier", "-"]
elif os.environ.get("SHOCKIDX_PERSIST", "0") != "1":
    nwg = 65536  # one tile per workgroup: phase sums land in 65536 slots
out = np.zeros(9 * nwg, dtype=np.uint64)
L.shockidx_debug_timing(ctx._h, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(nwg))
t = out.reshape(nwg, 9).astype(np.float64)
ntiles = t[:, 8].sum()
if "names" not in dir(): names = ["stage+wait", "scan", "lookback+nlpos", "barrier1", "emit(wave0)", "barrier2", "defer+badkey", "loopbar"]
tot = t[:, :8].sum()
print(f"fmt {fmt} size {size} grid {nwg} tiles {int(ntiles)} index_ms {r.timings['index_ms']:.3f} ok {r.ok} count {r.count} fixups {r.fixups}")
for k, nme in enumerate(names):
    print(f"  {nme:16s} {t[:, k].sum() / ntiles:10.0f} cycles/tile  {100 * t[:, k].sum() / tot:5.1f}%")
print(f"  total            {tot / ntiles:10.0f} cycles/tile (per workgroup, s_memtime ticks)")
