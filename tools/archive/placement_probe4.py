"""Dev probe: does k_fq_tiles' time follow where its OUTPUT lands (the tile status words and the
record-start slots: SHOCKIDX_CONTIG_WS bits 1 / 2 = contiguous HBM)?  The node body is always
contiguous; each trial is a fresh context (fresh workspace allocations), 6 builds each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402

size = 10 << 30
base = Context(0)
sf = SynthFile(base, "fastq", size)
data = sf.window(0, size)
rows = base.alloc(16 * (sf.expected_count() + 1024))
for trial in range(4):
    for ws in ("0", "3"):
        os.environ["SHOCKIDX_CONTIG_WS"] = ws
        ctx = Context(0)
        t, k = [], []
        for i in range(6):
            r = ctx.build_device(data.ptr, size, rows.ptr, sf.expected_count() + 1024, kind="record", fmt="fastq")
            t.append(r.timings["index_ms"])
            k.append(r.timings["kernel_ms"])
        t.sort(); k.sort()
        print(f"trial {trial} ws={ws} tiles min {t[0]:.3f} med {t[3]:.3f}  build med {k[3]:.3f} ok {r.ok}", flush=True)
        ctx.close()
