"""Dev probe: does k_fq_tiles' time depend on where the 10 GiB input lands in HBM?  The same
synthetic file is materialised into several fresh allocations (earlier ones kept, so each lands
elsewhere) and each is built 6 times; prints the index kernel ms per allocation."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402

size = 10 << 30
ctx = Context(0)
sf = SynthFile(ctx, "fastq", size)
rows = ctx.alloc(16 * (sf.expected_count() + 1024))
keep = []
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    data = sf.window(0, size)
    t = []
    for i in range(6):
        r = ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
        t.append(r.timings["index_ms"])
    t.sort()
    print(f"alloc {trial} ptr {data.ptr:#x} index_ms min {t[0]:.3f} med {t[3]:.3f} max {t[-1]:.3f} ok {r.ok}", flush=True)
    keep.append(data)
