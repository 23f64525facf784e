"""Dev probe: which buffers want physically contiguous HBM?  For each SHOCKIDX_CONTIG mode (none,
user = shockidx_dev_alloc buffers only, all = also the context's workspaces) a fresh context
builds the 10 GiB synthetic FASTQ 8 times: k_fq_tiles ms and the whole build's kernel ms."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402

size = 10 << 30
for rnd in range(2):
    for mode in ("none", "user", "all"):
        os.environ["SHOCKIDX_CONTIG"] = mode
        ctx = Context(0)
        sf = SynthFile(ctx, "fastq", size)
        data = sf.window(0, size)
        rows = ctx.alloc(16 * (sf.expected_count() + 1024))
        t, k = [], []
        for i in range(8):
            r = ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
            t.append(r.timings["index_ms"])
            k.append(r.timings["kernel_ms"])
        t.sort(); k.sort()
        print(f"{mode:5s} tiles min {t[0]:.3f} med {t[4]:.3f}  build min {k[0]:.3f} med {k[4]:.3f}  rest med {k[4]-t[4]:.3f} ok {r.ok}", flush=True)
        data.free(); rows.free(); sf.free(); ctx.close()
