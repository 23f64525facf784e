"""Probe (round 5): which slab of a 4-slab FASTQ build breaks row contiguity, and where."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gen  # noqa: E402
import oracle  # noqa: E402
from shock_amd import Context, dist, _lib as L  # noqa: E402

os.environ["SHOCKIDX_VERIFY"] = "0"
data = gen.fastq(random.Random(13), 4000)
exp, err = oracle.record_index(data, "fastq")
print("size", len(data), "records", len(exp), err)
ctx = Context(0)
world = 4
size = len(data)
engs = []
for r, (lo, hi) in enumerate(dist.plan_slabs(size, world)):
    wlo, whi = dist.slab_window(size, lo, hi)
    buf = ctx.alloc(whi - wlo + 64)
    buf.upload(np.frombuffer(data[wlo:whi], np.uint8))
    cap = (hi - lo) // 8 + 64
    rows = ctx.alloc(16 * cap)
    e = dist.DeviceSlabEngine(ctx, r, world)
    e.set_slab(buf, wlo, lo, hi, whi, size, rows, cap)
    engs.append(e)
fmt = L.FMT_FASTQ
for e in engs:
    g = e.guess(fmt)
    res = e.index(fmt, g, 16)
    n = max(0, e.local_count - e.row_base)
    t = e.rows.rows(min(n, e.row_cap))
    bad = np.nonzero(t[:-1, 0] + t[:-1, 1] != t[1:, 0])[0] if len(t) > 1 else []
    lo = e.slab.base
    print(f"slab {e.rank} lo {lo} guess {g} count {e.local_count} flags {e.local_flags} term {res.term_code} "
          f"fixups {res.fixups} fix_tiles {res.fix_tiles} noncontig {len(bad)}")
    for i in list(bad)[:5]:
        print("   at", i, t[max(0, i - 1):i + 3].tolist())
    # the true rows of this slab's records (oracle), first few
    k = np.searchsorted(exp[:, 0], lo)
    print("   oracle first rows from slab start:", exp[k:k + 3].tolist(), "gpu first rows:", t[:3].tolist())
