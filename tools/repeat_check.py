"""Repeat a device-resident build and report any nondeterminism with diagnostics.  Dev tool."""
import os, sys, collections
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context
from shock_amd.synth import SynthFile
ctx = Context(0)
fmt = sys.argv[1] if len(sys.argv) > 1 else "fastq"
size = int(float(sys.argv[2]) * (1 << 30)) if len(sys.argv) > 2 else 1 << 30
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
mode = sys.argv[4] if len(sys.argv) > 4 else "auto"
sf = SynthFile(ctx, fmt, size)
data = sf.window(0, size)
R = sf.expected_count()
rows = ctx.alloc(16 * (R + 1024))
hist = collections.Counter()
bad = 0
for i in range(reps):
    rows.fill(0)
    r = ctx.build_buffer(data, size, rows, kind="record", fmt=None if mode == "auto" else fmt)
    hist[(r.count, r.status, r.err, r.term_code)] += 1
    if r.count != R or not r.ok:
        bad += 1
        if bad <= 2:
            got = rows.rows(R + 8)
            exp_off = sf.d_off.download(8 * (R + 1)).view(np.uint64)
            exp_len = sf.d_len.download(4 * R).view(np.uint32)
            mis = np.nonzero((got[:R, 0] != exp_off[:R]) | (got[:R, 1] != exp_len))[0]
            print("bad run", i, "count", r.count, "R", R, "status", r.status, r.err, "term", r.term_code,
                  "flags", r.flags, "state_out", r.state_out, "selfhelp", r.selfhelp,
                  "mismatch rows", len(mis), mis[:5].tolist(), "rows R..R+8", got[R - 2:R + 6].tolist())
print(mode, "expected", R, "hist", dict(hist))
