"""Repeats test_gpu_multi.py::test_multi_resident_slabs (FASTA, 4 slabs on device 0) in one
process and reports every run whose count or rows differ from the oracle, with the per-slab
first / owned numbers.  Diagnostic for an intermittent count mismatch."""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import gen  # noqa: E402
from shock_amd import Context, MultiContext  # noqa: E402
import oracle as orc  # noqa: E402  (test infrastructure: the checker)

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
data = gen.fasta(random.Random(13), 4000)
rows, err = orc.record_index(data, "fasta")
ctx = Context(0)
bad = 0
for rep in range(REPS):
    m = MultiContext([0, 0, 0, 0])
    plan = m.plan(len(data))
    wins, outs, caps = [], [], []
    for lo, hi, wlo, whi in plan:
        w = ctx.alloc(whi - wlo + 64)
        w.upload(np.frombuffer(data[wlo:whi], np.uint8))
        cap = (hi - lo) // 8 + 64
        wins.append(w)
        outs.append(ctx.alloc(16 * cap))
        caps.append(cap)
    r, first, owned = m.build_resident(len(data), [w.ptr for w in wins], [o.ptr for o in outs], caps, fmt="fasta")
    table = np.concatenate([o.rows(k) if k else np.zeros((0, 2), np.uint64) for o, k in zip(outs, owned)])
    ok = r.ok and r.count == len(rows) and table.shape == rows.shape and np.array_equal(table, rows)
    if not ok:
        bad += 1
        print(f"rep {rep}: count {r.count} want {len(rows)} first {first} owned {owned} plan {plan} "
              f"path {r.path} err {r.err}", flush=True)
    for b in wins + outs:
        b.free()
    m.close()
print(f"{bad} of {REPS} runs differ", flush=True)
