"""Validate the device synthetic generator: offsets = prefix sums of lengths, and the oracle
indexes the materialised bytes to exactly the generator's table.  Development tool."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle
from shock_amd import Context
from shock_amd.synth import SynthFile
ctx = Context(0)
for fmt, size in (("fastq", 64 << 20), ("fastq", 1 << 30), ("fasta", 256 << 20)):
    sf = SynthFile(ctx, fmt, size)
    ln = sf.d_len.download(4 * sf.n_est).view(np.uint32).astype(np.uint64)
    off = sf.d_off.download(8 * (sf.n_est + 1)).view(np.uint64)
    ok_off = off[0] == 0 and np.array_equal(np.diff(off), ln)
    host = sf.window(0, size).download(size)
    t = time.time()
    rows, err = oracle.record_index(host, fmt)
    exp = np.stack([off[:sf.nrec], ln[:sf.nrec]], axis=1)
    if fmt == "fasta" and sf.nrec:
        exp[-1, 1] = size - exp[-1, 0]
    print(fmt, size, "n_est", sf.n_est, "nrec", sf.nrec, "offsets_ok", ok_off, "oracle", len(rows), err,
          "rows_match", len(rows) == sf.nrec and np.array_equal(rows, exp), f"{time.time()-t:.2f}s",
          "tail", bytes(host[-8:]))
