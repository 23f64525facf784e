"""Probe (round 6): is the slow FASTQ tile pass on the bench's input a property of the buffer's
physical placement, or of HOW its bytes were written?

Round 5 (profiles/r05/calls/r05t/placement_realloc.json): the synthetic node body A (filled by
libshocksynth's kernel, byte stores) ran k_fq_tiles in 2.08 ms; a copy B (hipMemcpy D2D) 1.85; A
freed and reallocated at the same virtual address, refilled by D2D copy, 1.86.  Here, in one
process, the same bytes written several ways, each measured (median index_ms over n builds):
  A_kernel        the generator's buffer (kernel byte stores), as bench.py uses it
  B_d2d           a second node allocation, filled by hipMemcpy D2D from A
  A_rewritten_d2d A again after hipMemcpy D2D B -> A (same memory, rewritten by the copy engine)
  C_h2d           a third allocation filled by hipMemcpy H2D from a host copy (how a node arrives)
  A_rewritten_h2d A again after H2D from the host copy
  E_kernel        a fourth allocation filled by the generator's kernel (is "kernel-written" slow,
                  or only "first"?)
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from shock_amd.core import Context  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402


def med(ctx, buf, size, rows, cap, n=12, warm=4):
    for _ in range(warm):
        ctx.build_device(buf.ptr, size, rows.ptr, cap)
    ks = []
    for _ in range(n):
        r = ctx.build_device(buf.ptr, size, rows.ptr, cap)
        assert r.ok
        ks.append(r.timings["index_ms"])
    return round(float(np.median(ks)), 4)


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    size = 10 << 30
    ctx = Context(0)
    sf = SynthFile(ctx, "fastq", size)
    A = sf.window(0, size)
    R = sf.expected_count()
    cap = R + 1024
    rows = ctx.alloc(16 * cap)
    out = {"A_kernel": med(ctx, A, size, rows, cap)}
    print(json.dumps(out), file=sys.stderr, flush=True)
    B = ctx.alloc(size + 64, node=True)
    assert hip.hipMemcpy(ctypes.c_void_p(B.ptr), ctypes.c_void_p(A.ptr), size + 64, 3) == 0
    out["B_d2d"] = med(ctx, B, size, rows, cap)
    assert hip.hipMemcpy(ctypes.c_void_p(A.ptr), ctypes.c_void_p(B.ptr), size + 64, 3) == 0
    out["A_rewritten_d2d"] = med(ctx, A, size, rows, cap)
    print(json.dumps(out), file=sys.stderr, flush=True)
    host = A.download(size + 64)
    C = ctx.alloc(size + 64, node=True)
    C.upload(host)
    out["C_h2d"] = med(ctx, C, size, rows, cap)
    A.upload(host)
    out["A_rewritten_h2d"] = med(ctx, A, size, rows, cap)
    print(json.dumps(out), file=sys.stderr, flush=True)
    del host
    E = sf.window(0, size)
    out["E_kernel"] = med(ctx, E, size, rows, cap)
    out["A_last"] = med(ctx, A, size, rows, cap)
    out["B_last"] = med(ctx, B, size, rows, cap)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
