"""Probe (round 5): does the way a node body was written decide the FASTQ tile pass's speed?

placement_realloc.py found the synthetic file's own buffer slow (2.08 ms) and every later
allocation of the same bytes fast (1.85 ms), including a new allocation at the same virtual
address after the first was freed.  The synthetic buffer is written by compute kernels
(synth_fill: byte-granular record writes); the copies by hipMemcpy.  Here, in one process:
  A  the synthetic window (kernel-written)
  B  a second synthetic window (kernel-written, allocated later)
  C  a node allocation filled from A by hipMemcpy (device to device)
  A2 A overwritten in place from C by hipMemcpy (same memory, rewritten by the copy engine)
  B2 B overwritten in place from C by a kernel copy (hipMemcpy D2D of the same bytes through a
     kernel is not selectable, so: shockidx_memset to 0 then hipMemcpy -- a second copy-engine
     write; reported for symmetry)
Prints the median k_fq_tiles time per step.
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


def med(ctx, buf, size, rows, cap, n=30, warm=10):
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
    out = {"A_synth_first": med(ctx, A, size, rows, cap)}
    B = sf.window(0, size)
    out["B_synth_second"] = med(ctx, B, size, rows, cap)
    C = ctx.alloc(size + 64, node=True)
    assert hip.hipMemcpy(ctypes.c_void_p(C.ptr), ctypes.c_void_p(A.ptr), size + 64, 3) == 0
    out["C_memcpy_copy"] = med(ctx, C, size, rows, cap)
    assert hip.hipMemcpy(ctypes.c_void_p(A.ptr), ctypes.c_void_p(C.ptr), size + 64, 3) == 0
    out["A2_A_rewritten_by_memcpy"] = med(ctx, A, size, rows, cap)
    B.fill(0)
    assert hip.hipMemcpy(ctypes.c_void_p(B.ptr), ctypes.c_void_p(C.ptr), size + 64, 3) == 0
    out["B2_B_zeroed_then_memcpy"] = med(ctx, B, size, rows, cap)
    out["A_after_all"] = med(ctx, A, size, rows, cap)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
