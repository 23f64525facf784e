"""Probe (round 5): is the slow FASTQ tile pass on the synthetic file's own buffer a property of
the physical memory it got, or of that allocation?

One process, one context.  A = the synthetic 10 GiB node body (the process's first large node
allocation), B = a second node allocation holding the same bytes.  Then A is freed and C allocated
(the allocator likely hands A's memory back), and D = another fresh context over C (its own stage
workspace, allocated after C).  Prints the median k_fq_tiles time (index_ms) per buffer and step:
if C is as slow as A, the memory range is what matters; if C is fast, the allocation's history.
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


def med(ctx, buf, size, rows, cap, n=40, warm=10):
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
    out = {"A_first": med(ctx, A, size, rows, cap)}
    B = ctx.alloc(size + 64, node=True)
    assert hip.hipMemcpy(ctypes.c_void_p(B.ptr), ctypes.c_void_p(A.ptr), size + 64, 3) == 0
    out["B_second"] = med(ctx, B, size, rows, cap)
    out["A_again"] = med(ctx, A, size, rows, cap)
    va_a = A.ptr
    A.free()
    C = ctx.alloc(size + 64, node=True)
    assert hip.hipMemcpy(ctypes.c_void_p(C.ptr), ctypes.c_void_p(B.ptr), size + 64, 3) == 0
    out["C_after_free_A"] = med(ctx, C, size, rows, cap)
    out["C_same_va_as_A"] = C.ptr == va_a
    ctx2 = Context(0)
    rows2 = ctx2.alloc(16 * cap)
    out["C_new_context"] = med(ctx2, C, size, rows2, cap)
    out["B_new_context"] = med(ctx2, B, size, rows2, cap)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
