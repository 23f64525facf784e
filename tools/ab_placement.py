"""Probe (round 5): does the input's physical placement set the FASTQ build's speed?

The same binary runs k_fq_tiles at 1.92 ms in one process and 2.09 ms in the next
(gpurun_out/r05e: stable within a process, every variant shifted alike), so the state lives in
something each process allocates anew.  Here one process holds several copies of the same 10 GiB
synthetic node file -- some from hipExtMallocWithFlags(hipDeviceMallocContiguous), some from
plain hipMalloc -- and builds over them in turns (one context, the same workspaces).  Prints one
JSON line: per copy its allocator, whether the contiguous request succeeded, and the median
k_fq_tiles / whole-build times.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shock_amd.core import Context  # noqa: E402
from shock_amd.synth import SynthFile, slib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", default="contig,plain,contig,plain")
    ap.add_argument("--size-gib", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--per", type=int, default=10)
    a = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    ctx = Context(0)
    size = int(a.size_gib * (1 << 30))
    sf = SynthFile(ctx, "fastq", size)
    src = sf.window(0, size)
    R = sf.expected_count()
    rows = ctx.alloc(16 * (R + 1024))
    bufs = []
    for kind in a.copies.split(","):
        p = ctypes.c_void_p()
        ok = False
        if kind == "contig":
            ok = hip.hipExtMallocWithFlags(ctypes.byref(p), size + 64, 4) == 0  # hipDeviceMallocContiguous (0x4)
        if not ok:
            assert hip.hipMalloc(ctypes.byref(p), size + 64) == 0
        assert hip.hipMemcpy(p, ctypes.c_void_p(src.ptr), size + 64, 3) == 0  # device to device
        bufs.append({"alloc": kind, "contiguous": ok, "ptr": p.value, "k": [], "b": []})
    bufs.insert(0, {"alloc": "window(node=True)", "contiguous": None, "ptr": src.ptr, "k": [], "b": []})
    for b in bufs:
        for _ in range(20):
            ctx.build_device(b["ptr"], size, rows.ptr, R + 1024)
    for r in range(a.rounds):
        for b in (bufs if r % 2 == 0 else bufs[::-1]):
            for _ in range(a.per):
                res = ctx.build_device(b["ptr"], size, rows.ptr, R + 1024)
                assert res.ok and res.count == R
                b["k"].append(res.timings["index_ms"])
                b["b"].append(res.timings["kernel_ms"])
    S = slib()
    S.synth_page_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p]
    sink = ctx.alloc(64)
    for b in bufs:
        ms = ctypes.c_float(0.0)
        assert S.synth_stream_floor(b["ptr"], size, 10, sink.ptr, ctypes.byref(ms), ctx.stream) == 0
        b["floor"] = round(ms.value, 4)
        for st in (4096, 65536, 2 << 20):
            assert S.synth_page_probe(b["ptr"], size, st, 5, sink.ptr, ctypes.byref(ms), ctx.stream) == 0
            b[f"page_{st}"] = round(ms.value, 4)
    out = [{"alloc": b["alloc"], "contiguous": b["contiguous"], "va": hex(b["ptr"]),
            "k_med": round(float(np.median(b["k"])), 4), "b_med": round(float(np.median(b["b"])), 4),
            "floor": b["floor"], "page_4k": b["page_4096"], "page_64k": b["page_65536"], "page_2m": b[f"page_{2 << 20}"]}
           for b in bufs]
    print(json.dumps({"bytes": size, "copies": out}))


if __name__ == "__main__":
    main()
