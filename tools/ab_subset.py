"""Paired A/B of the whole subset node (BASELINE configs[3]) inside ONE process (round 5).

The record index of a device-resident synthetic FASTQ node (50 GiB by default) and a subset of a
sorted random 1 % of its records are built once with shock_amd/libshockidx.so (as bench.py
--subset does); then every variant library (shock_amd/variants/libshockidx_<V>.so, or "base")
builds the subset node (shockidx_subset_node: the subset index and the gather in one call) from
the same ids over the same parent table and input, in turns.  Prints one JSON line: per variant
the median wall time of the call, its index-kernel and gather-kernel times, and whether its
output equals the first variant's byte for byte.

  python tools/ab_subset.py base sc0 --rounds 6 --per 10
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shock_amd import _lib as L  # noqa: E402
from shock_amd.core import Context  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402


def load(v):
    path = os.path.join(ROOT, "shock_amd", "libshockidx.so") if v == "base" else \
        os.path.join(ROOT, "shock_amd", "variants", f"libshockidx_{v}.so")
    lib = ctypes.CDLL(path)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    lib.shockidx_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.shockidx_subset_node.argtypes = [vp, vp, u64, vp, u64, ctypes.c_int64, vp, u64, vp, u64, vp, u64, vp, u64,
                                         ctypes.POINTER(L.SubsetResult)]
    h = vp()
    assert lib.shockidx_ctx_create(0, ctypes.byref(h)) == 0
    return lib, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--size-gib", type=float, default=50.0)
    ap.add_argument("--frac", type=float, default=0.01)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    ctx = Context(0)
    size = int(a.size_gib * (1 << 30))
    sf = SynthFile(ctx, "fastq", size)
    data = sf.window(0, size)
    R = sf.expected_count()
    rows = ctx.alloc(16 * (R + 1024))
    r = ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
    assert r.ok and r.count == R
    rng = np.random.default_rng(0x5EED)
    k = max(1, int(R * a.frac))
    ids = np.sort(rng.choice(R, size=k, replace=False) + 1)
    text = ("\n".join(map(str, ids.tolist())) + "\n").encode()
    d_ids = ctx.alloc(len(text) + 64)
    d_ids.upload(text)
    cap = k + 16
    res = ctx.subset_index(d_ids.ptr, len(text), rows.ptr, R, R, ctx.alloc(16 * cap).ptr, cap, ctx.alloc(16 * cap).ptr, cap)
    assert res.ok
    libs, outs = {}, {}
    for v in a.variants:
        libs[v] = load(v)
        outs[v] = (ctx.alloc(16 * cap), ctx.alloc(16 * cap), ctx.alloc(res.size + 64))
    sr = L.SubsetResult()
    times = {v: {"w": [], "k": [], "g": []} for v in a.variants}

    def run(v, n, keep):
        lib, h = libs[v]
        d_sub, d_runs, d_out = outs[v]
        for _ in range(n):
            t0 = time.perf_counter()
            rc = lib.shockidx_subset_node(h, d_ids.ptr, len(text), rows.ptr, R, R, d_sub.ptr, cap, d_runs.ptr, cap,
                                          data.ptr, size, d_out.ptr, res.size + 64, ctypes.byref(sr))
            t1 = time.perf_counter()
            assert rc == 0 and sr.size == res.size and sr.count == k, (v, rc, sr.count)
            if keep:
                times[v]["w"].append((t1 - t0) * 1e3)
                times[v]["k"].append(sr.kernel_ms)
                times[v]["g"].append(sr.gather_ms)

    for v in a.variants:
        run(v, a.warmup, False)
    for rd in range(a.rounds):
        for v in (a.variants if rd % 2 == 0 else a.variants[::-1]):
            run(v, a.per, True)
        print(f"round {rd + 1}/{a.rounds} done", file=sys.stderr, flush=True)
    digest = {v: hashlib.sha256(outs[v][2].download(res.size).tobytes()).hexdigest() for v in a.variants}
    summ = {v: {"node_ms_med": round(float(np.median(t["w"])), 4), "index_kernel_ms_med": round(float(np.median(t["k"])), 4),
                "gather_kernel_ms_med": round(float(np.median(t["g"])), 4), "n": len(t["w"]),
                "gib_s": round(res.size / (float(np.median(t["w"])) * 1e-3) / (1 << 30), 1),
                "same_bytes": digest[v] == digest[a.variants[0]]} for v, t in times.items()}
    print(json.dumps({"bytes": size, "ids": k, "runs": res.runs, "subset_bytes": res.size, "ab": summ}))


if __name__ == "__main__":
    main()
