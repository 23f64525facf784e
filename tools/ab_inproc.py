"""Paired A/B of libshockidx builds inside ONE process (round 5).

Separate bench processes of the same binary differ by up to 13 % (profiles/r05/ab_*: k_fq_tiles
1.84 vs 2.09 ms, consecutive runs), so variants are compared here on the same input buffer,
the same physical placement and the same device state: every variant library
(shock_amd/variants/libshockidx_<V>.so, or "base" = shock_amd/libshockidx.so) is loaded side by
side (ctypes loads each with RTLD_LOCAL: separate symbols, one HIP runtime), each gets its own
context, and the variants take turns, `--per` builds each, for `--rounds` rounds.  Prints one
JSON line: per variant the median / mean k_fq_tiles time (index_ms) and whole-build time
(kernel_ms) over all its builds, and whether every build's count matched.

  python tools/ab_inproc.py base ring0 lean0 --rounds 6 --per 10
"""
import argparse
import ctypes
import json
import os
import sys

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
    lib.shockidx_build_device.argtypes = [vp, vp, u64, i32, i32, vp, u64, vp, ctypes.POINTER(L.Result)]
    lib.shockidx_dev_alloc.argtypes = [vp, u64, ctypes.POINTER(vp)]
    lib.shockidx_sync.argtypes = [vp]
    h = vp()
    assert lib.shockidx_ctx_create(0, ctypes.byref(h)) == 0
    return lib, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--fmt", default="fastq")
    ap.add_argument("--kind", default="record", choices=("record", "line"))
    ap.add_argument("--size-gib", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--turn-warmup", type=int, default=0,
                    help="untimed builds at the start of every turn (a variant right after another can run slow "
                         "for several builds, profiles/r05/calls/r05r)")
    ap.add_argument("--copies", type=int, default=1,
                    help="inputs: the file in this many separately allocated buffers (the same bytes; the "
                         "build's speed depends on the input's placement, gpurun_out/r05f), every variant on each")
    ap.add_argument("--check-rows", action="store_true",
                    help="hash every variant's whole table (one extra build each, copy 0) and report agreement")
    a = ap.parse_args()
    ctx = Context(0)  # the input and the synthetic generator (shock_amd/libshockidx.so)
    size = int(a.size_gib * (1 << 30))
    sf = SynthFile(ctx, a.fmt, size)
    data = sf.window(0, size)
    R = sf.expected_count()
    inputs = [data] + [ctx.alloc(size + 64, node=True) for _ in range(a.copies - 1)]
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    for b in inputs[1:]:
        assert hip.hipMemcpy(ctypes.c_void_p(b.ptr), ctypes.c_void_p(data.ptr), size + 64, 3) == 0
    kind = 1 if a.kind == "line" else 0
    fmt = -1
    cap = (size // 8 if kind else R) + 1024
    libs = {}
    for v in a.variants:
        lib, h = load(v)
        rows = ctypes.c_void_p()
        assert lib.shockidx_dev_alloc(h, 16 * cap, ctypes.byref(rows)) == 0
        libs[v] = (lib, h, rows)
    res = L.Result()
    keys = [(v, c) for c in range(a.copies) for v in a.variants]
    out = {k: {"k": [], "b": [], "count_ok": True} for k in keys}

    def run(key, n, keep):
        v, c = key
        lib, h, rows = libs[v]
        for _ in range(n):
            rc = lib.shockidx_build_device(h, inputs[c].ptr, size, kind, fmt, rows, cap, None, ctypes.byref(res))
            if keep:
                out[key]["k"].append(res.index_ms)
                out[key]["b"].append(res.kernel_ms)
                out[key]["count_ok"] &= (rc == 0 and (kind == 1 or res.count == R))

    for key in keys:
        run(key, a.warmup, False)
    for r in range(a.rounds):
        for key in (keys if r % 2 == 0 else keys[::-1]):
            run(key, a.turn_warmup, False)
            run(key, a.per, True)
        print(f"round {r + 1}/{a.rounds} done", file=sys.stderr, flush=True)  # (progress: gpurun's hang watch)
    digests = {}
    if a.check_rows:  # one more build per variant on copy 0, its whole table hashed on the host
        import hashlib
        for v in a.variants:
            lib, h, rows = libs[v]
            rc = lib.shockidx_build_device(h, inputs[0].ptr, size, kind, fmt, rows, cap, None, ctypes.byref(res))
            nb = 16 * int(res.count)
            buf = (ctypes.c_uint8 * nb)()
            assert rc == 0 and hip.hipMemcpy(ctypes.cast(buf, ctypes.c_void_p), rows, nb, 2) == 0
            digests[v] = hashlib.sha256(memoryview(buf)).hexdigest()[:16]
    summ = {}
    for (v, c) in keys:
        o = out[(v, c)]
        summ[f"{v}@{c}" if a.copies > 1 else v] = {
            "k_med": round(float(np.median(o["k"])), 4), "k_mean": round(float(np.mean(o["k"])), 4),
            "k_rounds": [round(float(np.median(o["k"][i:i + a.per])), 3) for i in range(0, len(o["k"]), a.per)],
            "b_med": round(float(np.median(o["b"])), 4), "b_mean": round(float(np.mean(o["b"])), 4),
            "n": len(o["k"]), "count_ok": bool(o["count_ok"])}
    print(json.dumps({"fmt": a.fmt, "kind": a.kind, "bytes": size, "rounds": a.rounds, "per": a.per, "ab": summ,
                      "rows_sha256_16": digests, "rows_agree": len(set(digests.values())) <= 1}))


if __name__ == "__main__":
    main()
