"""Probe (round 5): FASTQ host builds in fresh contexts of several library builds, checked
against the C oracle -- which layout of the tile pass's start arrays breaks
tests/test_gpu_parity.py::test_workspace_trim_gpu ("device invariant violated").

  python tools/probes/fq_layout_probe.py base il0 pk0

Prints one line per (variant, seed, repeat): status, count, expected count, first differing row.
Run with SHOCKIDX_VERIFY unset to see the table a violation would have returned.
"""
import ctypes
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import gen  # noqa: E402
import oracle  # noqa: E402
from shock_amd import _lib as L  # noqa: E402


def load(v):
    path = os.path.join(ROOT, "shock_amd", "libshockidx.so") if v == "base" else \
        os.path.join(ROOT, "shock_amd", "variants", f"libshockidx_{v}.so")
    lib = ctypes.CDLL(path)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    lib.shockidx_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.shockidx_ctx_destroy.argtypes = [vp]
    lib.shockidx_build_host.argtypes = [vp, vp, u64, i32, i32, ctypes.POINTER(ctypes.POINTER(u64)), ctypes.POINTER(L.Result)]
    lib.shockidx_free.argtypes = [vp]
    return lib


def main():
    variants = sys.argv[1:] or ["base"]
    libs = {v: load(v) for v in variants}
    for seed, n in ((4, 20000), (5, 3000), (6, 60000)):
        data = gen.fastq(random.Random(seed), n)
        exp, _ = oracle.record_index(data, "fastq")
        buf = ctypes.create_string_buffer(data, len(data))
        for v, lib in libs.items():
            for rep in range(2):
                h = ctypes.c_void_p()
                assert lib.shockidx_ctx_create(0, ctypes.byref(h)) == 0
                rows_p = ctypes.POINTER(ctypes.c_uint64)()
                res = L.Result()
                rc = lib.shockidx_build_host(h, buf, len(data), 0, -1, ctypes.byref(rows_p), ctypes.byref(res))
                got = np.ctypeslib.as_array(rows_p, shape=(res.count * 2,)).reshape(-1, 2).copy() if rows_p and res.count else np.zeros((0, 2), np.uint64)
                first = None
                m = min(len(got), len(exp))
                d = np.nonzero(np.any(got[:m] != exp[:m], axis=1))[0]
                if len(d):
                    i = int(d[0])
                    first = (i, got[i].tolist(), exp[i].tolist())
                print(f"{v} seed={seed} rep={rep} rc={rc} count={res.count} exp={len(exp)} bytes={len(data)} "
                      f"ndiff={len(d)} first={first} flags={res.flags} term={res.term_code} fixups={res.fixups} "
                      f"fix_tiles={res.fix_tiles} path={res.path} err={bytes(res.err)[:res.err_len]!r}", flush=True)
                if rows_p:
                    lib.shockidx_free(rows_p)
                lib.shockidx_ctx_destroy(h)


if __name__ == "__main__":
    main()
