"""SAM build timing on the device: the tile pass vs the two-pass build (SHOCKIDX_SAM_MODE=two)
over a SAM body resident in HBM (a generated block repeated to --mib MiB), rows compared.
Prints one JSON line.  Dev tool; the GPU tests carry the parity cases."""
import argparse
import json
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gen  # noqa: E402
from shock_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    block = np.frombuffer(gen.sam(random.Random(1), 40000, headers=0, blank=0.0), np.uint8)
    reps = (a.mib << 20) // block.size
    body = np.tile(block, reps)
    n = body.size
    ctx = Context(0)
    data = ctx.alloc(n + 64, node=True)
    data.upload(body)
    rows = ctx.alloc(16 * (n // 40 + 4096))
    out = {"metric": "device-resident SAM record index build", "bytes": n, "unit": "GiB/s"}
    tabs = {}
    for mode in ("tiles", "two"):
        if mode == "two":
            os.environ["SHOCKIDX_SAM_MODE"] = "two"
        for _ in range(3):
            r = ctx.build_buffer(data, n, rows, kind="record", fmt="sam")
        ks, bs = [], []
        for _ in range(a.steps):
            r = ctx.build_buffer(data, n, rows, kind="record", fmt="sam")
            ks.append(r.timings["index_ms"])
            bs.append(r.timings["kernel_ms"])
        tabs[mode] = rows.rows(r.count).copy()
        out[mode] = {"path": r.path, "rows": r.count, "index_kernel_ms": round(float(np.mean(ks)), 4),
                     "build_ms": round(float(np.mean(bs)), 4),
                     "build_gib_s": round(n / (float(np.mean(bs)) * 1e-3) / (1 << 30), 1)}
    os.environ.pop("SHOCKIDX_SAM_MODE", None)
    out["identical"] = bool(np.array_equal(tabs["tiles"], tabs["two"]))
    print(json.dumps(out))
    return 0 if out["identical"] else 1


if __name__ == "__main__":
    sys.exit(main())
