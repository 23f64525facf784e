"""Per-input-copy counters of k_fq_tiles (the slow input copy).

One process: the configs[1] FASTQ node (copy 0, the synthetic generator's window) and --copies - 1
more allocations of the same bytes; after --warmup builds on copy 0, --per builds on each copy in
order (copy 0 first).  Prints one JSON line with each timed build's copy and index_ms.  Run under
`rocprofv3 --pmc ...`: the k_fq_tiles dispatches after the warm-up are then the timed builds in
that order, and `--summarize <pmc dir> <this run's json>` folds the counters per copy.

  rocprofv3 --pmc TCC_EA0_WRREQ_sum -d out -o pmc --output-format csv -- python3 tools/probes/copy_pmc.py > run.json
  python tools/probes/copy_pmc.py --summarize out run.json
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def summarize(d, run_json):
    run = json.load(open(run_json))
    per = {}  # dispatch -> {counter: value}
    names = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p, newline="")):
            if "k_fq_tiles" not in r.get("Kernel_Name", ""):
                continue
            k = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per.setdefault(k, {})
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[r["Counter_Name"]] = 1
    ids = sorted(per)
    timed = ids[-len(run["builds"]):]
    out = {}
    for (copy, ms), k in zip(run["builds"], timed):
        o = out.setdefault(str(copy), {"ms": [], **{n: [] for n in names}})
        o["ms"].append(ms)
        for n in names:
            o[n].append(per[k].get(n, 0.0))
    res = {c: {n: round(float(np.median(v)), 1) for n, v in o.items()} for c, o in out.items()}
    print(json.dumps({"dispatches": len(ids), "timed": len(timed), "per_copy_median": res}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--per", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-gib", type=float, default=10.0)
    ap.add_argument("--summarize", nargs=2, metavar=("PMC_DIR", "RUN_JSON"))
    a = ap.parse_args()
    if a.summarize:
        return summarize(*a.summarize)
    from shock_amd.core import Context
    from shock_amd.synth import SynthFile
    ctx = Context(0)
    size = int(a.size_gib * (1 << 30))
    sf = SynthFile(ctx, "fastq", size)
    data = sf.window(0, size)
    R = sf.expected_count()
    inputs = [data] + [ctx.alloc(size + 64, node=True) for _ in range(a.copies - 1)]
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    for b in inputs[1:]:
        assert hip.hipMemcpy(ctypes.c_void_p(b.ptr), ctypes.c_void_p(data.ptr), size + 64, 3) == 0
    rows = ctx.alloc(16 * (R + 1024))
    for _ in range(a.warmup):
        r = ctx.build_buffer(inputs[0], size, rows, kind="record", fmt="fastq")
    builds = []
    for c in range(a.copies):
        for _ in range(a.per):
            r = ctx.build_buffer(inputs[c], size, rows, kind="record", fmt="fastq")
            assert r.ok and r.count == R
            builds.append((c, round(r.timings["index_ms"], 4)))
        print(f"copy {c} done", file=sys.stderr, flush=True)
    print(json.dumps({"builds": builds}))


if __name__ == "__main__":
    main()
