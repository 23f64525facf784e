"""Hunt for the input on which the round-5 ID-compare experiment built a wrong table
(profiles/r05/calls/pytest_gpu_idc_failure.txt: test_generated_gpu[fastq_plain] ->
EINTERNAL "device invariant violated"; the seed was a salted hash() and is lost).

For each seed, the fastq_plain corpus of tests/test_gpu_parity.py (gen.fastq(r, 30000,
plus_id=0.1)) is indexed at many tile alignments -- the first j records cut off -- through the
loaded library (SHOCKIDX_VARIANT=idc for the experiment) and compared with the oracle.  Every
failing (seed, j) is printed as one JSON line; the first few inputs are kept gzip'd under --out,
with the table the build returns when SHOCKIDX_VERIFY is off, diffed against
the oracle's so the first wrong row -- and its tile -- is named.

  SHOCKIDX_VARIANT=idc python tools/probes/idc_hunt.py --seeds 1 2 3 --cuts 64
"""
import argparse
import gzip
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import gen  # noqa: E402
import oracle  # noqa: E402
from shock_amd.core import Context  # noqa: E402
from shock_amd import _lib as L  # noqa: E402

TILE = 16384


def check(ctx, data):
    exp, err = oracle.record_index(data, "fastq")
    os.environ["SHOCKIDX_VERIFY"] = "1"  # (read by every build: sidx_capi.cpp verify_rows)
    try:
        r = ctx.build_host(data, kind="record", fmt="fastq")
    except L.ShockIdxError as e:
        return f"raise {e}", exp
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    if r.err != err or got.shape != exp.shape or not np.array_equal(got, exp):
        return f"mismatch count {r.count} vs {len(exp)} err {r.err!r} vs {err!r}", exp
    return None, exp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--cuts", type=int, default=64)
    ap.add_argument("--nrec", type=int, default=30000)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "idc"))
    ap.add_argument("--keep", type=int, default=3)
    ap.add_argument("--data", nargs="*", default=[], help="re-check saved inputs (.bin.gz) instead of generating")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    ctx = Context(0)
    kept = 0
    nfail = ntry = 0

    def one(tag, data):
        nonlocal kept, nfail, ntry
        ntry += 1
        why, exp = check(ctx, data)
        if why is None:
            return
        nfail += 1
        rec = {"case": tag, "bytes": len(data), "why": why}
        os.environ["SHOCKIDX_VERIFY"] = "0"
        try:
            r = ctx.build_host(data, kind="record", fmt="fastq")
            got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
            n = min(len(got), len(exp))
            bad = np.nonzero((got[:n] != exp[:n]).any(axis=1))[0]
            i = int(bad[0]) if len(bad) else n
            rec["noverify"] = {"count": int(r.count), "first_bad_row": i,
                               "gpu": got[i:i + 2].tolist(), "oracle": exp[i:i + 2].tolist(),
                               "tile": int(exp[i][0]) // TILE if i < len(exp) else None}
        except L.ShockIdxError as e:
            rec["noverify"] = f"raise {e}"
        if kept < a.keep:
            p = os.path.join(a.out, f"fail_{tag}.bin.gz")
            with gzip.open(p, "wb", compresslevel=3) as f:
                f.write(data)
            rec["saved"] = p
            kept += 1
        print(json.dumps(rec), flush=True)

    if a.data:
        for p in a.data:
            with gzip.open(p, "rb") as f:
                one(os.path.basename(p), f.read())
    for seed in ([] if a.data else a.seeds):
        data = gen.fastq(random.Random(seed), a.nrec, plus_id=0.1)
        starts = [0]
        for j in range(a.cuts):  # record starts: every 4th '\n'
            p = starts[-1]
            for _ in range(4):
                p = data.index(b"\n", p) + 1
            starts.append(p)
        for j in range(a.cuts):
            one(f"s{seed}_c{j}", data[starts[j]:])
        print(json.dumps({"seed": seed, "tried": ntry, "failed": nfail}), file=sys.stderr, flush=True)
    print(json.dumps({"tried": ntry, "failed": nfail}), flush=True)


if __name__ == "__main__":
    main()
