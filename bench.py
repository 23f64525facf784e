"""bench.py -- device-resident record-index build throughput (BASELINE.json metric).

Workload (N=1): BASELINE.json configs[1] -- a 10 GiB synthetic FASTQ node file resident in
HBM, record index built by libshockidx exactly as Shock's
index/record.go would (auto-detected format, full validation, offset table left in HBM).
A "step" is one complete build: detect + index kernel + finalize.  N>1: the file is
N x 10 GiB, one slab per GPU (weak scaling), with one RCCL all-gather of slab summaries.

Prints one JSON line (rank 0).  --check verifies every row against the generator.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = 1 << 30
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "device-resident index-build GiB/s + Mrecords/s, 10 GiB FASTQ, 1/2/4/8 GPU"  # BASELINE.json
TILE = 16384  # bytes per workgroup tile (sidx_common.hpp SIDX_TILE)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--fmt", default="fastq", choices=("fastq", "fasta"))
    ap.add_argument("--size-gib", type=float, default=10.0)
    ap.add_argument("--cpu-sec", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--cpu-sample-gib", type=float, default=1.0)
    ap.add_argument("--check", action="store_true", default=True)
    ap.add_argument("--no-check", dest="check", action="store_false")
    ap.add_argument("--pmc", default=None, help="rocprofv3 PMC summary (default profiles/pmc_<fmt>.json)")
    ap.add_argument("--e2e", action="store_true",
                    help="host-memory build (POSTed body): pinned H2D staging + kernel + table D2H")
    return ap.parse_args()


def cpu_baseline(sample: np.ndarray, fmt: str, budget_s: float):
    """Oracle (C restatement of the Go path, single thread) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    oracle.build()
    reps, t_total, nrec = 0, 0.0, 0
    while t_total < budget_s or reps == 0:
        t0 = time.perf_counter()
        rows, err = oracle.record_index(sample, fmt)
        t_total += time.perf_counter() - t0
        reps += 1
        nrec = len(rows)
    gibs = reps * sample.size / t_total / GIB
    return {"value": round(gibs, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "mrec_per_s": round(reps * nrec / t_total / 1e6, 3),
            "sample": f"first {sample.size / GIB:.2f} GiB of the same synthetic {fmt} file, "
                      f"{reps} passes in {t_total:.1f} s, oracle/shockidx_oracle.c (C restatement of "
                      f"index/record.go + format/{fmt}), 1 thread"}


def load_pmc(path, cfg):
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if d.get("config") != cfg:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        a.gpus = world
    if world > 1:
        from shock_amd import dist
        return dist.bench_main(a, rank, world, local)

    from shock_amd import Context
    from shock_amd.synth import SynthFile

    ctx = Context(local)
    size = int(a.size_gib * GIB)
    sf = SynthFile(ctx, a.fmt, size)
    data = sf.window(0, size)
    R = sf.expected_count()
    if a.e2e:
        return e2e(a, ctx, sf, data, size, R)
    rows = ctx.alloc(16 * (R + 1024))

    for _ in range(a.warmup):
        r = ctx.build_buffer(data, size, rows, kind="record", fmt=None)
        assert r.ok or os.environ.get("SHOCKIDX_DEBUG"), r
    ctx.sync()
    idx_ms = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = ctx.build_buffer(data, size, rows, kind="record", fmt=None)
        idx_ms.append(r.timings["index_ms"])
    ctx.sync()
    dt = time.perf_counter() - t0
    ms = dt / a.steps * 1e3
    count = r.count

    ok = (count == R and r.fmt == a.fmt)
    mism = -1
    if a.check:
        if a.fmt == "fastq":
            mism = sf.check_rows(rows, 0, count)
        else:  # FASTA: the '\n' padding belongs to the last record (fasta.go EOF piece)
            mism = sf.check_rows(rows, 0, count - 1)
            last = rows.download(16, 16 * (count - 1)).view(np.uint64)
            off_last = int(sf.d_off.download(8, 8 * (count - 1)).view(np.uint64)[0])
            mism += int(not (last[0] == off_last and last[1] == size - off_last))
        ok = ok and mism == 0

    k_ms = float(np.mean(idx_ms))
    alg_bytes = size + 16 * count
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    cfg = {"workload": f"{a.fmt} record index, {a.size_gib:g} GiB synthetic node file in HBM (BASELINE configs[1])"
           if a.fmt == "fastq" else f"fasta record index, {a.size_gib:g} GiB (BASELINE configs[2])",
           "records": count, "bytes": size, "tile": TILE, "parallelism": "single slab"}
    traffic = load_pmc(a.pmc or os.path.join(ROOT, "profiles", f"pmc_{a.fmt}.json"), {"fmt": a.fmt, "bytes": size})
    out = {
        "metric": METRIC,
        "value": round(size / (ms * 1e-3) / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated, seed 0x5EED, SURVEY.md §8(d))",
        "config": cfg,
        "mrecords_per_s": round(count / (ms * 1e-3) / 1e6, 2),
        "index_kernel_ms": round(k_ms, 4),
        "lookback_selfhelp": r.selfhelp,
        "fixups": r.fixups, "fixup_tiles": r.fix_tiles,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes": alg_bytes},
        "parity": {"rows_checked": count if a.check else 0, "mismatches": mism, "count_ok": count == R},
    }
    if a.cpu_sec > 0:
        sample_n = min(size, int(a.cpu_sample_gib * GIB))
        k = sf._count_le(sample_n) - 1  # cut the sample at a record boundary
        sample_n = int(sf.d_off.download(8, 8 * k).view(np.uint64)[0]) if k > 0 else sample_n
        host = data.download(sample_n)
        out["cpu_baseline"] = cpu_baseline(host, a.fmt, a.cpu_sec)
    print(json.dumps(out))
    if not ok:
        print(f"PARITY FAILURE: count {count} expected {R}, mismatches {mism}, status {r.status} "
              f"err {r.err} state_out {r.state_out} term {r.term_code} flags {r.flags}", file=sys.stderr)
        return 1
    return 0


def e2e(a, ctx, sf, data, size, R):
    """End-to-end rate of shockidx_build_host: the file starts and ends in host memory
    (a POSTed body): chunked H2D through pinned staging, index kernels, table D2H."""
    host = data.download(size)
    data.free()
    sf.free()
    for _ in range(a.warmup):
        r = ctx.build_host(host, kind="record")
    t = []
    parts = []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        r = ctx.build_host(host, kind="record")
        t.append(time.perf_counter() - t0)
        parts.append(r.timings)
    ms = float(np.mean(t)) * 1e3
    avg = {k: round(float(np.mean([p[k] for p in parts])), 3) for k in parts[0]}
    print(json.dumps({"metric": "end-to-end index build from host memory (PCIe-inclusive)", "value": round(size / (ms * 1e-3) / GIB, 3),
                      "unit": "GiB/s", "ms_per_step": round(ms, 3), "steps": a.steps, "fmt": a.fmt, "bytes": size,
                      "records": r.count, "count_ok": r.count == R, "ok": r.ok, "timings_ms": avg,
                      "path": "pageable host buffer -> memcpy into 2 x 64 MiB pinned staging -> hipMemcpyAsync H2D; "
                              "table D2H through the same staging"}))
    return 0 if (r.ok and r.count == R) else 1


if __name__ == "__main__":
    sys.exit(main())
