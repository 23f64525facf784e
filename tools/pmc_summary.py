"""Summarise rocprofv3 output of bench.py runs into profiles/ (dev tool, runs on the GPU box).

usage: python tools/pmc_summary.py <kernel-trace dir> <FETCH_SIZE dir> <WRITE_SIZE dir> <out.json> [fmt] [bytes]

Per-launch HBM traffic of the dominant kernel (k_fq_tiles for FASTQ, k_fa_tiles for FASTA), with the
gfx950 corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes
of a 16-B/lane streaming read -> x2; WRITE_SIZE is exact for 16-B/lane stores.  rocprofv3
reports both counters in KiB.
"""
import csv
import glob
import json
import os
import sys


def _rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


KERNEL = os.environ.get("PMC_KERNEL", "")


def kernel_name(fmt: str) -> str:
    if KERNEL:
        return KERNEL
    if fmt == "fastq":
        return "k_fq_tiles"
    return "k_index1" if os.environ.get("SHOCKIDX_FA_MODE", "") in ("two", "0") else "k_fa_tiles"


def dominant(name: str, fmt: str) -> bool:
    return kernel_name(fmt) + "(" in name or kernel_name(fmt) + "<" in name


def counter_per_launch(d, counter, fmt):
    per = {}
    for r in _rows(d, "counter_collection.csv"):
        if r.get("Counter_Name") != counter or not dominant(r.get("Kernel_Name", ""), fmt):
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    vals = list(per.values())
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def source_sha() -> str:
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = hashlib.sha256()
    for f in ("sidx_kernels.hip", "sidx_common.hpp", "sidx_device.hpp"):
        with open(os.path.join(root, "shock_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def kernel_stats(d):
    rows = _rows(d, "kernel_stats.csv")
    return [{k: r[k] for k in ("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")
             if k in r} for r in rows]


def main():
    kt, fd, wd, out = sys.argv[1:5]
    fmt = sys.argv[5] if len(sys.argv) > 5 else "fastq"
    nbytes = int(sys.argv[6]) if len(sys.argv) > 6 else 10 << 30
    stats = kernel_stats(kt)
    fetch_kib, nf = counter_per_launch(fd, "FETCH_SIZE", fmt)
    write_kib, nw = counter_per_launch(wd, "WRITE_SIZE", fmt)
    res = {
        "config": {"fmt": fmt, "bytes": nbytes},
        "kernel": kernel_name(fmt),
        "source_sha": source_sha(),
        "kernel_stats": stats,
        "fetch_size_kib_raw": fetch_kib, "fetch_launches": nf,
        "write_size_kib_raw": write_kib, "write_launches": nw,
        "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 16-B/lane streaming reads); "
                      "write bytes = WRITE_SIZE x 1024",
    }
    if fetch_kib is not None and write_kib is not None:
        rd = 2 * fetch_kib * 1024
        wr = write_kib * 1024
        res.update({"hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                    "hbm_bytes_per_launch": rd + wr, "read_over_input": rd / nbytes})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernel_stats"}))
    for s in stats:
        print(s)


if __name__ == "__main__":
    main()
