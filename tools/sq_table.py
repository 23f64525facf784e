"""Per-launch SQ counters of one kernel from a rocprofv3 --pmc run (dev tool, runs on the GPU box).

usage: KN=k_fq_tiles python tools/sq_table.py <pmc dir under gpurun_out/>
Prints, per counter, the mean over the kernel's dispatches (each dispatch summed over instances).
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    if not os.path.isabs(d):
        d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", d)
    kn = os.environ.get("KN", "k_fq_tiles")
    per = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p, newline="")):
            name = r.get("Kernel_Name", "")
            if kn + "(" not in name and kn + "<" not in name:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            c = per.setdefault(r["Counter_Name"], {})
            c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    print(f"{kn} ({d})")
    for n in sorted(per):
        v = list(per[n].values())
        print(f"  {n:28s} {sum(v) / len(v):16.4g}   ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
