"""Print per-launch SQ counters of one kernel ($KN, default k_fq_tiles) from gpurun_out/sqabl_<dbg>/ (dev tool)."""
import csv, glob, os, sys, collections
KN = os.environ.get("KN", "k_fq_tiles")
for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for p in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if KN in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {k: f"{sum(v)/len(v):.3e}" for k, v in sorted(agg.items())})
