"""Scratch: print median counter values per pass dir (rtn_pc kernels only)."""
import collections, csv, glob, statistics, sys
for tag in sys.argv[1:]:
    print("==", tag)
    for d in sorted(glob.glob(f"gpurun_out/pc_{tag}_*/run_counter_collection.csv")):
        rows = list(csv.DictReader(open(d)))
        vals = collections.defaultdict(list); ts = {}
        for r in rows:
            if "rtn_pc" not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            ts[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        t = statistics.median(ts.values()) if ts else 0
        print(f"  t={t:.1f}us " + " ".join(f"{k}={statistics.median(v):.4g}" for k, v in vals.items()))
