"""Scratch: per-dispatch counters (grouped by dispatch order) for a pmc_ctx.sh tag."""
import collections, csv, glob, sys
tag = sys.argv[1]
for d in sorted(glob.glob(f"gpurun_out/pc_{tag}_*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(d)))
    disp = collections.OrderedDict()
    for r in rows:
        if "rtn_pc" not in r["Kernel_Name"]:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), {"t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    print("==", d)
    for k, v in disp.items():
        print(f"  {k:3d} " + " ".join(f"{a}={b:.4g}" for a, b in v.items()))
