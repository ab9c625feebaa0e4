"""Summarise scripts/profile_ct.sh outputs into profiles/<tag>_ct_pmc.json.

    python scripts/ct_pmc_summary.py <tag>

Kernel-trace stats of the steady passes (the first insert, which opens the connections, is
reported apart) and the median per dispatch of every PMC counter of rtn_ct_insert / rtn_ct_lookup.
FETCH_SIZE / WRITE_SIZE are KiB; the table's 64-B probe reads are not the wide coalesced reads the
gfx950 half-count applies to, so FETCH_SIZE is reported raw."""
from __future__ import annotations

import collections
import csv
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNELS = ("rtn_ct_insert", "rtn_ct_lookup")


def main(tag: str) -> None:
    out = ROOT / "gpurun_out"
    trace = list(csv.DictReader(open(out / f"ctprof_{tag}" / "run_kernel_trace.csv")))
    res: dict = {"source": f"rocprofv3 over tools/ct_ab.py --profile (cfg2 batch of 2^25 frames, 2^25-slot table), {tag}"}
    for k in KERNELS:
        ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace if r["Kernel_Name"].startswith(k)]
        res[k] = {"first_us": round(ns[0] / 1e3, 1), "steady_median_us": round(statistics.median(ns[1:]) / 1e3, 1),
                  "steady_launches": len(ns) - 1}
    for p in sorted(out.glob(f"ctpmc_{tag}_*/run_counter_collection.csv")):
        per: dict = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(p)):
            for k in KERNELS:
                if r["Kernel_Name"].startswith(k):
                    per[(k, r["Counter_Name"])][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
        for (k, c), d in per.items():
            # the first dispatch is the opening pass: the median is the steady state
            res[k].setdefault("counters", {})[c] = statistics.median(d.values())
    for k in KERNELS:
        c = res[k].get("counters", {})
        if "TCC_HIT_sum" in c:
            res[k]["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
        if "SQ_WAIT_INST_ANY" in c:
            res[k]["wait_inst_any_frac"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3)
    dst = ROOT / "profiles" / f"{tag}_ct_pmc.json"
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
