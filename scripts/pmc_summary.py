"""Summarise rocprofv3 outputs into profiles/ (committed evidence for bench.py's roofline block).

    python scripts/pmc_summary.py <tag> <cfg> <frames>

Reads gpurun_out/prof_<tag>_<cfg>/run_kernel_stats.csv (kernel-trace --stats pass) and
gpurun_out/pmc_<tag>_<cfg>_<k>/run_counter_collection.csv (separate --pmc passes of
scripts/profile.sh: 1 FETCH_SIZE, 2 WRITE_SIZE, then request / wave counters) and writes
profiles/<tag>_<cfg>_kernel_stats.csv and profiles/pmc_<cfg>.json.
HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: FETCH_SIZE/WRITE_SIZE are in KiB
and gfx950 reports exactly half the bytes of a wide coalesced read in FETCH_SIZE
(MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact for 16-B-per-lane stores.
"""
from __future__ import annotations

import csv
import json
import shutil
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL = "rtn_pc_kernel"


def counter(path: Path, name: str | None = None) -> list[float]:
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows if r.get("Kernel_Name", "").startswith(KERNEL)
            and (name is None or r.get("Counter_Name") == name)]


def counters(path: Path) -> dict:
    """Median per dispatch of every counter of one pass (values summed over a dispatch's rows)."""
    per: dict = {}
    for r in csv.DictReader(open(path)):
        if not r.get("Kernel_Name", "").startswith(KERNEL):
            continue
        key = (r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    out: dict = {}
    for (cn, _), v in per.items():
        out.setdefault(cn, []).append(v)
    return {cn: statistics.median(v) for cn, v in out.items()}


def main(tag: str, cfg: str, frames: int) -> None:
    out = ROOT / "gpurun_out"
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    ks = out / f"prof_{tag}_{cfg}" / "run_kernel_stats.csv"
    shutil.copy(ks, prof / f"{tag}_{cfg}_kernel_stats.csv")
    stats = {r["Name"]: r for r in csv.DictReader(open(ks))}
    # the dominant packet-stage kernel (rtn_pc_kernel_s64 for 64-byte slots, rtn_pc_kernel otherwise)
    name = max((n for n in stats if n.startswith(KERNEL)), key=lambda n: float(stats[n]["TotalDurationNs"]))
    k = stats[name]
    # per-launch durations: bench.py runs warm-up + timed launches on preallocated outputs, then
    # one launch on freshly allocated outputs for the totals (first-touch of new buffers makes that
    # one slow); the bench's HIP-event figure corresponds to the launches before it
    trace = [r for r in csv.DictReader(open(out / f"prof_{tag}_{cfg}" / "run_kernel_trace.csv"))
             if r["Kernel_Name"] == name]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
    steady = durs[:-1] if len(durs) > 1 else durs
    fetch = counter(out / f"pmc_{tag}_{cfg}_1" / "run_counter_collection.csv", "FETCH_SIZE")
    write = counter(out / f"pmc_{tag}_{cfg}_2" / "run_counter_collection.csv", "WRITE_SIZE")
    extra = {}
    for ps in (3, 4):
        p = out / f"pmc_{tag}_{cfg}_{ps}" / "run_counter_collection.csv"
        if p.exists():
            extra.update(counters(p))
    f_kb, w_kb = statistics.median(fetch), statistics.median(write)
    d = {
        "tag": tag, "config": cfg, "frames": frames, "kernel": name,
        "kernel_avg_ns": float(k["AverageNs"]), "kernel_calls": int(k["Calls"]),
        "kernel_avg_ns_preallocated_outputs": statistics.mean(steady),
        "kernel_median_ns": statistics.median(durs), "kernel_durations_ns": durs,
        "fetch_size_kib_median": f_kb, "write_size_kib_median": w_kb, "pmc_dispatches": [len(fetch), len(write)],
        "read_bytes_per_launch": int(2 * f_kb * 1024), "write_bytes_per_launch": int(w_kb * 1024),
        "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
        "counters_per_launch": extra,
        "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of wide coalesced reads); write = WRITE_SIZE KiB",
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; kernel stats from "
                  f"rocprofv3 --kernel-trace --stats ({tag})",
    }
    (prof / f"pmc_{cfg}.json").write_text(json.dumps(d, indent=2) + "\n")
    print(json.dumps(d, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
