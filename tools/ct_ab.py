"""In-process A/B of connection-lookup kernel variants (experiments build, tools/README.md).

    python tools/ct_ab.py [--frames N] [--reps R] [--steps K] [--profile] VARIANT ...

Builds the bench's cfg2 batch (2^25 frames: 8.4 M forwarded, 1.05 M SYN-only openers), runs the
packet stage with the connection stage once, then per variant a 2^25-slot table admitting 10 M
connections (configs/online.toml) and its first pass (the openers open). The timed passes are
the steady state the bench's conn_stage.ct_lookup reports: openers find their connection, the
other frames of unknown flows drop. VARIANT is `base` (the embedded ct_kernel.hip) or a
tools/ct_variants.py name; every variant's statuses must equal base's. --profile runs base only,
K steady passes, for rocprofv3."""
from __future__ import annotations

import argparse
import os
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tools")]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", default=["base"])
    ap.add_argument("--frames", type=int, default=1 << 25)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    import torch

    import bench
    import ct_variants
    from retina_amd import pc

    exp = pc._LIB_PATH.with_name("libretina_pc_exp.so")
    if not exp.exists() or exp.stat().st_mtime < pc._LIB_PATH.stat().st_mtime:
        raise SystemExit("libretina_pc_exp.so is missing or older than libretina_pc.so: run tools/build_experiments.py")
    pc._LIB_PATH = exp
    n = args.frames
    slab, dlen = bench.gen_frames("cfg2", n, 0)
    dev = torch.device("cuda", 0)
    ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for("cfg2")), 0)
    out = ctx.alloc_outputs(n, addr6=True, counters=False, conn=True)
    ctx.run(torch.from_numpy(slab).to(dev), 64, torch.from_numpy(dlen.view(np.int16)).to(dev), n, out, dl_le64=True)
    torch.cuda.synchronize()
    del slab
    names = ["base"] if args.profile else args.variants
    tables = {}
    tmp = ROOT / "tools" / "_ab" / "ct"
    for v in names:
        if v == "base":
            os.environ.pop("RTN_CT_TEMPLATE", None)
        else:
            os.environ["RTN_CT_TEMPLATE"] = str(ct_variants.write(v, tmp))
        ct = pc.ConnTable(0, 25, 10_000_000)
        ent = ct.process(out)
        torch.cuda.synchronize()
        tables[v] = (ct, ent)
    os.environ.pop("RTN_CT_TEMPLATE", None)
    if args.profile:
        ct, ent = tables["base"]
        for _ in range(args.steps):
            ct.process(out, out=ent)
        torch.cuda.synchronize()
        print("profiled", args.steps, "steady passes")
        return
    ref = pc.decode_ct(tables["base"][1], out)[:, 1]
    times = {v: [] for v in names}
    for _ in range(args.reps):
        for v in names:
            ct, ent = tables[v]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                ct.process(out, out=ent)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.steps)
    for v in names:
        st = pc.decode_ct(tables[v][1], out)[:, 1]
        same = bool(np.array_equal(st, ref))
        print(f"{v:24s} {statistics.median(times[v]):.4f} ms  (min {min(times[v]):.4f})  statuses equal base: {same}",
              flush=True)


if __name__ == "__main__":
    main()
