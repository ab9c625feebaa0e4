"""Kernel time over several seconds of back-to-back cfg2 launches in one process, then again
after an idle pause: does the "two speeds" state follow sustained load?

    python tools/speed_trace.py [seconds] [pause]

Prints one line per window of 50 launches: elapsed wall time, median kernel ms."""
from __future__ import annotations

import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    import torch

    import bench
    from retina_amd import pc

    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
    pause = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    n = 1 << 25
    slab, dlen = bench.gen_frames("cfg2", n, 0)
    dev = torch.device("cuda", 0)
    d_slab = torch.from_numpy(slab).to(dev)
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for("cfg2")), 0)
    out = ctx.alloc_outputs(n, addr6=True, counters=False)
    ctx.run(d_slab, 64, d_dlen, n, out, dl_le64=True)
    torch.cuda.synchronize()
    for phase in ("load", "after pause"):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(51)]
            evs[0].record()
            for k in range(50):
                ctx.run(d_slab, 64, d_dlen, n, out, dl_le64=True)
                evs[k + 1].record()
            torch.cuda.synchronize()
            ts = [evs[k].elapsed_time(evs[k + 1]) for k in range(50)]
            print(f"{phase:12s} t={time.perf_counter() - t0:6.2f}s median {statistics.median(ts):.4f} ms "
                  f"min {min(ts):.4f} max {max(ts):.4f}", flush=True)
        if phase == "load":
            time.sleep(pause)


if __name__ == "__main__":
    main()
