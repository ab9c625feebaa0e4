"""Kernel time per window of 10 back-to-back launches from the first launch of a process on, for
the bench's layout of a config: does the kernel speed up after some launches?

    python tools/warm_probe.py cfg2|cfg3|cfg4 [seconds]

Prints one line per window (the first 20 windows, then every 100th): elapsed wall time since the
first launch, launches so far, median kernel ms of the window."""
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

    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    _, stride, n, _ = bench.CONFIGS[cfg]
    slab, dlen = bench.gen_frames(cfg, n, 0)
    dev = torch.device("cuda", 0)
    ext = chunk = None
    if stride > 64:
        head, e, c = pc.split_slab(slab, stride, dlen, compact=True)
        d_slab = torch.from_numpy(head).to(dev)
        ext = torch.from_numpy(e).to(dev)
        chunk = torch.from_numpy(c.view(np.int32)).to(dev)
    else:
        d_slab = torch.from_numpy(slab).to(dev)
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    le64 = stride == 64 and int(dlen.max()) <= 64
    ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
    out = ctx.alloc_outputs(n, addr6=True, counters=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = w = 0
    while time.perf_counter() - t0 < secs:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
        evs[0].record()
        for j in range(10):
            ctx.run(d_slab, 64, d_dlen, n, out, ext=ext, ext_chunk=chunk, dl_le64=le64)
            evs[j + 1].record()
        torch.cuda.synchronize()
        ts = [evs[j].elapsed_time(evs[j + 1]) for j in range(10)]
        k += 10
        if w < 20 or w % 100 == 0:
            print(f"{cfg} t={time.perf_counter() - t0:6.3f}s launches {k:5d} median {statistics.median(ts):.4f} ms "
                  f"min {min(ts):.4f} max {max(ts):.4f}", flush=True)
        w += 1


if __name__ == "__main__":
    main()
