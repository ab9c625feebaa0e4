"""One process, one cfg2 batch, 30 timed launches of the product kernel: prints the median
kernel time. Run several times (separately, or under rocprofv3 --pmc) to see the per-process
"two speeds" (DESIGN.md §4).

    python tools/speed_probe.py [frames]
"""
from __future__ import annotations

import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main() -> None:
    import torch

    import bench
    from retina_amd import pc

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 25
    slab, dlen = bench.gen_frames("cfg2", n, 0)
    dev = torch.device("cuda", 0)
    d_slab = torch.from_numpy(slab).to(dev)
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for("cfg2")), 0)
    out = ctx.alloc_outputs(n, addr6=True, counters=False)
    ts = []
    for _ in range(3):
        ctx.run(d_slab, 64, d_dlen, n, out, dl_le64=True)
    for _ in range(30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ctx.run(d_slab, 64, d_dlen, n, out, dl_le64=True)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"median {statistics.median(ts):.4f} ms min {min(ts):.4f} max {max(ts):.4f} "
          f"slab 0x{d_slab.data_ptr():x} l4 0x{out.l4.data_ptr():x}", flush=True)


if __name__ == "__main__":
    main()
