"""Is the per-process "two speeds" of one code object a property of where the
buffers land? Times the product kernel on several device copies of the same cfg2 slab and
several output sets, in one process, interleaved.

    python tools/alloc_probe.py [copies] [outsets] [--hipmalloc]
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

    copies = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    outsets = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    n = 1 << 25
    slab, dlen = bench.gen_frames("cfg2", n, 0)
    dev = torch.device("cuda", 0)
    slabs = [torch.from_numpy(slab).to(dev) for _ in range(copies)]
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for("cfg2")), 0)
    outs = [ctx.alloc_outputs(n, addr6=True, counters=False) for _ in range(outsets)]
    combos = [(i, j) for i in range(copies) for j in range(outsets)]
    times = {c: [] for c in combos}
    for _ in range(5):
        for i, j in combos:
            for _ in range(3):
                ctx.run(slabs[i], 64, d_dlen, n, outs[j], dl_le64=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ctx.run(slabs[i], 64, d_dlen, n, outs[j], dl_le64=True)
            e1.record()
            torch.cuda.synchronize()
            times[(i, j)].append(e0.elapsed_time(e1) / 10)
    for (i, j), ts in times.items():
        print(f"slab {i} (0x{slabs[i].data_ptr():x}) out {j} (l4 0x{outs[j].l4.data_ptr():x}): "
              f"{statistics.median(ts):.4f} ms  [{min(ts):.4f} .. {max(ts):.4f}]", flush=True)


if __name__ == "__main__":
    main()
