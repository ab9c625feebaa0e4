"""Scratch: per-launch kernel times over a long back-to-back run (does the rate drift under load?),
then again after an idle gap.

    python scratch/trace_launches.py cfg2 [launches] [idle_s]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

cfg = sys.argv[1]
L = int(sys.argv[2]) if len(sys.argv) > 2 else 300
idle = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
out = ctx.alloc_outputs(n, addr6=True, counters=False)
ctx.run(d_slab, stride, d_dlen, n, out)
torch.cuda.synchronize()
for phase in range(2):
    time.sleep(idle)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
    ev[0].record()
    for i in range(L):
        ctx.run(d_slab, stride, d_dlen, n, out)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = [ev[i].elapsed_time(ev[i + 1]) for i in range(L)]
    rows = [f"{np.median(ts[i:i + 10]):.4f}" for i in range(0, L, 10)]
    print(f"phase {phase} (after {idle}s idle): median per 10 launches:", " ".join(rows), flush=True)
