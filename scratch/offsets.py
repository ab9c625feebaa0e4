"""Scratch: does the relative placement of the record output (and the slab) decide the fast/slow
mode? Times one kernel variant with out.l4 placed at several byte offsets inside one big buffer.

    python scratch/offsets.py cfg2 "DEFINES" "0,4096,65536,1048576" [slab_offsets]
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

cfg = sys.argv[1]
os.environ["RTN_KERNEL_DEFINES"] = sys.argv[2]
offs = [int(x) for x in sys.argv[3].split(",")]
soffs = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
PAD = max(soffs) + 4096
big_slab = torch.empty(slab.size + PAD, dtype=torch.uint8, device=dev)
h = torch.from_numpy(slab)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
if os.environ.get("GRID"):
    ctx.set_grid(int(os.environ["GRID"]))
out = ctx.alloc_outputs(n, addr6=True, counters=False)
l4n = out.l4.numel()
big = torch.empty(l4n + max(offs) + 4096, dtype=torch.uint8, device=dev)
print("slab", hex(big_slab.data_ptr()), "l4 base", hex(big.data_ptr()), "bm", hex(out.pc_bitmap.data_ptr()), flush=True)
times = {}
K = 10
for so in soffs:
    d_slab = big_slab[so:so + slab.size]
    d_slab.copy_(h)
    for r in range(5):
        for o in offs:
            out.l4 = big[o:o + l4n]
            for _ in range(2):
                ctx.run(d_slab, stride, d_dlen, n, out)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                ctx.run(d_slab, stride, d_dlen, n, out)
            e1.record()
            torch.cuda.synchronize()
            times.setdefault((so, o), []).append(e0.elapsed_time(e1) / K)
for (so, o), ts in times.items():
    ms = statistics.median(ts)
    print(f"{cfg} slab+{so:<9d} l4+{o:<10d} {ms:.4f} ms {n / ms / 1e3:9.1f} Mpkt/s spread {(max(ts) - min(ts)) / ms:.3f}",
          flush=True)
