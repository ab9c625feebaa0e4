"""Scratch: interleaved A/B timing of kernel variants (RTN_KERNEL_DEFINES) + an in-run ceiling."""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
variants = sys.argv[2].split(";") if len(sys.argv) > 2 else ["", "RTN_NO_PREFETCH"]
grid = int(sys.argv[3]) if len(sys.argv) > 3 else 1536
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 7
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
alg = synth.alg_read_bytes(slab, dlen, stride)
dev = torch.device("cuda", 0)
d_ext = None
if os.environ.get("SPLIT") and stride > 64:
    head, ext = pc.split_slab(slab, stride)
    d_slab = torch.from_numpy(head).to(dev)
    d_ext = torch.from_numpy(ext).to(dev)
    stride = 64
else:
    d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
spec = bench.spec_for(cfg)
ctxs = {}
shared_out = None
for j, var in enumerate(["RTN_EXP_CEILING"] + variants):
    os.environ["RTN_KERNEL_DEFINES"] = var.split("#")[0]
    ctx = pc.PacketContinue(pc.Program.from_spec(spec), 0)
    ctx.set_grid(grid)
    out = shared_out = (shared_out if j else ctx.alloc_outputs(n, addr6=True, counters=False))
    key = var if var not in ctxs else f"{var}#{j}"
    ctxs[key] = (ctx, out)
    print(key, hex(out.l4.data_ptr()), hex(out.pc_bitmap.data_ptr()), hex(d_slab.data_ptr()), flush=True)
times = {v: [] for v in ctxs}
K = 10
for r in range(reps):
    for var, (ctx, out) in ctxs.items():
        for _ in range(2):
            ctx.run(d_slab, stride, d_dlen, n, out, ext=d_ext)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            ctx.run(d_slab, stride, d_dlen, n, out, ext=d_ext)
        e1.record()
        torch.cuda.synchronize()
        times[var].append(e0.elapsed_time(e1) / K)
ceil = statistics.median(times["RTN_EXP_CEILING"])
print(f"{cfg} grid {grid}: ceiling {ceil:.4f} ms = {n * stride / ceil / 1e6:.0f} GB/s slab read")
for var, ts in times.items():
    ms = statistics.median(ts)
    print(f"{cfg} var={var or 'default':34s} {ms:.4f} ms  {n / ms / 1e3:9.1f} Mpkt/s  frac {alg / ms / 1e6 / 8000:.3f}"
          f"  vs ceiling {ceil / ms:.3f}  spread {(max(ts) - min(ts)) / ms:.3f}", flush=True)
