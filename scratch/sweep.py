"""Scratch: interleaved timing of kernel variants, each "DEFINES@GRID" (DEFINES comma-separated,
GRID blocks; 0 = runtime default), plus an in-run read ceiling.

    python scratch/sweep.py cfg2 "@0;@1280;RTN_CHUNK_GROUPS=4u@0" [reps]
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc, synth  # noqa: E402

cfg = sys.argv[1]
entries = ["RTN_EXP_CEILING@0"] + sys.argv[2].split(";")
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
_, stride, n, _ = bench.CONFIGS[cfg]
n = int(os.environ.get("FRAMES", n))
slab, dlen = bench.gen_frames(cfg, n, 0)
alg = synth.alg_read_bytes(slab, dlen, stride)
dev = torch.device("cuda", 0)
d_ext = None
if stride > 64 and not os.environ.get("MONO"):
    head, ext = pc.split_slab(slab, stride)
    d_slab = torch.from_numpy(head).to(dev)
    d_ext = torch.from_numpy(ext).to(dev)
    stride = 64
else:
    d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
spec = bench.spec_for(cfg)
ctxs = []
out = None
for e in entries:
    defs, grid = e.split("@")
    os.environ["RTN_KERNEL_DEFINES"] = defs
    ctx = pc.PacketContinue(pc.Program.from_spec(spec), 0)
    if int(grid):
        ctx.set_grid(int(grid))
    out = out or ctx.alloc_outputs(n, addr6=True, counters=False)
    ctxs.append((e, ctx))
    print("compiled", e, flush=True)
times = {e: [] for e, _ in ctxs}
K = 10
for r in range(reps):
    for e, ctx in ctxs:
        for _ in range(2):
            ctx.run(d_slab, stride, d_dlen, n, out, ext=d_ext)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            ctx.run(d_slab, stride, d_dlen, n, out, ext=d_ext)
        e1.record()
        torch.cuda.synchronize()
        times[e].append(e0.elapsed_time(e1) / K)
ceil = statistics.median(times[entries[0]])
print(f"{cfg} n={n}: ceiling {ceil:.4f} ms = {d_slab.numel() / ceil / 1e6:.0f} GB/s slab read")
for e, ts in times.items():
    ms = statistics.median(ts)
    print(f"{cfg} {e:44s} {ms:.4f} ms {n / ms / 1e3:9.1f} Mpkt/s frac {alg / ms / 1e6 / 8000:.3f} "
          f"vs-ceil {ceil / ms:.3f} spread {(max(ts) - min(ts)) / ms:.3f}", flush=True)
