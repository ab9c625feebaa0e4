"""Scratch: same code object loaded several times (different code addresses), same buffers."""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

os.environ["RTN_KERNEL_DEFINES"] = sys.argv[1] if len(sys.argv) > 1 else "RTN_UNROLL2"
nctx = int(sys.argv[2]) if len(sys.argv) > 2 else 6
cfg = "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
prog = pc.Program.from_spec(bench.spec_for(cfg))
ctxs = [pc.PacketContinue(prog, 0) for _ in range(nctx)]
for c in ctxs:
    c.set_grid(1536)
out = ctxs[0].alloc_outputs(n, addr6=True, counters=False)
times = [[] for _ in ctxs]
for r in range(5):
    for j, c in enumerate(ctxs):
        c.run(d_slab, stride, d_dlen, n, out)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            c.run(d_slab, stride, d_dlen, n, out)
        e1.record()
        torch.cuda.synchronize()
        times[j].append(e0.elapsed_time(e1) / 10)
for j, ts in enumerate(times):
    ms = statistics.median(ts)
    print(f"ctx {j}: {ms:.4f} ms {n / ms / 1e3:8.1f} Mpkt/s spread {(max(ts) - min(ts)) / ms:.3f}", flush=True)
