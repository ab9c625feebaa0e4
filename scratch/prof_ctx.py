"""Scratch: several contexts (separate module loads) of one variant, each run R times in turn.
Dispatch order under rocprofv3: ctx0 x R, ctx1 x R, ... (after one warm-up round)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

os.environ["RTN_KERNEL_DEFINES"] = sys.argv[1] if len(sys.argv) > 1 else ""
nctx = int(sys.argv[2]) if len(sys.argv) > 2 else 4
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cfg = "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
spec = bench.spec_for(cfg)
ctxs = [pc.PacketContinue(pc.Program.from_spec(spec), 0) for _ in range(nctx)]
out = ctxs[0].alloc_outputs(n, addr6=True, counters=False)
for c in ctxs:
    c.set_grid(1536)
    c.run(d_slab, stride, d_dlen, n, out)
torch.cuda.synchronize()
for j, c in enumerate(ctxs):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(R):
        c.run(d_slab, stride, d_dlen, n, out)
    e1.record()
    torch.cuda.synchronize()
    print(f"ctx {j}: {e0.elapsed_time(e1) / R:.4f} ms", flush=True)
