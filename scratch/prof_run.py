"""Scratch: run one kernel variant K times (for rocprofv3 --pmc passes)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

os.environ["RTN_KERNEL_DEFINES"] = sys.argv[1] if len(sys.argv) > 1 else ""
cfg = sys.argv[2] if len(sys.argv) > 2 else "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
ctx.set_grid(1536)
out = ctx.alloc_outputs(n, addr6=True, counters=False)
for _ in range(6):
    ctx.run(d_slab, stride, d_dlen, n, out)
torch.cuda.synchronize()
print("ok")
