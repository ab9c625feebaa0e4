"""Scratch: is the fast/slow mode a property of the loaded module or of time?
Per-launch event timings for C contexts, launched round-robin, L rounds."""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

os.environ["RTN_KERNEL_DEFINES"] = sys.argv[1] if len(sys.argv) > 1 else ""
C = int(sys.argv[2]) if len(sys.argv) > 2 else 6
L = int(sys.argv[3]) if len(sys.argv) > 3 else 40
cfg = "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
spec = bench.spec_for(cfg)
ctxs = [pc.PacketContinue(pc.Program.from_spec(spec), 0) for _ in range(C)]
out = ctxs[0].alloc_outputs(n, addr6=True, counters=False)
for c in ctxs:
    c.set_grid(1536)
    c.run(d_slab, stride, d_dlen, n, out)
torch.cuda.synchronize()
ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(L)] for _ in range(C)]
for r in range(L):
    for j, c in enumerate(ctxs):
        ev[j][r][0].record()
        c.run(d_slab, stride, d_dlen, n, out)
        ev[j][r][1].record()
torch.cuda.synchronize()
for j in range(C):
    ts = [a.elapsed_time(b) for a, b in ev[j]]
    print(f"ctx {j}: median {statistics.median(ts):.4f} ms  min {min(ts):.4f}  max {max(ts):.4f}  "
          + " ".join(f"{t:.3f}" for t in ts[:16]), flush=True)
# same context, long run
c = ctxs[0]
ts = []
for r in range(200):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); c.run(d_slab, stride, d_dlen, n, out); b.record()
    ts.append((a, b))
torch.cuda.synchronize()
t = [a.elapsed_time(b) for a, b in ts]
print("ctx0 x200:", " ".join(f"{x:.3f}" for x in t[::5]))
