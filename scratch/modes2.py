"""Scratch: back-to-back launches (events only around the batch) vs an event after every launch."""
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
C = int(sys.argv[2]) if len(sys.argv) > 2 else 4
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
K = 10


def batch(c):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        c.run(d_slab, stride, d_dlen, n, out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


def each(c, sync=False):
    evs = []
    for _ in range(K):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); c.run(d_slab, stride, d_dlen, n, out); b.record()
        evs.append((a, b))
        if sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs)


def each_total(c):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mid = [torch.cuda.Event() for _ in range(K)]
    e0.record()
    for k in range(K):
        c.run(d_slab, stride, d_dlen, n, out)
        mid[k].record()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


res = {}
for r in range(4):
    for j, c in enumerate(ctxs):
        for name, fn in (("batch", batch), ("each", each), ("each_total(non-timing events)", each_total),
                         ("each+sync", lambda c: each(c, True))):
            res.setdefault((j, name), []).append(fn(c))
for (j, name), ts in sorted(res.items()):
    print(f"ctx {j} {name:32s} median {statistics.median(ts):.4f} ms  " + " ".join(f"{t:.4f}" for t in ts), flush=True)
