"""Scratch: which output array's allocation decides the fast/slow mode."""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

os.environ["RTN_KERNEL_DEFINES"] = "RTN_UNROLL2"
cfg = "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
ctx.set_grid(1536)


def timeit(out, K=10, reps=3):
    ts = []
    for _ in range(reps):
        ctx.run(d_slab, stride, d_dlen, n, out)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            ctx.run(d_slab, stride, d_dlen, n, out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / K)
    return statistics.median(ts)


sets = [ctx.alloc_outputs(n, addr6=True, counters=False) for _ in range(6)]
res = []
for j, o in enumerate(sets):
    ms = timeit(o)
    res.append(ms)
    print(f"set {j}: l4 {o.l4.data_ptr():#x} pc {o.pc_bitmap.data_ptr():#x} fwd {o.fwd_bitmap.data_ptr():#x} "
          f"{ms:.4f} ms {n / ms / 1e3:8.1f}", flush=True)
fast = int(np.argmin(res))
slow = int(np.argmax(res))
F, S = sets[fast], sets[slow]
import copy  # noqa: E402
for name in ("l4", "pc_bitmap", "fwd_bitmap"):
    o = copy.copy(F)
    setattr(o, name, getattr(S, name))
    ms = timeit(o)
    print(f"fast set with slow {name}: {ms:.4f} ms {n / ms / 1e3:8.1f}", flush=True)
    o = copy.copy(S)
    setattr(o, name, getattr(F, name))
    ms = timeit(o)
    print(f"slow set with fast {name}: {ms:.4f} ms {n / ms / 1e3:8.1f}", flush=True)
