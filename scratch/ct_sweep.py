"""Scratch: connection-lookup timing vs table capacity on the cfg2 batch (first pass inserts,
then timed passes over the same batch).

    python scratch/ct_sweep.py [cap_log2,...]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

caps = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "21,22,24").split(",")]
import os  # noqa: E402
defs = sys.argv[2].split(";") if len(sys.argv) > 2 else [""]
cfg = "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
out = ctx.alloc_outputs(n, addr6=True, counters=False, conn=True)
ctx.run(d_slab, stride, d_dlen, n, out)
torch.cuda.synchronize()
for c, d in [(c, d) for d in defs for c in caps]:
    os.environ["RTN_KERNEL_DEFINES"] = d
    ct = pc.ConnTable(0, c)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    ent = ct.process(out)
    e1.record()
    K = 10
    for _ in range(K):
        ct.process(out, out=ent)
    e2.record()
    torch.cuda.synchronize()
    st = ct.stats()
    print(f"[{d}] cap 2^{c} ({(1 << c) * 64 >> 20} MiB): first pass {e0.elapsed_time(e1):.3f} ms, "
          f"steady {e1.elapsed_time(e2) / K:.4f} ms, live {st['live']}", flush=True)
    del ct
    torch.cuda.empty_cache()
