"""Scratch: how output-buffer placement (relative to the slab) changes kernel time."""
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
cfg = "cfg2"
_, stride, n, _ = bench.CONFIGS[cfg]
slab, dlen = bench.gen_frames(cfg, n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
ctx.set_grid(1536)
L = pc.lib()
nb = L.rtn_out_bitmap_bytes(n)
nl = L.rtn_out_l4_bytes(n)
MB = 1 << 20
pool_r = torch.empty(nl + 512 * MB, dtype=torch.uint8, device=dev)
pool_b = torch.empty(2 * nb + 512 * MB, dtype=torch.uint8, device=dev)
print("slab", hex(d_slab.data_ptr()), "pool_r", hex(pool_r.data_ptr()), "pool_b", hex(pool_b.data_ptr()))


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


def mk(off_r, off_b):
    return pc.PCOutputs(n=n, pc_bitmap=pool_b[off_b:off_b + nb], fwd_bitmap=pool_b[off_b + nb:off_b + 2 * nb],
                        l4=pool_r[off_r:off_r + nl], addr6=None, dlv_bitmap=None, dlv_records=None, counters=None,
                        deliver_words=0)


for off_r in [0, 1 * MB, 2 * MB, 4 * MB, 8 * MB, 16 * MB, 32 * MB, 64 * MB, 128 * MB, 256 * MB, 3 * MB + 4096]:
    ms = timeit(mk(off_r, 0))
    print(f"records +{off_r / MB:8.3f} MB  bitmaps +0     : {ms:.4f} ms  {n / ms / 1e3:8.1f} Mpkt/s", flush=True)
for off_b in [0, 4096, 64 * 1024, 1 * MB, 2 * MB, 8 * MB, 64 * MB, 256 * MB]:
    ms = timeit(mk(0, off_b))
    print(f"records +0  bitmaps +{off_b / MB:8.3f} MB: {ms:.4f} ms  {n / ms / 1e3:8.1f} Mpkt/s", flush=True)
