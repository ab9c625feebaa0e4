"""Scratch: first end-to-end GPU check of config 2 (throwaway; the real tests live in tests/)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from retina_amd import pc, synth  # noqa: E402

n = 1 << 25
t = time.time()
slab, dlen = synth.cfg2(n)
print("gen", time.time() - t, flush=True)
dev = torch.device("cuda", 0)
slab_d = torch.from_numpy(slab).to(dev)
dlen_d = torch.from_numpy(dlen.view(np.int16)).to(dev)
prog = pc.Program.from_spec(synth.CFG2_SPEC)
ctx = pc.PacketContinue(prog, 0)
out = ctx.alloc_outputs(n)
ctx.run(slab_d, 64, dlen_d, n, out)
torch.cuda.synchronize()
res = out.decode()
cnt = out.counters_host()
b = slab.reshape(n, 64)
dport = (b[:, 36].astype(np.uint32) << 8) | b[:, 37]
exp = dport == 80
print("counters", cnt, "expected pc", exp.sum())
assert np.array_equal(res["pc"], exp), "pc mismatch"
assert np.array_equal(res["fwd"], exp), "fwd mismatch"
l4 = res["l4"]
ei = np.nonzero(exp)[0]
assert np.array_equal(l4["pkt_idx"], ei)
src = (b[ei, 26].astype(np.uint32) << 24) | (b[ei, 27].astype(np.uint32) << 16) | (b[ei, 28].astype(np.uint32) << 8) | b[ei, 29]
assert np.array_equal(l4["src_ip4"], src)
sport = (b[ei, 34].astype(np.uint32) << 8) | b[ei, 35]
assert np.array_equal(l4["ports"], sport | (80 << 16))
assert np.all(l4["off_len"] == (54 | (10 << 16)))
seq = (b[ei, 38].astype(np.uint32) << 24) | (b[ei, 39].astype(np.uint32) << 16) | (b[ei, 40].astype(np.uint32) << 8) | b[ei, 41]
assert np.array_equal(l4["seq_no"], seq)
assert np.all((l4["proto_flags"] & 0xff) == 6)
assert np.array_equal((l4["proto_flags"] >> 8) & 0xff, b[ei, 47])
print("parity ok")
for grid in (1024, 2048, 4096):
    ctx.set_grid(grid)
    out2 = ctx.alloc_outputs(n, addr6=False, counters=False)
    for _ in range(3):
        ctx.run(slab_d, 64, dlen_d, n, out2)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    K = 20
    for _ in range(K):
        ctx.run(slab_d, 64, dlen_d, n, out2)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    print(f"grid {grid}: {ms:.3f} ms  {n / ms / 1e3:.1f} Mpkt/s  alg {n * 66 / ms / 1e6:.1f} GB/s  "
          f"frac {n * 66 / ms / 1e6 / 8000:.3f}")
