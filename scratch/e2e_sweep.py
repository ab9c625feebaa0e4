"""Scratch: bench.e2e_rate over chunk sizes and stream counts (cfg2, 2^25 frames)."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402
from retina_amd import pc  # noqa: E402

_, stride, n, _ = bench.CONFIGS["cfg2"]
slab, dlen = bench.gen_frames("cfg2", n, 0)
dev = torch.device("cuda", 0)
ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for("cfg2")), 0)
for chunk, ns in ((1 << 21, 4), (1 << 20, 8), (1 << 21, 6), (1 << 20, 4), (1 << 21, 8), (1 << 21, 4)):
    print(chunk, ns, bench.e2e_rate(ctx, slab, dlen, stride, dev, chunk, ns)["mpps"], flush=True)
