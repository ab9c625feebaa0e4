"""Scratch: rtn_pd_run timing on the cfg2 batch for kernel variants (RTN_KERNEL_DEFINES).

    python scratch/pd_sweep.py "RTN_PD_GPW=1;RTN_PD_GPW=2;RTN_PD_GPW=4"
"""
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402

defs = sys.argv[1].split(";") if len(sys.argv) > 1 else [""]
_, stride, n, _ = bench.CONFIGS["cfg2"]
slab, dlen = bench.gen_frames("cfg2", n, 0)
dev = torch.device("cuda", 0)
d_slab = torch.from_numpy(slab).to(dev)
d_dlen = torch.from_numpy(dlen.view("int16")).to(dev)
stream = torch.cuda.current_stream(0)
for d in defs:
    os.environ["RTN_KERNEL_DEFINES"] = d
    print(f"[{d}]", bench.pd_rate("cfg2", d_slab, stride, d_dlen, n, None, 0, stream, 20), flush=True)
