"""Bitmap tail probe (debugging): the raw last words of the pc / fwd bitmaps of a ragged batch, after
rtn_pc_run and after rtn_ct_process; bits past n must be zero.

    python tools/bm_probe.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def main() -> None:
    import torch

    torch.cuda.init()
    import helpers
    import test_ct as T
    from retina_amd import pc

    rng = np.random.default_rng(7)
    pool = helpers.flow_pool(rng, 1500)
    r = T._Run()
    for b in range(3):
        frames = helpers.flow_frames(rng, pool, 6000 + 37 * b)
        n = len(frames)
        slab, dlen = pc.pack_frames(frames, 128)
        dev = torch.device("cuda", 0)
        for fill in (0x00, 0xFF):
            out = r.ctx.alloc_outputs(n, conn=True)
            out.fwd_bitmap.fill_(fill)
            out.pc_bitmap.fill_(fill)
            r.ctx.run(torch.from_numpy(slab).to(dev), 128, torch.from_numpy(dlen.view(np.int16)).to(dev), n, out)
            torch.cuda.synchronize()
            f = out.fwd_bitmap.cpu().numpy().view(np.uint64)
            p = out.pc_bitmap.cpu().numpy().view(np.uint64)
            nw = (n + 63) // 64
            tail = n % 64
            mask = np.uint64(((1 << 64) - 1) ^ ((1 << tail) - 1)) if tail else np.uint64(0)
            print(f"batch {b} n={n} fill={fill:#x} words={len(f)} last fwd={int(f[nw - 1]):#018x} "
                  f"pc={int(p[nw - 1]):#018x} bits past n: fwd {int(f[nw - 1] & mask):#x} pc {int(p[nw - 1] & mask):#x}",
                  flush=True)
            r.ct.process(out)
            torch.cuda.synchronize()
            f2 = out.fwd_bitmap.cpu().numpy().view(np.uint64)
            print(f"   after ct: fwd last {int(f2[nw - 1]):#018x} changed {not np.array_equal(f, f2)}", flush=True)


if __name__ == "__main__":
    main()
