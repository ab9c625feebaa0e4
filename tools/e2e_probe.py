"""End-to-end-from-mbufs probe (experiments only): bench.e2e_from_mbufs over a few
(chunk frames, stager threads, streams) settings, one JSON line each.

    python tools/e2e_probe.py cfg2|cfg3 [frames]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def main() -> None:
    import torch

    import bench
    from retina_amd import pc

    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 21
    stride = bench.CONFIGS[cfg][1]
    slab, dlen = bench.gen_frames(cfg, m, 0)
    dev = torch.device("cuda", 0)
    ctx = pc.PacketContinue(pc.Program.from_spec(bench.spec_for(cfg)), 0)
    for chunk, threads, ns in ((1 << 19, 14, 4), (1 << 18, 14, 4), (1 << 18, 12, 4), (1 << 18, 10, 4),
                               (1 << 17, 12, 4), (1 << 18, 12, 2), (1 << 20, 12, 2)):
        r = bench.e2e_from_mbufs(ctx, slab, dlen, stride, dev, frames=m, chunk=chunk, nstreams=ns, threads=threads)
        r.pop("note", None)
        print(json.dumps({"cfg": cfg, "chunk": chunk, "threads": threads, "streams": ns, **r}), flush=True)


if __name__ == "__main__":
    main()
