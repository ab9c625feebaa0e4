"""Host staging probe (experiments only): the rate of rtn_stage_mbufs on its own, with a
concurrent host -> HBM DMA stream, and by thread count, on mbuf-shaped buffers.

    python tools/stage_probe.py [cfg2|cfg3] [frames]
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

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
    pool, ptrs = pc.mbuf_pool(slab, dlen, stride, seed=17)
    cpus = sorted(os.sched_getaffinity(0))
    q = bench._host_cpus()["cgroup_quota_cpus"]
    if q:
        cpus = cpus[:max(1, int(q))]
    head = torch.empty(m * 64, dtype=torch.uint8).pin_memory()
    ext = torch.empty(m * 64, dtype=torch.uint8).pin_memory()
    chunk = torch.empty(m // 256 + 1, dtype=torch.int32).pin_memory()
    dl = torch.empty(m, dtype=torch.int16).pin_memory()

    def rate(st, reps=5):
        st.stage(ptrs, dlen, head, ext, chunk, dl, n=m, cap=m, ext_cap=m)
        t0 = time.perf_counter()
        for _ in range(reps):
            st.stage(ptrs, dlen, head, ext, chunk, dl, n=m, cap=m, ext_cap=m)
        return m * reps / (time.perf_counter() - t0) / 1e6

    for t in (1, 4, 8, 12, 14, 16):
        if t > len(cpus):
            continue
        pinned = rate(pc.Stager(t, cpus[-t:]))
        free = rate(pc.Stager(t, None))  # left to the scheduler (any CPU of the affinity mask)
        print(json.dumps({"cfg": cfg, "threads": t, "nt": True, "stage_mpps": round(pinned, 1),
                          "stage_mpps_unpinned": round(free, 1)}), flush=True)
    # with a concurrent DMA stream (1 GiB pinned -> HBM, back to back)
    dev = torch.device("cuda", 0)
    src = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    dst = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    stop = threading.Event()
    moved = [0]

    def dma():
        while not stop.is_set():
            with torch.cuda.stream(s):
                dst.copy_(src, non_blocking=True)
            s.synchronize()
            moved[0] += src.numel()

    t0 = time.perf_counter()
    th = threading.Thread(target=dma)
    th.start()
    st = pc.Stager(14 if len(cpus) >= 16 else max(1, len(cpus) - 2), cpus[-14:] if len(cpus) >= 16 else None)
    r = rate(st, 10)
    stop.set()
    th.join()
    gbs = moved[0] / (time.perf_counter() - t0) / 1e9
    print(json.dumps({"cfg": cfg, "threads": st.threads, "stage_mpps_with_dma": round(r, 1), "dma_gbs": round(gbs, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
