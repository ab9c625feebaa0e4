"""Where the GPU capture walk's host time goes (diagnostics for DESIGN §9): on a cfg2 / cfg3
capture in the page cache, times hipHostRegister / host->HBM copy / hipHostUnregister of a
256-MiB range of the file mapping, a host memcpy of it into pinned memory, and each
rtn_pcap_next_batch_gpu call of a walk over the capture (1M-frame batches).

    python tools/walk_probe.py cfg2|cfg3 [frames]
"""
from __future__ import annotations

import ctypes
import json
import mmap
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main() -> None:
    import torch

    import bench
    from offline_bench import write_pcap
    from retina_amd import pc

    cfg = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 24 if cfg == "cfg2" else 1 << 21)
    slab, dlen = bench.gen_frames(cfg, n, 0)
    torch.zeros(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    W = 256 << 20
    with tempfile.TemporaryDirectory() as d:
        cap = Path(d) / "cap.pcap"
        write_pcap(cap, slab, dlen, bench.CONFIGS[cfg][1])
        del slab
        out = {"cfg": cfg, "frames": n, "bytes": cap.stat().st_size}
        f = open(cap, "rb")
        m = mmap.mmap(f.fileno(), 0, prot=mmap.PROT_READ)
        view = np.frombuffer(m, np.uint8)
        base = view.ctypes.data
        _ = int(view[::4096].sum())  # page in
        dev = torch.empty(W, dtype=torch.uint8, device="cuda")
        pinned = torch.empty(W, dtype=torch.uint8, pin_memory=True)
        s = {}
        for rep in range(3):
            off = (rep * W) % max(1, (len(m) - W)) & ~4095
            t0 = time.perf_counter()
            rc = hip.hipHostRegister(ctypes.c_void_p(base + off), ctypes.c_size_t(W), ctypes.c_uint(8))
            t1 = time.perf_counter()
            assert rc == 0, rc
            rc = hip.hipMemcpy(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(base + off), ctypes.c_size_t(W), 1)
            t2 = time.perf_counter()
            assert rc == 0, rc
            hip.hipHostUnregister(ctypes.c_void_p(base + off))
            t3 = time.perf_counter()
            ctypes.memmove(pinned.data_ptr(), base + off, W)
            t4 = time.perf_counter()
            dev.copy_(pinned)
            torch.cuda.synchronize()
            t5 = time.perf_counter()
            s = {"register_ms": (t1 - t0) * 1e3, "h2d_registered_ms": (t2 - t1) * 1e3,
                 "unregister_ms": (t3 - t2) * 1e3, "memcpy_1thread_ms": (t4 - t3) * 1e3,
                 "h2d_pinned_ms": (t5 - t4) * 1e3}
            print(json.dumps({"range_MiB": W >> 20, "rep": rep, **{k: round(v, 3) for k, v in s.items()}}), flush=True)
        del view
        m.close()
        f.close()
        B = 1 << 20
        head = torch.empty(B * 64, dtype=torch.uint8, device="cuda")
        ext = torch.empty(pc.gather_ext_rows(B) * 64, dtype=torch.uint8, device="cuda")
        ch = torch.empty(B // 256, dtype=torch.int32, device="cuda")
        dl = torch.empty(B, dtype=torch.int16, device="cuda")
        for rep in range(2):
            r = pc.PcapReader(cap)
            calls = []
            while True:
                t0 = time.perf_counter()
                k = r.next_batch_gpu(head, ext, ch, dl)
                torch.cuda.synchronize()
                calls.append(((time.perf_counter() - t0) * 1e3, k))
                if k == 0:
                    break
            out[f"calls_ms_rep{rep}"] = [round(c[0], 3) for c in calls]
            out[f"total_ms_rep{rep}"] = round(sum(c[0] for c in calls), 3)
            del r
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
