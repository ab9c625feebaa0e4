"""Scratch: write a libpcap capture of a bench config's synthetic frames (for timing
retina_amd/_lib/rtn_offline end to end).

    python scratch/mk_pcap.py cfg2 16777216 /tmp/cfg2.pcap
"""
import struct
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import bench  # noqa: E402

cfg, n, path = sys.argv[1], int(sys.argv[2]), sys.argv[3]
stride = bench.CONFIGS[cfg][1]
with open(path, "wb") as f:
    f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
    chunk = 1 << 20
    for s in range(0, n, chunk):
        k = min(chunk, n - s)
        slab, dlen = bench.gen_frames(cfg, k, s)
        rec = np.zeros((k, 16 + stride), np.uint8)
        hdr = rec[:, :16].view(np.uint32)
        hdr[:, 0] = np.arange(s, s + k, dtype=np.uint32)
        hdr[:, 2] = dlen
        hdr[:, 3] = dlen
        rec[:, 16:] = slab.reshape(k, stride)
        mask = np.arange(16 + stride)[None, :] < (16 + dlen.astype(np.int64))[:, None]
        f.write(rec[mask].tobytes())
