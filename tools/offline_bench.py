"""End-to-end offline runtime (examples/rtn_offline.cpp) on a synthetic capture: writes a libpcap
file of full frames (the bench's seeded cfg2 or cfg3 frames, zero payload), then runs the C++
offline runtime over it in each layout (gpu: the capture walk on the GPU) and prints its JSON
summary lines.

    python tools/offline_bench.py cfg2|cfg3 [frames] [--no-ct]
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def write_pcap(path: Path, slab: np.ndarray, dlen: np.ndarray, stride: int) -> None:
    rows = slab.reshape(-1, stride)
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        if len(dlen) and int(dlen.min()) == int(dlen.max()) <= stride:  # fixed-size frames: vectorised
            k = int(dlen[0])
            rec = np.zeros((len(dlen), 16 + k), np.uint8)
            hdr = rec[:, :16].view(np.uint32)
            hdr[:, 0] = np.arange(len(dlen), dtype=np.uint32)
            hdr[:, 2] = k
            hdr[:, 3] = k
            rec[:, 16:] = rows[:, :k]
            f.write(rec.tobytes())
            return
        chunk = 1 << 16
        for s in range(0, len(dlen), chunk):
            parts = []
            for i in range(s, min(s + chunk, len(dlen))):
                n = int(dlen[i])
                body = rows[i, :min(n, stride)].tobytes()
                parts.append(struct.pack("<IIII", i, 0, n, n) + body + bytes(max(0, n - stride)))
            f.write(b"".join(parts))


def main() -> None:
    import bench

    cfg = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else (1 << 24 if cfg == "cfg2" else 1 << 21)
    extra = ["--no-ct"] if "--no-ct" in sys.argv else []
    slab, dlen = bench.gen_frames(cfg, n, 0)
    stride = bench.CONFIGS[cfg][1]
    with tempfile.TemporaryDirectory() as d:
        cap = Path(d) / "cap.pcap"
        write_pcap(cap, slab, dlen, stride)
        spec = Path(d) / "spec.toml"
        spec.write_text(bench.spec_for(cfg))
        exe = ROOT / "retina_amd" / "_lib" / "rtn_offline"
        # gpu: the window's file pages registered and copied by the copy engine; gpu-staged: the
        # fallback, worker threads copying them into pinned memory first (RTN_GPU_WALK_STAGED)
        # gpu-1s: the walk on the stages' stream (--one-stream)
        # gpu-w256m / gpu-w1g: 256-MiB / 1-GiB windows (default 64 MiB)
        # *-inline: the results walked on the main thread (--inline-results)
        for name, layout in (("gpu", "gpu"), ("gpu-inline", "gpu"), ("gpu-1s", "gpu"), ("gpu-staged", "gpu"),
                             ("gpu-w256m", "gpu"), ("gpu-w1g", "gpu"), ("compact", "compact"),
                             ("compact-inline", "compact"), ("mono", "mono"), ("gpu", "gpu"), ("compact", "compact")):
            env = dict(os.environ, RTN_GPU_WALK_STAGED="1" if name == "gpu-staged" else "0")
            more = {"gpu-inline": ["--inline-results"], "compact-inline": ["--inline-results"],
                    "gpu-1s": ["--one-stream"], "gpu-w256m": ["--window", str(256 << 20)],
                    "gpu-w1g": ["--window", str(1 << 30)]}.get(name, [])
            for _ in range(2):  # the second run has the capture in the page cache
                r = subprocess.run([str(exe), str(spec), str(cap), "--layout", layout, *extra, *more],
                                   capture_output=True, text=True, timeout=300, env=env)
                if r.returncode:
                    sys.stderr.write(r.stderr)
                    raise SystemExit(r.returncode)
            line = json.loads(r.stdout.strip().splitlines()[-1])
            line["walk"] = name
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
