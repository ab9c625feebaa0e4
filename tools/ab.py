"""In-process A/B timing of kernel variants on one GPU (tools/README.md).

    python tools/ab.py cfg2|cfg3|cfg4 VARIANT[:DEFINES][@GRID][%OPTS][^CPW][#split|#compact|#mono] ... [--reps R]
        [--frames N] [--mono] [--compact]

VARIANT names a tools/variants.py function (or several joined with '+'). Prints, per entry, the
median kernel time over R interleaved rounds of 10 launches, Mpkt/s and the HBM-read roofline
fraction of the bench's algorithmic bytes."""
from __future__ import annotations

import argparse
import os
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tools"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("entries", nargs="+")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--mono", action="store_true")
    ap.add_argument("--compact", action="store_true", help="compact split layout (RTN_BATCH_EXT_COMPACT)")
    args = ap.parse_args()
    import torch

    import bench
    import variants
    from retina_amd import pc, synth

    exp = pc._LIB_PATH.with_name("libretina_pc_exp.so")  # the experiments build
    if not exp.exists() or exp.stat().st_mtime < pc._LIB_PATH.stat().st_mtime:
        raise SystemExit("libretina_pc_exp.so is missing or older than libretina_pc.so: run tools/build_experiments.py")
    pc._LIB_PATH = exp
    _, stride, n, _ = bench.CONFIGS[args.cfg]
    n = args.frames or n
    slab, dlen = bench.gen_frames(args.cfg, n, 0)
    alg = synth.alg_read_bytes(slab, dlen, stride)
    dev = torch.device("cuda", 0)
    # the layouts an entry may ask for ("VARIANT#compact"): split (default for wide slots),
    # compact split, or the monolithic slots with --mono
    lay = {}
    if stride > 64:
        head, ext = pc.split_slab(slab, stride)
        lay["split"] = (torch.from_numpy(head).to(dev), 64, torch.from_numpy(ext).to(dev), None)
        if args.compact or any("#compact" in e for e in args.entries):
            h2, ext2, chunk = pc.split_slab(slab, stride, dlen, compact=True)
            lay["compact"] = (lay["split"][0], 64, torch.from_numpy(ext2).to(dev),
                              torch.from_numpy(chunk.view(np.int32)).to(dev))
        for cf in (128, 256, 512):
            if any(e.endswith(f"#compact{cf}") for e in args.entries):
                # the same ext rows, first rows per cf-frame chunk (timing of the chunk-size variants)
                need = pc.ext_needed(slab.reshape(-1, stride), dlen).astype(np.int64)
                per = np.add.reduceat(need, np.arange(0, n, cf))
                cx = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint32)
                lay[f"compact{cf}"] = (lay["split"][0], 64, lay["compact"][2], torch.from_numpy(cx.view(np.int32)).to(dev))
    if stride == 64 or args.mono or any(e.endswith("#mono") for e in args.entries):
        lay["mono"] = (torch.from_numpy(slab).to(dev), stride, None, None)
    default = "mono" if (stride == 64 or args.mono) else ("compact" if args.compact else "split")
    d_dlen = torch.from_numpy(dlen.view(np.int16)).to(dev)
    le64 = stride == 64 and int(dlen.max()) <= 64
    spec = bench.spec_for(args.cfg)
    tmp = ROOT / "gpurun_out" / "variants"
    ctxs, out = [], None
    for e in args.entries:
        name, _, layout = e.partition("#")
        name, _, cpw = name.partition("^")  # VARIANT^N: N chunks per wave in the compact split kernel
        if cpw:
            os.environ["RTN_CPW"] = cpw
        else:
            os.environ.pop("RTN_CPW", None)
        name, _, kopts = name.partition("%")  # VARIANT%opt,opt: extra hiprtc options (comma-separated)
        os.environ["RTN_KERNEL_OPTS"] = kopts.replace(",", " ")
        name, _, grid = name.partition("@")
        name, _, defs = name.partition(":")
        os.environ["RTN_KERNEL_TEMPLATE"] = str(variants.write(name, tmp))
        os.environ["RTN_KERNEL_DEFINES"] = defs
        os.environ["RTN_BLOCK"] = "128" if "wpb2" in name.split("+") else "256"
        ctx = pc.PacketContinue(pc.Program.from_spec(spec), 0)
        if grid:
            ctx.set_grid(int(grid))
        if out is None:
            out = ctx.alloc_outputs(n, addr6=True, counters=False)
            if any(x.startswith("file=") for x in args.entries):
                # a kernel from before round 3's 24-B addr6 entries writes 32 B per IPv6 record
                import dataclasses
                out = dataclasses.replace(out, addr6=torch.empty(out.addr6.numel() * 32 // 24, dtype=torch.uint8, device=dev))
        ctxs.append((e, ctx, lay[layout or default]))
        print("compiled", e, flush=True)
    times = {e: [] for e, _, _ in ctxs}
    for _ in range(args.reps):
        for e, ctx, (d_slab, st, d_ext, d_chunk) in ctxs:
            for _ in range(2):
                ctx.run(d_slab, st, d_dlen, n, out, ext=d_ext, dl_le64=le64 and d_ext is None, ext_chunk=d_chunk)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ctx.run(d_slab, st, d_dlen, n, out, ext=d_ext, dl_le64=le64 and d_ext is None, ext_chunk=d_chunk)
            e1.record()
            torch.cuda.synchronize()
            times[e].append(e0.elapsed_time(e1) / 10)
    for e, ts in times.items():
        ms = statistics.median(ts)
        print(f"{args.cfg} {e:40s} {ms:.4f} ms {n / ms / 1e3:9.1f} Mpkt/s frac {alg / ms / 1e6 / 8000:.3f} "
              f"spread {(max(ts) - min(ts)) / ms:.3f}", flush=True)


if __name__ == "__main__":
    main()
