"""Register / LDS / spill report of a config's specialised kernels, compiled here (hiprtc needs no
GPU) from the product kernel or from tools/variants.py variants (tools/README.md).

    python tools/kernel_resources.py cfg2|cfg3|cfg4 [VARIANT ...] [--isa DIR]

Prints, per variant and kernel: VGPRs, SGPRs, SGPR spills, LDS bytes, waves per SIMD the VGPRs
allow, and the count of v_readlane / v_writelane (SGPR spill traffic) in the kernel body. --isa
writes each variant's disassembly to DIR."""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
LLVM = Path("/opt/rocm/lib/llvm/bin")


def report(co: bytes, isa_out: Path | None = None) -> list[dict]:
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "k.co"
        f.write_bytes(co)
        notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(f)], check=True, capture_output=True,
                               text=True).stdout
        dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(f)], check=True,
                             capture_output=True, text=True).stdout
    if isa_out:
        isa_out.write_text(dis)
    bodies = {m.group(1): m.start() for m in re.finditer(r"^[0-9a-f]+ <(\w+)>:", dis, re.M)}
    order = sorted(bodies.items(), key=lambda kv: kv[1])
    text = {}
    for i, (name, at) in enumerate(order):
        text[name] = dis[at:order[i + 1][1] if i + 1 < len(order) else len(dis)]
    out = []
    for blk in notes.split("  - .agpr_count")[1:]:
        g = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
        name = g.get("name", "?")
        vg = int(g.get("vgpr_count", 0))
        body = text.get(name, "")
        out.append({"kernel": name, "vgpr": vg, "sgpr": int(g.get("sgpr_count", 0)),
                    "sgpr_spill": int(g.get("sgpr_spill_count", 0)), "vgpr_spill": int(g.get("vgpr_spill_count", 0)),
                    "lds": int(g.get("group_segment_fixed_size", 0)),
                    "waves_per_simd": min(8, 512 // max(8, -(-vg // 8) * 8)),
                    "readlane": body.count("v_readlane"), "writelane": body.count("v_writelane"),
                    "insts": sum(1 for ln in body.splitlines() if ln.startswith("\t"))})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("variants", nargs="*", default=["base"])
    ap.add_argument("--isa", type=Path, default=None)
    args = ap.parse_args()
    import bench
    import variants
    from retina_amd import pc

    exp = pc._LIB_PATH.with_name("libretina_pc_exp.so")
    if not exp.exists() or exp.stat().st_mtime < pc._LIB_PATH.stat().st_mtime:
        raise SystemExit("libretina_pc_exp.so is missing or older than libretina_pc.so: run tools/build_experiments.py")
    pc._LIB_PATH = exp
    spec = bench.spec_for(args.cfg)
    tmp = Path(tempfile.mkdtemp())
    for v in args.variants or ["base"]:
        name, _, kopts = v.partition("%")  # VARIANT%opt,opt: extra hiprtc options, as in tools/ab.py
        os.environ["RTN_KERNEL_OPTS"] = kopts.replace(",", " ")
        os.environ["RTN_KERNEL_TEMPLATE"] = str(variants.write(name, tmp))
        co = pc.Program.from_spec(spec).code_object()
        isa = None
        if args.isa:
            args.isa.mkdir(parents=True, exist_ok=True)
            isa = args.isa / f"{args.cfg}_{name.replace('+', '_')}{'_' + str(abs(hash(kopts)) % 10**6) if kopts else ''}.s"
        for r in report(co, isa):
            if r["kernel"].startswith("rtn_pc_kernel"):
                print(f"{args.cfg} {v:24s} {r['kernel']:22s} vgpr {r['vgpr']:3d} ({r['waves_per_simd']} waves) "
                      f"sgpr {r['sgpr']:3d} spill {r['sgpr_spill']:3d} readlane {r['readlane']:3d} "
                      f"lds {r['lds']:6d} insts {r['insts']}", flush=True)


if __name__ == "__main__":
    main()
