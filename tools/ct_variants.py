"""Timing variants of retina_amd/csrc/kernels/ct_kernel.hip (tools/ct_ab.py), made by text patches."""
from __future__ import annotations

from pathlib import Path

KERNEL = Path(__file__).resolve().parent.parent / "retina_amd" / "csrc" / "kernels" / "ct_kernel.hip"


def _sub(src: str, old: str, new: str) -> str:
    assert old in src, f"variant patch does not apply: {old[:60]!r}"
    return src.replace(old, new)


def base(src: str) -> str:
    return src


VARIANTS = {"base": base}


def write(name: str, outdir: Path) -> Path:
    outdir.mkdir(parents=True, exist_ok=True)
    src = KERNEL.read_text()
    for s in name.split("+"):
        src = VARIANTS[s](src)
    p = outdir / f"ct_kernel_{name.replace('+', '_')}.hip"
    p.write_text(src)
    return p
