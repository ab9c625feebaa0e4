"""Timing variants of retina_amd/csrc/kernels/ct_kernel.hip (tools/ct_ab.py), made by text patches."""
from __future__ import annotations

from pathlib import Path

KERNEL = Path(__file__).resolve().parent.parent / "retina_amd" / "csrc" / "kernels" / "ct_kernel.hip"


def _sub(src: str, old: str, new: str) -> str:
    assert old in src, f"variant patch does not apply: {old[:60]!r}"
    return src.replace(old, new)


def base(src: str) -> str:
    return src


def dbg(src: str) -> str:
    """printf every insert-pass opener whose frame index is past the batch (debugging)."""
    return _sub(src, "      frame = rtn_ct_frame(ch, it.k);\n",
                "      frame = rtn_ct_frame(ch, it.k);\n"
                "      if (frame >= a.n) printf(\"BADFRAME c=%u lane=%u rd=%u e=%u nop=%u k=%u frame=%u total=%u p=%u,%u,%u w=%llx,%llx,%llx,%llx cv=%llx\\n\", "
                "c, lane, rd, e, nop, it.k, frame, ch.total, ch.p0, ch.p01, ch.p012, ch.w[0], ch.w[1], ch.w[2], ch.w[3], it.cv);\n")


VARIANTS = {"base": base, "dbg": dbg}


def write(name: str, outdir: Path) -> Path:
    outdir.mkdir(parents=True, exist_ok=True)
    src = KERNEL.read_text()
    for s in name.split("+"):
        src = VARIANTS[s](src)
    p = outdir / f"ct_kernel_{name.replace('+', '_')}.hip"
    p.write_text(src)
    return p
