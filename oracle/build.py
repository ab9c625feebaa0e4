"""ORACLE (test infrastructure only): prebuild the generated-C oracle for the benchmark and test
subscription sets into oracle/_build/ (gcc -O3 -march=native). The reference itself is not
buildable here (Rust + DPDK + libpcap, no cargo/rustc), so there is no oracle/_ref build."""
from __future__ import annotations

import sys
from pathlib import Path


def build_all() -> None:
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    from golden.filter_sets import SETS  # noqa: E402

    from oracle import cgen, filterlang  # noqa: E402

    for spec in SETS.values():
        cgen.OracleLib(filterlang.PacketTree(filterlang.load_spec(spec)))


if __name__ == "__main__":
    build_all()
