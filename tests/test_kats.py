"""The reference's own filter-compiler unit tests (ptree.rs, ast.rs, actions.rs, datatypes.rs),
ported to C++ in tests/cpp/test_kats.cpp and run against the product compiler sources."""
from __future__ import annotations

import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
FG = ROOT / "retina_amd" / "csrc" / "filtergen"


def test_reference_compiler_kats():
    with tempfile.TemporaryDirectory() as d:
        exe = Path(d) / "kats"
        srcs = [str(FG / s) for s in ("ast.cpp", "parser.cpp", "filter.cpp", "ptree.cpp")]
        subprocess.run(["g++", "-std=c++17", "-O1", f"-I{FG}", str(ROOT / "tests/cpp/test_kats.cpp"), *srcs,
                        "-o", str(exe)], check=True, capture_output=True)
        r = subprocess.run([str(exe)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr + r.stdout
        assert "0 failed" in r.stdout
