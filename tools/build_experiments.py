"""Build the experiments variant of the runtime library (tools/README.md)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from retina_amd import _build  # noqa: E402


def main() -> Path:
    _build.build_library()
    so = _build.LIB / "libretina_pc_exp.so"
    fg = [str(_build.CSRC / "filtergen" / s) for s in _build.FILTERGEN_SRCS]
    rt = [str(_build.CSRC / s) for s in _build.RUNTIME_SRCS]
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-DRTN_EXPERIMENTS", "-D__HIP_PLATFORM_AMD__",
           f"-I{ROOT / 'include'}", f"-I{_build.ROCM / 'include'}", *fg, *rt, "-o", str(so),
           f"-L{_build.ROCM / 'lib'}", f"-Wl,-rpath,{_build.ROCM / 'lib'}", "-lamdhip64", "-lhiprtc"]
    subprocess.run(cmd, check=True)
    return so


if __name__ == "__main__":
    print(main())
