"""Build the native parts in-tree (no setuptools, no JIT cache): the filter compiler + HIP runtime
shared library, the rtnc CLI, and an ahead-of-time gfx950 compile of the kernel template as a
build check. Outputs land in retina_amd/_lib/ (git-ignored, shipped to the GPU box by gpurun)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "_lib"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

FILTERGEN_SRCS = ["ast.cpp", "parser.cpp", "filter.cpp", "ptree.cpp", "codegen.cpp", "hwfilter.cpp"]
SO_NAME = "libretina_pc.so"
RUNTIME_SRCS = ["runtime/rtn_runtime.cpp", "runtime/rtn_hw.cpp", "ingest/pcap_ingest.cpp", "ingest/mbuf_stage.cpp"]


def _run(cmd: list[str], cwd: Path | None = None) -> None:
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} (exit {r.returncode})")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _gen_kernel_inc(name: str = "pc_kernel", var: str = "kPcKernelSrc", where: str = "runtime") -> Path:
    """Embed a kernel source as a C++ raw string (compiled by hiprtc at run time)."""
    src = CSRC / "kernels" / f"{name}.hip"
    inc = CSRC / where / f"{name}_src.inc"
    text = src.read_text()
    delim = "RTNSRC"
    assert f"){delim}\"" not in text
    body = f'static const char* const {var} = R"{delim}(' + text + f'){delim}";\n'
    if not inc.exists() or inc.read_text() != body:
        inc.write_text(body)
    return inc


def build_library(force: bool = False) -> Path:
    LIB.mkdir(exist_ok=True)
    inc = _gen_kernel_inc()
    inc_ct = _gen_kernel_inc("ct_kernel", "kCtKernelSrc")
    inc_st = _gen_kernel_inc("stage_kernel", "kStageKernelSrc", "ingest")
    inc_cw = _gen_kernel_inc("capwalk_kernel", "kCapwalkKernelSrc", "ingest")
    fg = [CSRC / "filtergen" / s for s in FILTERGEN_SRCS]
    rt = [CSRC / s for s in RUNTIME_SRCS]
    hdrs = (list((CSRC / "filtergen").glob("*.hpp")) + list((CSRC / "runtime").glob("*.hpp"))
            + list((ROOT / "include").glob("*.h")) + [inc, inc_ct, inc_st, inc_cw])
    so = LIB / SO_NAME
    if force or _stale(so, fg + rt + hdrs):
        cmd = [
            "g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-pthread", "-Wall", "-Wextra", "-Wno-unused-parameter",
            "-D__HIP_PLATFORM_AMD__", f"-I{ROOT / 'include'}", f"-I{ROCM / 'include'}",
            *map(str, fg), *map(str, rt), "-o", str(so),
            f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}", "-lamdhip64", "-lhiprtc",
        ]
        _run(cmd)
    # the batched offline runtime in C++ (examples/rtn_offline.cpp) on the C ABI
    off = LIB / "rtn_offline"
    off_src = ROOT / "examples" / "rtn_offline.cpp"
    if force or _stale(off, [off_src, so] + hdrs):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", f"-I{ROOT / 'include'}",
              f"-I{ROCM / 'include'}", str(off_src), "-o", str(off), f"-L{LIB}", "-lretina_pc",
              "-Wl,-rpath,$ORIGIN", f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}", "-lamdhip64"])
    # the C++ Subscription mirror (include/retina_subscription.hpp) driven by its GPU test
    chk = LIB / "subscription_check"
    chk_src = ROOT / "tests" / "cpp" / "subscription_check.cpp"
    if force or _stale(chk, [chk_src, so, ROOT / "include" / "retina_subscription.hpp"] + hdrs):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-D__HIP_PLATFORM_AMD__", f"-I{ROOT / 'include'}",
              f"-I{ROCM / 'include'}", str(chk_src), "-o", str(chk), f"-L{LIB}", "-lretina_pc",
              "-Wl,-rpath,$ORIGIN", f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}", "-lamdhip64"])
    cli = LIB / "rtnc"
    main = CSRC / "filtergen" / "rtnc_main.cpp"
    if force or _stale(cli, fg + [main] + hdrs):
        _run(["g++", "-std=c++17", "-O2", "-Wall", *map(str, fg), str(main), "-o", str(cli)])
    return so


def build_kernel_check() -> Path:
    """Ahead-of-time hipcc compile of the kernel template with the config-2 filter spliced in
    (the same translation unit hiprtc builds at run time) to catch template breakage at build."""
    so = LIB / SO_NAME
    # the program-independent gather kernel (rtn_stage_gather), hiprtc-compiled at pool registration
    st_src = CSRC / "kernels" / "stage_kernel.hip"
    st_out = LIB / "stage_kernel.hsaco"
    if _stale(st_out, [st_src]):
        _run([str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--genco",
              str(st_src), "-o", str(st_out)])
    # ... and the capture-walk kernels (rtn_pcap_next_batch_gpu)
    cw_src = CSRC / "kernels" / "capwalk_kernel.hip"
    cw_out = LIB / "capwalk_kernel.hsaco"
    if _stale(cw_out, [cw_src]):
        _run([str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--genco",
              str(cw_src), "-o", str(cw_out)])
    out = LIB / "pc_kernel_cfg2.hsaco"
    src = LIB / "pc_kernel_cfg2.hip"
    tpl = CSRC / "kernels" / "pc_kernel.hip"
    if not _stale(out, [tpl, so]):
        return out
    sys.path.insert(0, str(ROOT))
    from retina_amd import pc  # noqa: E402

    prog = pc.Program.from_filter("tcp.dst_port = 80", ["ConnRecord"])
    src.write_text(prog.source)
    _run([str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--genco",
          str(src), "-o", str(out)])
    return out


def build_oracle() -> None:
    sys.path.insert(0, str(ROOT))
    from oracle import build as obuild  # noqa: E402

    obuild.build_all()


def build_all(force: bool = False) -> None:
    build_library(force)
    build_kernel_check()
    build_oracle()


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built", LIB)
