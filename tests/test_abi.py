"""The C-ABI library: loads on a machine without a GPU, exports every function declared in
include/*.h (retina_pc.h, retina_ingest.h), reports errors the way the header says, and its hiprtc path produces a
gfx950 code object for every named subscription set (no GPU needed to compile)."""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import pytest

from golden.filter_sets import SETS
from retina_amd import pc

HEADERS = sorted((Path(__file__).resolve().parent.parent / "include").glob("*.h"))


def declared_functions() -> list[str]:
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(rtn_[a-z0-9_]+)\s*\(", text))
        # header-only helpers (static inline) are not library symbols
        names -= set(re.findall(r"static inline [\w\s\*]+?\b(rtn_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_exports_every_declared_symbol():
    lib = C.CDLL(str(pc._LIB_PATH))
    names = declared_functions()
    assert len(names) >= 23 and len(HEADERS) >= 2
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(pc.EXPORTS), set(names) ^ set(pc.EXPORTS)


def test_error_codes_and_messages():
    with pytest.raises(pc.FilterError) as e:
        pc.Program.from_filter("tcp.dst_port = 99999", ["ConnRecord"])
    assert e.value.code == -74 and "out of range" in str(e.value)
    with pytest.raises(pc.FilterError):
        pc.Program.from_spec("[[subscriptions]]\nfilter = \"tcp\"\ndatatypes = [\"NoSuchType\"]\ncallback = \"x\"\n")
    with pytest.raises(pc.FilterError):
        pc.Program.from_spec("[[subscriptions]]\nfilter = \"tcp\"\ndatatypes = [\"ZcFrame\", \"ConnRecord\"]\ncallback = \"x\"\n")
    with pytest.raises(pc.FilterError):
        pc.Program.from_spec("[[subscriptions]]\nfilter = \"tcp\"\ndatatypes = [\"ZcFrame\", \"FiveTuple\"]\ncallback = \"x\"\n")
    L = pc.lib()
    assert L.rtn_pc_run(None, None, None, None) == -22
    assert L.rtn_program_info(None, None) == -22
    assert b"null" in L.rtn_last_error()


def test_program_text_outputs():
    p = pc.Program.from_spec(SETS["cfg2"])
    assert p.info == {"n_subscriptions": 1, "n_deliver_stmts": 0, "deliver_words": 0, "tree_size": 7,
                      "n_conn_stmts": 0, "conn_words": 0, "conn_tree_size": 3, "n_pd_stmts": 0,
                      "n_pd_facts": 0, "pd_tree_size": 1}
    assert "tcp.dst_port = 80" in p.tree
    assert "if tcp.dst_port() == 80 {" in p.rust
    assert "rtn_pc_kernel" in p.source and "RTN_DELIVER_WORDS 0" in p.source


@pytest.mark.parametrize("fset", list(SETS))
def test_hiprtc_builds_gfx950_code_object(fset):
    co = pc.Program.from_spec(SETS[fset]).code_object()
    assert len(co) > 1000
    assert b"gfx950" in co or co[:4] == b"\x7fELF" or co[:24].startswith(b"__CLANG_OFFLOAD_BUNDLE__")
    # every entry point rtn_pc_create looks up (rtn_runtime.cpp): four slot layouts, each with and
    # without the connection stage, the PacketDeliver filter and the index kernels
    for name in ("rtn_pc_kernel", "rtn_pc_kernel_s64", "rtn_pc_kernel_split", "rtn_pc_kernel_splitc",
                 "rtn_pd_kernel", "rtn_idx_count", "rtn_idx_scan", "rtn_idx_write"):
        for sym in (name, name + "_conn") if name.startswith("rtn_pc_kernel") else (name,):
            assert (sym + ".kd").encode() in co, sym


def test_output_sizes():
    L = pc.lib()
    assert L.rtn_out_bitmap_bytes(65) == 16
    CF = pc.CHUNK_FRAMES
    assert CF == 256
    assert L.rtn_out_l4_bytes(65) == CF * 16
    assert L.rtn_out_l4_bytes(1025) == 1280 * 16
    assert L.rtn_out_seqack_bytes(1025) == 1280 * 8
    assert L.rtn_out_addr6_bytes(1) == CF * 24  # source bytes 8..15 + destination (bytes 0..7 in the record)
    assert L.rtn_out_dlv_bytes(64, 2) == CF * 2 * 8      # masks only: the frame is the rank in dlv_bitmap
    assert L.rtn_out_bitmap_bytes(0xFFFFFFFF) == ((1 << 32) // 64) * 8   # 64-bit arithmetic, no wrap
    assert L.rtn_out_l4_bytes(0xFFFFFFFF) == (1 << 32) * 16


def test_headers_are_c(tmp_path):
    """include/*.h are plain C: a C11 translation unit including all of them compiles with gcc
    -Wall -Wextra -Werror, and links against libretina_pc.so (every declared symbol resolves)."""
    import re
    import subprocess

    inc = Path(__file__).resolve().parent.parent / "include"
    lib = Path(pc.__file__).resolve().parent / "_lib"
    names = set()
    for h in HEADERS:
        names |= set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rtn_\w+)\s*\(", h.read_text(), re.M))
    src = "".join(f'#include "{h.name}"\n' for h in HEADERS)
    src += "#include <stdio.h>\nint main(void) {\n"
    src += "".join(f'  printf("%p\\n", (void*)&{n});\n' for n in sorted(names))
    src += "  return 0;\n}\n"
    c = tmp_path / "abi.c"
    c.write_text(src)
    exe = tmp_path / "abi"
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", f"-I{inc}", str(c),
                        "-o", str(exe), f"-L{lib}", "-lretina_pc", f"-Wl,-rpath,{lib}",
                        "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert len(names) > 40


def test_rec_index_macro_matches_host_decoder(tmp_path):
    """RTN_REC_INDEX (retina_pc.h) and pc._rec_index (the decoder the parity tests use) agree, and
    the index is a bijection of every (chunk, rank) pair onto [0, ceil(n/CF)*CF)."""
    import subprocess

    import numpy as np

    inc = Path(__file__).resolve().parent.parent / "include"
    src = ('#include "retina_pc.h"\n#include <stdio.h>\n#include <inttypes.h>\n'
           "int main(void) {\n  const uint32_t ns[] = {1u, 255u, 256u, 257u, 4097u, 33554432u};\n"
           "  for (int i = 0; i < 6; ++i) for (uint32_t c = 0; c < 3; ++c) for (uint32_t k = 0; k < RTN_CHUNK_FRAMES; k += 37)\n"
           '    printf("%u %u %u %" PRIu64 "\\n", ns[i], c, k, RTN_REC_INDEX(ns[i], c, k));\n  return 0;\n}\n')
    (tmp_path / "ri.c").write_text(src)
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{inc}", str(tmp_path / "ri.c"), "-o",
                        str(tmp_path / "ri")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(tmp_path / "ri")], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        n, c, k, want = map(int, line.split())
        frames = c * pc.CHUNK_FRAMES + np.arange(k + 1)  # the chunk's first k+1 frames, all forwarded
        assert pc._rec_index(frames, n)[-1] == want
    for n in (1, 700, 5000):
        cf = pc.CHUNK_FRAMES
        nch = (n + cf - 1) // cf
        frames = np.arange(nch * cf)  # every slot of every chunk forwarded
        idx = pc._rec_index(frames, n)
        assert np.array_equal(np.sort(idx), np.arange(nch * cf))


_RUST_C = {"u8": "uint8_t", "u16": "uint16_t", "u32": "uint32_t", "u64": "uint64_t", "i32": "int32_t",
           "usize": "size_t"}
_RUST_TO_HEADER = {"RtnBatch": "rtn_batch_t", "RtnPcOut": "rtn_pc_out_t", "RtnL4Ctx": "rtn_l4ctx_t",
                   "RtnConn": "rtn_conn_t", "RtnProgramInfo": "rtn_program_info_t",
                   "RtnFlowItem": "rtn_flow_item_t", "RtnFlowRule": "rtn_flow_rule_t",
                   "RtnStageSlab": "rtn_stage_slab_t"}


def _c_decl(t: str, f: str) -> str:
    """A Rust field type as a C declaration (scalars, raw pointers, [T; N] arrays)."""
    import re

    m = re.fullmatch(r"\[(\w+);\s*(\d+)\]", t)
    if m:
        inner = _RUST_C.get(m.group(1)) or f"twin_{m.group(1)}"
        return f"{inner} {f}[{m.group(2)}]"
    return f"{'void*' if t.startswith('*') else _RUST_C[t]} {f}"


def _rust_structs(text: str) -> dict:
    """`#[repr(C)] ... pub struct Name { pub field: type, ... }` blocks of INTEGRATION.md."""
    import re

    out = {}
    for m in re.finditer(r"#\[repr\(C\)\][^\n]*\n?\s*pub struct (\w+)\s*\{(.*?)\}", text, re.S):
        body = re.sub(r"//[^\n]*", "", m.group(2))
        fields = re.findall(r"pub (\w+):\s*([^,]+?)\s*(?:,|$)", body, re.M)
        if fields:
            out[m.group(1)] = [(f, t.strip()) for f, t in fields]
    return out


def test_integration_rust_structs_match_header(tmp_path):
    """The Rust #[repr(C)] structs documented in INTEGRATION.md §2 have the header's field order,
    offsets and sizes: a C twin of each is compiled next to the header and compared with
    _Static_assert (the documented binding had drifted)."""
    import subprocess

    text = (Path(__file__).resolve().parent.parent / "INTEGRATION.md").read_text()
    structs = _rust_structs(text)
    assert set(_RUST_TO_HEADER) <= set(structs), sorted(structs)
    src = '#include "retina_pc.h"\n#include "retina_hw.h"\n#include "retina_stage.h"\n#include <stddef.h>\n#include <stdint.h>\n'
    for name, cname in _RUST_TO_HEADER.items():
        src += f"typedef struct {{\n"
        for f, t in structs[name]:
            src += f"  {_c_decl(t, f)};\n"
        src += f"}} twin_{name};\n"
        src += f"_Static_assert(sizeof(twin_{name}) == sizeof({cname}), \"size of {name}\");\n"
        for f, _ in structs[name]:
            src += (f"_Static_assert(offsetof(twin_{name}, {f}) == offsetof({cname}, {f}), \"{name}.{f}\");\n"
                    f"_Static_assert(sizeof(((twin_{name}*)0)->{f}) == sizeof((({cname}*)0)->{f}), \"{name}.{f} size\");\n")
    src += "int main(void) { return 0; }\n"
    (tmp_path / "twin.c").write_text(src)
    inc = Path(__file__).resolve().parent.parent / "include"
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{inc}", str(tmp_path / "twin.c"), "-o",
                        str(tmp_path / "twin")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # every field of the C structs is in the twin (no field missing at the end either)
    import re

    hdr = (inc / "retina_pc.h").read_text() + (inc / "retina_hw.h").read_text() + (inc / "retina_stage.h").read_text()
    for name, cname in _RUST_TO_HEADER.items():
        body = re.search(r"typedef struct \w+ \{([^{}]*)\} " + cname + ";", hdr).group(1)
        cfields = re.findall(r"^\s*[\w\s\*]+?\b(\w+)(?:\[\w+\])?;", re.sub(r"/\*.*?\*/", "", body, flags=re.S), re.M)
        assert cfields == [f for f, _ in structs[name]], (name, cfields)


def test_integration_extern_fns_exist():
    """Every function the INTEGRATION.md bindings declare is declared by a header."""
    import re

    root = Path(__file__).resolve().parent.parent
    text = (root / "INTEGRATION.md").read_text()
    declared = set(re.findall(r"pub fn (rtn_\w+)\s*\(", text))
    hdrs = "".join(h.read_text() for h in HEADERS)
    missing = [f for f in declared if not re.search(r"\b" + f + r"\s*\(", hdrs)]
    assert declared and not missing, missing


def test_ext_needed_rule_matches_header(tmp_path):
    """The compact split layout depends on the caller and the kernel agreeing on which frames
    have an ext row: rtn_ext_needed (retina_pc.h, C) and pc.ext_needed (numpy, the packer the
    tests and the bench use) agree on every frame of the traces, adversarial and synthetic
    corpora, and the kernel's own rule is the same expression (GPU tests: compact layout)."""
    import subprocess

    import numpy as np

    from retina_amd import synth

    t = np.load(Path(__file__).resolve().parent / "golden" / "traces.npz")
    a = np.load(Path(__file__).resolve().parent / "golden" / "corpus_adversarial.npz")
    s3, d3 = synth.cfg3(4096, start=3)
    s4, d4 = synth.cfg4(4096, start=4)
    slab = np.concatenate([t["slab"], a["slab"], s3, s4]).reshape(-1, 128)
    dlen = np.concatenate([t["dlen"], a["dlen"], d3, d4])
    (tmp_path / "in.bin").write_bytes(np.ascontiguousarray(slab[:, :64]).tobytes())
    (tmp_path / "dl.bin").write_bytes(dlen.astype(np.uint16).tobytes())
    src = ('#include "retina_pc.h"\n#include <stdio.h>\nint main(int c, char** v) {\n'
           '  FILE* f = fopen(v[1], "rb"); FILE* g = fopen(v[2], "rb"); unsigned char h[64]; uint16_t d;\n'
           '  while (fread(h, 1, 64, f) == 64 && fread(&d, 2, 1, g) == 1) putchar(rtn_ext_needed(h, d) ? 49 : 48);\n'
           '  return 0;\n}\n')
    (tmp_path / "en.c").write_text(src)
    inc = Path(__file__).resolve().parent.parent / "include"
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{inc}", str(tmp_path / "en.c"), "-o",
                        str(tmp_path / "en")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(tmp_path / "en"), str(tmp_path / "in.bin"), str(tmp_path / "dl.bin")],
                         capture_output=True, text=True, check=True).stdout
    c_rule = np.frombuffer(out.encode(), np.uint8) == ord("1")
    assert len(c_rule) == len(dlen)
    py_rule = pc.ext_needed(slab, dlen)
    assert np.array_equal(c_rule, py_rule) and 0 < py_rule.sum() < len(dlen)
    head, ext, chunk = pc.split_slab(slab.reshape(-1), 128, dlen, compact=True)
    assert ext.size == 64 * int(py_rule.sum()) and chunk[0] == 0 and len(chunk) == (len(dlen) + pc.CHUNK_FRAMES - 1) // pc.CHUNK_FRAMES
    assert np.array_equal(ext.reshape(-1, 64), slab[py_rule, 64:128])


def test_deliver_callbacks_name_each_statement():
    """rtn_program_deliver_callback: statement k's callback is its subscription's (the C++ and
    Python Subscription mirrors read callback names through it); out of range gives 0."""
    from golden.filter_sets import SETS
    from oracle import filterlang

    for fset in ("payload", "cfg4", "quirks"):
        prog = pc.Program.from_spec(SETS[fset])
        subs, _ = prog.deliver_table()
        cbs = [s.callback for s in filterlang.load_spec(SETS[fset])]
        assert prog.deliver_callbacks() == [cbs[int(s)] for s in subs]
        assert pc.lib().rtn_program_deliver_callback(prog._h, prog.info["n_deliver_stmts"], None, 0) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("fset", ["cfg2", "cfg3", "cfg4"])
def test_chunks_per_wave_follow_occupancy(gpu, fset):
    """rtn_pc_run gives the compact split kernel 2 chunks per wave exactly when the runtime's
    occupancy (registers incl. AGPRs, and LDS) holds it below 4 waves per SIMD, and
    that occupancy agrees with the code object's own register and LDS counts."""
    import sys

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
    import kernel_resources

    prog = pc.Program.from_spec(SETS[fset])
    meta = {r["kernel"]: r for r in kernel_resources.report(prog.code_object())}
    ctx = pc.PacketContinue(prog, 0)
    names = ["rtn_pc_kernel", "rtn_pc_kernel_s64", "rtn_pc_kernel_split", "rtn_pc_kernel_splitc"]
    for layout, name in enumerate(names):
        for conn in (False, True):
            i = ctx.kernel_info(layout, conn)
            m = meta[name + ("_conn" if conn else "")]
            reg_bound = 512 // max(8, -(-m["vgpr"] // 8) * 8)
            lds_bound = (160 * 1024 // max(m["lds"], 1)) * (i["threads"] // 64) // 4
            assert i["lds_bytes"] == m["lds"], (name, conn, i, m)
            assert 1 <= i["waves_per_simd"] <= min(8, reg_bound, lds_bound), (name, conn, i, m)
            want = 2 if layout == 3 and i["waves_per_simd"] < 4 else 1
            assert i["chunks_per_wave"] == want, (name, conn, i)
