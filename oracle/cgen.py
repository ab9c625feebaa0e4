"""ORACLE (test infrastructure only): generate + build C for a subscription set.

The emitted `packet_continue` follows the control flow filtergen produces
(filtergen/src/packet_filter.rs:7-73, utils.rs:251-379): nested `parse_to::<X>` calls, the
first unary child of a node opens an `if`, later unary children are `else if`, binary children
chain per `if_else`, a node's own actions/callbacks come after its children (the root's before),
and the whole body is wrapped in the Ethernet parse iff the root has packet-level children.
The C is compiled with gcc -O3 -march=native into oracle/_build/ and driven through ctypes.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess
from pathlib import Path

import numpy as np

from .filterlang import Node, PacketTree, Pred
from .packet import statement_table

HERE = Path(__file__).resolve().parent
BUILD = HERE / "_build"

_ACC = {
    "ipv4": {
        "version": ("(F8(m,&ipv4,0) >> 4)", "u8"), "ihl": ("(F8(m,&ipv4,0) & 15u)", "u8"),
        "version_ihl": ("F8(m,&ipv4,0)", "u8"), "dscp": ("(F8(m,&ipv4,1) >> 2)", "u8"),
        "ecn": ("(F8(m,&ipv4,1) & 3u)", "u8"), "dscp_ecn": ("F8(m,&ipv4,1)", "u8"),
        "type_of_service": ("F8(m,&ipv4,1)", "u8"), "total_length": ("F16(m,&ipv4,2)", "u16"),
        "identification": ("F16(m,&ipv4,4)", "u16"), "flags_to_fragment_offset": ("F16(m,&ipv4,6)", "u16"),
        "flags": ("(F16(m,&ipv4,6) >> 13)", "u8"), "rf": ("((F16(m,&ipv4,6) & 0x8000u) != 0)", "bool"),
        "df": ("((F16(m,&ipv4,6) & 0x4000u) != 0)", "bool"), "mf": ("((F16(m,&ipv4,6) & 0x2000u) != 0)", "bool"),
        "fragment_offset": ("(F16(m,&ipv4,6) & 0x1fffu)", "u16"), "time_to_live": ("F8(m,&ipv4,8)", "u8"),
        "protocol": ("F8(m,&ipv4,9)", "u8"), "header_checksum": ("F16(m,&ipv4,10)", "u16"),
        "src_addr": ("F32(m,&ipv4,12)", "v4"), "dst_addr": ("F32(m,&ipv4,16)", "v4"),
    },
    "ipv6": {
        "version": ("(F32(m,&ipv6,0) >> 28)", "u8"), "dscp": ("((F32(m,&ipv6,0) >> 22) & 0x3fu)", "u8"),
        "ecn": ("((F32(m,&ipv6,0) >> 20) & 3u)", "u8"), "traffic_class": ("((F32(m,&ipv6,0) >> 20) & 0xffu)", "u8"),
        "flow_label": ("(F32(m,&ipv6,0) & 0xfffffu)", "u32"), "version_to_flow_label": ("F32(m,&ipv6,0)", "u32"),
        "payload_length": ("F16(m,&ipv6,4)", "u16"), "next_header": ("F8(m,&ipv6,6)", "u8"),
        "hop_limit": ("F8(m,&ipv6,7)", "u8"), "src_addr": ("be128(m->d + ipv6.off + 8)", "v6"),
        "dst_addr": ("be128(m->d + ipv6.off + 24)", "v6"),
    },
    "tcp": {
        "src_port": ("F16(m,&tcp,0)", "u16"), "dst_port": ("F16(m,&tcp,2)", "u16"),
        "seq_no": ("F32(m,&tcp,4)", "u32"), "ack_no": ("F32(m,&tcp,8)", "u32"),
        "data_offset": ("(F8(m,&tcp,12) >> 4)", "u8"), "reserved": ("(F8(m,&tcp,12) & 15u)", "u8"),
        "data_offset_to_ns": ("F8(m,&tcp,12)", "u8"), "flags": ("F8(m,&tcp,13)", "u8"),
        "window": ("F16(m,&tcp,14)", "u16"), "checksum": ("F16(m,&tcp,16)", "u16"),
        "urgent_pointer": ("F16(m,&tcp,18)", "u16"), "ns": ("(F8(m,&tcp,12) & 1u)", "u8"),
        "cwr": ("((F8(m,&tcp,13) >> 7) & 1u)", "u8"), "ece": ("((F8(m,&tcp,13) >> 6) & 1u)", "u8"),
        "urg": ("((F8(m,&tcp,13) >> 5) & 1u)", "u8"), "ack": ("((F8(m,&tcp,13) >> 4) & 1u)", "u8"),
        "psh": ("((F8(m,&tcp,13) >> 3) & 1u)", "u8"), "rst": ("((F8(m,&tcp,13) >> 2) & 1u)", "u8"),
        "syn": ("((F8(m,&tcp,13) >> 1) & 1u)", "u8"), "fin": ("(F8(m,&tcp,13) & 1u)", "u8"),
        "synack": ("((F8(m,&tcp,13) & 0x12u) != 0)", "u8"),
    },
    "udp": {
        "src_port": ("F16(m,&udp,0)", "u16"), "dst_port": ("F16(m,&udp,2)", "u16"),
        "length": ("F16(m,&udp,4)", "u16"), "checksum": ("F16(m,&udp,6)", "u16"),
    },
}
_MAX = {"u8": 0xFF, "u16": 0xFFFF, "u32": 0xFFFFFFFF}


class OracleTypeError(Exception):
    pass


def c_binary(p: Pred) -> str:
    if p.proto not in _ACC or p.field not in _ACC[p.proto]:
        raise OracleTypeError(f"no accessor {p.proto}.{p.field}")
    expr, ty = _ACC[p.proto][p.field]
    k, op = p.value.kind, p.op
    cmp = {"Eq": "==", "Ne": "!=", "Ge": ">=", "Le": "<=", "Gt": ">", "Lt": "<"}
    if k == "Int":
        if op not in cmp or ty not in _MAX or p.value.data[0] > _MAX[ty]:
            raise OracleTypeError(str(p))
        return f"({expr} {cmp[op]} {p.value.data[0]}ull)"
    if k == "IntRange":
        a, b = p.value.data
        if op != "In" or ty not in _MAX or b > _MAX[ty]:
            raise OracleTypeError(str(p))
        return f"({expr} >= {a}ull && {expr} <= {b}ull)"
    if k in ("Ipv4", "Ipv6"):
        if op not in ("Eq", "Ne", "In"):
            raise OracleTypeError(str(p))
        bits = 32 if k == "Ipv4" else 128
        if (k == "Ipv4" and ty == "v6") or (k == "Ipv6" and ty == "v4"):
            raise OracleTypeError(str(p))
        addr, plen = p.value.data
        x = f"((u128){expr})"
        lit = lambda v: f"(((u128){v >> 64}ull << 64) | (u128){v & ((1 << 64) - 1)}ull)"  # noqa: E731
        if plen == bits:
            e = f"({x} == {lit(addr)})"
        else:
            mask = ((1 << bits) - 1) ^ ((1 << (bits - plen)) - 1) if plen else 0
            e = f"(({x} & {lit(mask)}) == {lit(addr & mask)})"
        return f"(!{e})" if op == "Ne" else e
    raise OracleTypeError(str(p))


def generate_c(tree: PacketTree) -> tuple[str, int]:
    stmts = statement_table(tree)
    nd = (len(stmts) + 63) // 64
    lines: list[str] = []
    k = [0]

    def emit(s, d):
        lines.append("  " * d + s)

    def body(n: Node, d):
        if n.act:
            emit(f"act |= {n.act}u;", d)
        for _sid in sorted(n.deliver):
            idx = k[0]
            k[0] += 1
            bit = f"dm[{idx // 64}] |= 1ull << {idx % 64};"
            if stmts[idx][1] == "Payload":
                emit(f"if (payload_from_mbuf(m)) {{ {bit} }}", d)
            else:
                emit(bit, d)

    def kids(n: Node, d):
        unary = [c.pred.proto for c in n.kids if c.pred.unary]
        if unary:
            emit("hdr_t " + ", ".join(unary) + ";", d)
        first = True
        for c in n.kids:
            if c.pred.unary:
                kw = "if" if first else "else if"
                first = False
                emit(f"{kw} (parse_{c.pred.proto}(m, &{n.pred.proto}, &{c.pred.proto})) {{", d)
            else:
                kw = "else if" if c.if_else else "if"
                emit(f"{kw} {c_binary(c.pred)} {{", d)
            kids(c, d + 1)
            body(c, d + 1)
            emit("}", d)

    root = tree.root
    emit("static inline uint32_t packet_continue(const mbuf_t* m, uint64_t* dm) {", 0)
    emit("uint32_t act = 0; (void)dm;", 1)
    if root.kids:
        emit("hdr_t ethernet;", 1)
        emit("if (parse_ethernet(m, &ethernet)) {", 1)
        body(root, 2)
        kids(root, 2)
        emit("}", 1)
    else:
        body(root, 1)
    emit("return act;", 1)
    emit("}", 0)
    return "\n".join(lines) + "\n", nd


_BATCH = r"""
typedef unsigned __int128 u128;
#define ORACLE_ND (ND_WORDS > 0 ? ND_WORDS : 1)

/* per-frame outputs for parity checks */
void oracle_eval(const uint8_t* slab, uint64_t stride, const uint16_t* dlen, uint32_t n,
                 uint8_t* pc, uint8_t* fwd, l4ctx_t* rec, uint64_t* dm) {
  for (uint32_t i = 0; i < n; ++i) {
    mbuf_t m = {slab + (uint64_t)i * stride, dlen[i]};
    uint64_t* d = dm + (uint64_t)i * ORACLE_ND;
    for (int k = 0; k < ORACLE_ND; ++k) d[k] = 0;
    uint32_t act = packet_continue(&m, d);
    pc[i] = (act & 1u) != 0;
    fwd[i] = 0;
    if (pc[i]) fwd[i] = (uint8_t)l4context(&m, &rec[i]);
  }
}

/* CPU baseline: the per-mbuf loop of rx_core.rs:117-141 / offline.rs:67-82 over an array of
 * mbuf data pointers, continue_packet then (if PacketContinue) L4Context::new. */
typedef struct {
  const uint8_t* const* frames; const uint16_t* dlen; uint64_t lo, hi; uint32_t reps; int cpu;
  uint64_t pc, fwd, dlv, sum;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  if (j->cpu >= 0) {
    cpu_set_t s; CPU_ZERO(&s); CPU_SET(j->cpu, &s);
    pthread_setaffinity_np(pthread_self(), sizeof s, &s);
  }
  uint64_t pc = 0, fwd = 0, dlv = 0, sum = 0;
  for (uint32_t r = 0; r < j->reps; ++r) {
    for (uint64_t i = j->lo; i < j->hi; ++i) {
      mbuf_t m = {j->frames[i], j->dlen[i]};
      uint64_t d[ORACLE_ND] = {0};
      uint32_t act = packet_continue(&m, d);
      for (int k = 0; k < ORACLE_ND; ++k) dlv += __builtin_popcountll(d[k]);
      if (act & 1u) {
        ++pc;
        l4ctx_t c;
        if (l4context(&m, &c)) {
          ++fwd;
          sum += c.sport ^ (c.dport << 16) ^ c.length ^ c.seq ^ ((uint64_t)c.offset << 32);
        }
      }
    }
  }
  j->pc = pc; j->fwd = fwd; j->dlv = dlv; j->sum = sum;
  return 0;
}

int oracle_bench(const uint8_t* const* frames, const uint16_t* dlen, uint64_t n, uint32_t reps,
                 uint32_t nthreads, const int* cpus, uint64_t* out4) {
  pthread_t th[256];
  job_t jobs[256];
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  for (uint32_t t = 0; t < nthreads; ++t) {
    jobs[t].frames = frames; jobs[t].dlen = dlen; jobs[t].reps = reps;
    jobs[t].lo = n * t / nthreads; jobs[t].hi = n * (t + 1) / nthreads;
    jobs[t].cpu = cpus ? cpus[t] : -1;
    pthread_create(&th[t], 0, worker, &jobs[t]);
  }
  for (int k = 0; k < 4; ++k) out4[k] = 0;
  for (uint32_t t = 0; t < nthreads; ++t) {
    pthread_join(th[t], 0);
    out4[0] += jobs[t].pc; out4[1] += jobs[t].fwd; out4[2] += jobs[t].dlv; out4[3] ^= jobs[t].sum;
  }
  return 0;
}
"""

L4_DTYPE = np.dtype([("ver", "<u4"), ("proto", "<u4"), ("sport", "<u4"), ("dport", "<u4"), ("offset", "<u4"),
                     ("length", "<u4"), ("seq", "<u4"), ("ack", "<u4"), ("flags", "<u4"), ("src", "u1", 16),
                     ("dst", "u1", 16)])


def full_source(tree: PacketTree) -> tuple[str, int]:
    fn, nd = generate_c(tree)
    src = ("#define _GNU_SOURCE\n#include <pthread.h>\n#include <sched.h>\n"
           f'#include "{HERE / "pc_oracle_rt.h"}"\n'
           "typedef unsigned __int128 u128;\n"
           "static inline u128 be128(const uint8_t* p) { u128 v = 0; for (int k = 0; k < 16; ++k) v = (v << 8) | p[k]; return v; }\n"
           f"#define ND_WORDS {nd}\n" + fn + _BATCH)
    return src, nd


def _host_cpu() -> str:
    try:
        info = Path("/proc/cpuinfo").read_text()
        model = next((l for l in info.splitlines() if l.startswith("model name")), "")
        flags = next((l for l in info.splitlines() if l.startswith("flags")), "")
        return model + flags
    except OSError:
        return ""


class OracleLib:
    """A generated-and-compiled oracle for one subscription set."""

    def __init__(self, tree: PacketTree):
        self.tree = tree
        src, self.nd = full_source(tree)
        # -march=native: the build is keyed by the host CPU too, so a library built on another
        # machine (oracle/_build/ travels with the tree) is never loaded where it may not run
        h = hashlib.sha1((src + _host_cpu()).encode()).hexdigest()[:16]
        BUILD.mkdir(exist_ok=True)
        so = BUILD / f"pc_oracle_{h}.so"
        if not so.exists():
            # per-process temporaries: several ranks may build the same oracle at once
            c = BUILD / f"pc_oracle_{h}.{os.getpid()}.c"
            c.write_text(src)
            tmp = so.with_suffix(f".{os.getpid()}.tmp")
            cc = os.environ.get("CC", "gcc")
            subprocess.run([cc, "-O3", "-march=native", "-fPIC", "-shared", "-pthread", str(c), "-o", str(tmp)],
                           check=True, capture_output=True)
            os.replace(tmp, so)
            c.unlink(missing_ok=True)
        self.lib = C.CDLL(str(so))
        self.lib.oracle_eval.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p]
        self.lib.oracle_bench.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p,
                                          C.c_void_p]
        self.lib.oracle_bench.restype = C.c_int
        self.source = src

    def eval(self, slab: np.ndarray, stride: int, dlen: np.ndarray) -> dict:
        n = len(dlen)
        slab = np.ascontiguousarray(slab, np.uint8)
        dlen = np.ascontiguousarray(dlen, np.uint16)
        if stride < 128:
            assert int(dlen.max(initial=0)) <= stride, "oracle slab too narrow for these frames"
        pc = np.zeros(n, np.uint8)
        fwd = np.zeros(n, np.uint8)
        rec = np.zeros(n, L4_DTYPE)
        ndw = max(self.nd, 1)
        dm = np.zeros((n, ndw), np.uint64)
        self.lib.oracle_eval(slab.ctypes.data, stride, dlen.ctypes.data, n, pc.ctypes.data, fwd.ctypes.data,
                             rec.ctypes.data, dm.ctypes.data)
        return {"pc": pc.astype(bool), "fwd": fwd.astype(bool), "l4": rec, "dm": dm[:, :self.nd]}

    def bench(self, frame_ptrs: np.ndarray, dlen: np.ndarray, reps: int, cpus: list[int], pin: bool = True) -> np.ndarray:
        """len(cpus) threads on disjoint shards, each pinned to its CPU, or (pin=False) left to the
        scheduler."""
        out = np.zeros(4, np.uint64)
        cp = np.asarray(cpus, np.int32)
        self.lib.oracle_bench(frame_ptrs.ctypes.data, dlen.ctypes.data, len(dlen), reps, len(cpus),
                              cp.ctypes.data if pin else None, out.ctypes.data)
        return out
