"""Range runs in the straight-line filter (codegen.cpp RangeRun): sibling leaves that test one
header field for equality against constants in arithmetic progression, each delivering one
packet-level statement, are emitted as one subtract-and-compare whose offset picks the statement
bit. The oracle's generated C (oracle/cgen.py) keeps the per-predicate chain of
packet_filter.rs:31-73, so the GPU test below checks the lowering against the reference's
emission, and the CPU tests pin where the lowering does and does not apply."""
from __future__ import annotations

import re

import numpy as np
import pytest

import helpers
from retina_amd import pc, synth


def _subs():
    subs = []
    subs += [(f"ipv4.dst_addr = 192.168.{k}.0/24", ["ZcFrame"], f"net{k}") for k in range(70)]   # crosses dm word 0 -> 1
    subs += [(f"tcp.dst_port = {8000 + k}", ["Payload"], f"pay{k}") for k in range(10)]           # Payload statements
    subs += [(f"ipv4.src_addr = 255.255.255.{k}", ["ZcFrame", "FilterStr"], f"top{k}") for k in range(250, 256)]  # top of u32
    subs += [(f"udp.src_port = {p}", ["ZcFrame"], f"gap{p}") for p in (100, 101, 102, 104, 105, 106, 107)]  # a gap
    subs += [("udp.src_port = 103", ["ConnRecord"], "conn103")]             # a connection-level sub inside the gap
    subs += [("ipv4.dst_addr = 10.1.0.0/16 and tcp.port = 22", ["ZcFrame"], "ssh10")]
    subs += [(f"ipv4.dst_addr = 10.{k}.0.0/16", ["ZcFrame"], f"ten{k}") for k in range(6)]       # 10.1/16 has a child
    return subs


SPEC = synth._toml(_subs())


def test_range_runs_emitted_where_they_apply():
    prog = pc.Program.from_spec(SPEC)
    body = prog.source.split("void rtn_filter(")[1].split("\n}\n")[0]
    spans = sorted(int(s) for s in re.findall(r"\(unsigned long long\)q\d+ < (\d+)ull", body))
    # 192.168.k/24: 64 in word 0 and 6 in word 1; the 10.k/16 siblings split by 10.1/16 (it has a
    # child): 10.2-10.5 is a run, 10.0 alone is not; 255.255.255.250-255 (/32); under both ipv4
    # and ipv6: tcp.dst_port 8000-8009 and udp.src_port 104-107 (100-102 before the gap are too few)
    assert spans == sorted([64 << 8, 6 << 8, 4 << 16, 6, 10, 4, 10, 4]), spans
    assert body.count("RTN_DM_SETV(dm, 1, 0 + (q") == 1          # the word-1 remainder starts at bit 0
    assert "v.payload_ok" in body


def test_range_runs_not_applied_to_single_or_unequal_tests():
    subs = [(f"tcp.dst_port = {p}", ["ZcFrame"], f"p{p}") for p in (80, 82, 84, 86)]         # step 2 on a /0 shift
    subs += [(f"ipv4.dst_addr = 10.{k}.0.0/{16 if k % 2 else 24}", ["ZcFrame"], f"m{k}") for k in range(6)]  # mixed masks
    subs += [(f"tcp.src_port != {p}", ["ZcFrame"], f"n{p}") for p in range(5000, 5006)]    # not equality
    body = pc.Program.from_spec(synth._toml(subs)).source.split("void rtn_filter(")[1].split("\n}\n")[0]
    assert "(unsigned long long)q" not in body


def _frames(n: int, seed: int):
    rng = np.random.default_rng(seed)
    frames = []
    for _ in range(n):
        v6 = bool(rng.random() < 0.1)
        proto = 6 if rng.random() < 0.55 else 17
        r = rng.random()
        dst = (0xC0A80000 | int(rng.integers(0, 80)) << 8 | int(rng.integers(0, 256))) if r < 0.4 else \
              (0x0A000000 | int(rng.integers(0, 8)) << 16 | int(rng.integers(0, 1 << 16))) if r < 0.7 else \
              int(rng.integers(0, 1 << 32))
        src = (0xFFFFFF00 | int(rng.integers(240, 256))) if rng.random() < 0.3 else int(rng.integers(0, 1 << 32))
        if v6:
            src, dst = src << 96 | 7, dst << 96 | 9
        sp = int(rng.choice([int(rng.integers(98, 110)), 22, int(rng.integers(1, 65536))]))
        dp = int(rng.choice([int(rng.integers(7995, 8015)), 22, int(rng.integers(1, 65536))]))
        frames.append(helpers.build_frame(v6, src, dst, sp, dp, proto, 0x18, payload=bytes(int(rng.integers(0, 3)))))
    return pc.pack_frames(frames, 128)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, "compact"])
def test_range_runs_match_oracle(split, gpu):
    slab, dlen = _frames(20000, 17)
    helpers.assert_same(helpers.gpu_run(SPEC, slab, 128, dlen, split=split),
                        helpers.oracle_run(SPEC, slab, 128, dlen), f"range runs/{split}")
