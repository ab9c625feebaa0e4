"""The C++ offline runtime (examples/rtn_offline.cpp, built as retina_amd/_lib/rtn_offline): a
capture goes through ingest, the packet filter, the connection stage and the connection table
in batches, all through the C ABI, and its per-frame output matches the oracle: the forwarded
frames in capture order with their 5-tuples, and their connection outcomes batch by batch
(oracle/conn.py TableModel), with the offline runtime's mtu rule (offline.rs:68-70)."""
from __future__ import annotations

import json
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from oracle import conn as oconn
from oracle import filterlang
from oracle import packet
from retina_amd import pc

EXE = Path(__file__).resolve().parent.parent / "retina_amd" / "_lib" / "rtn_offline"
SPEC = SETS["port_count"]


def _write_pcap(path: Path, frames: list[tuple[bytes, int]]) -> None:
    b = bytearray(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
    for t, (data, orig) in enumerate(frames):
        b += struct.pack("<IIII", t, 0, len(data), orig) + data
    path.write_bytes(bytes(b))


def test_offline_runtime_is_built():
    assert EXE.exists(), "build() builds examples/rtn_offline.cpp"


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["compact", "mono", "gpu"])
def test_offline_runtime_vs_oracle(gpu, tmp_path, layout):
    rng = np.random.default_rng(3)
    pool = helpers.flow_pool(rng, 700)
    frames = helpers.flow_frames(rng, pool, 9000, p_syn=0.3)
    caps = []
    for j, f in enumerate(frames):
        orig = len(f)
        if j % 97 == 5:
            orig = 1600          # longer than --mtu 1500 on the wire: skipped (offline.rs:68)
        if j % 89 == 7:
            f = f[:30]           # truncated capture: parse fails, not forwarded
        caps.append((f, orig))
    cap = tmp_path / "flows.pcap"
    _write_pcap(cap, caps)
    spec = tmp_path / "spec.toml"
    spec.write_text(SPEC)
    dump = tmp_path / "dump.txt"
    batch = 2048
    r = subprocess.run([str(EXE), str(spec), str(cap), "--batch", str(batch), "--mtu", "1500", "--ct-log2", "16",
                        "--dump", str(dump), "--layout", layout, "--window", str(1 << 24)],
                       capture_output=True, text=True, timeout=120)
    # (the window holds the whole capture, so the GPU walk's batches are full like the host's:
    # the connection outcomes below are per batch; window seams: tests/test_ingest_gpu.py)
    assert r.returncode == 0, r.stderr
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["layout"] == layout

    kept = [f for f, orig in caps if orig <= 1500]
    assert summary["frames"] == len(kept) and summary["skipped_mtu"] == len(caps) - len(kept)
    slab, dlen = pc.pack_frames(kept, 128)
    ora = helpers.oracle_run(SPEC, slab, 128, dlen)
    idx = np.nonzero(ora["fwd"])[0]
    assert summary["forwarded"] == len(idx) and summary["packet_continue"] == int(ora["pc"].sum())

    prog = pc.Program.from_spec(SPEC)
    subs = helpers.subs_from_spec(SPEC)
    pf = oconn.PacketFilter(filterlang.ConnTree(subs).to_json(), subs)
    model = oconn.TableModel()
    exp_status = []
    for b0 in range(0, len(kept), batch):
        mf = []
        for i in idx[(idx >= b0) & (idx < b0 + batch)]:
            f = kept[i]
            ctx = packet.l4context(f + bytes(64), len(f))
            data, term, _ = pf.evaluate(f, len(f))
            mf.append((oconn.conn_key(ctx), oconn.creates(ctx), data == 0 and term == 0))
        exp_status += [s for _, s in model.process(mf)]

    lines = dump.read_text().split()
    got = np.array(lines, dtype=object).reshape(-1, 8)
    assert len(got) == len(idx)
    assert [int(x) for x in got[:, 0]] == idx.tolist()
    rec = ora["rec"]
    for j in range(len(idx)):
        v6 = rec["ver"][j] == 6
        ip = lambda a: a.tobytes().hex() if v6 else a[:4].tobytes().hex()  # noqa: E731
        assert int(got[j, 1]) == rec["proto"][j]
        assert got[j, 2] == ip(rec["src"][j]) and int(got[j, 3]) == rec["sport"][j]
        assert got[j, 4] == ip(rec["dst"][j]) and int(got[j, 5]) == rec["dport"][j]
    assert [int(x) for x in got[:, 6]] == exp_status
    assert summary["ct"]["live"] == len(model.present)
