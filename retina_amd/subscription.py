"""Host-side mirror of Retina's `Subscription` for the packet stage (core/src/subscription/mod.rs),
over the C ABI (retina_pc.h through retina_amd.pc). The names follow the reference:

  Subscription(spec)            Subscription::new(filter()) (subscription/mod.rs:81-92): the
                                #[subscription] spec compiled by filtergen (rtn_program_compile)
                                and loaded on one GPU (rtn_pc_create); one per RX core, like the
                                reference's per-lcore use
  run(batch)                    one launch for a whole burst: continue_packet per mbuf
                                (subscription/mod.rs:125-127) plus the PacketContinue gate and
                                L4Context::new of process_packet (:94-116)
  Burst.continue_packet(i)      the Actions (data bits) continue_packet returned for frame i
  Burst.process_packets()       the frames process_packet hands to conn_tracker.process, in
                                frame order, each with its L4Context (pdu.rs:66-84)
  Burst.packet_callbacks()      the ZcFrame / Payload callbacks the generated packet_continue ran
                                inline (filtergen/src/data.rs:299-331), in call order
  stats                         the thread-local counters of core/src/stats/mod.rs:9-27 that
                                rx_core.rs:127-139 and process_packet update per frame

There is no CPU path: every result comes from the gfx950 kernel (pc.PacketContinue raises if
the library or the GPU is missing). Errors follow the C ABI: pc.FilterError for a spec filtergen
would refuse, pc.RetinaError otherwise.
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass

import numpy as np

from . import pc

PACKET_CONTINUE = 1  # ActionData::PacketContinue (core/src/filter/actions.rs:17-76)

STAT_NAMES = ("TOTAL_PKT", "TOTAL_BYTE", "IGNORED_BY_PACKET_FILTER_PKT", "IGNORED_BY_PACKET_FILTER_BYTE",
              "TCP_PKT", "TCP_BYTE", "UDP_PKT", "UDP_BYTE")


@dataclass(frozen=True)
class L4Context:
    """conntrack/pdu.rs:66-84 (src/dst are SocketAddr: an (ip, port) pair here)."""
    src: tuple
    dst: tuple
    proto: int
    offset: int
    length: int
    seq_no: int
    ack_no: int
    flags: int

    def five_tuple(self) -> dict:
        """FiveTuple::from_ctxt (conn_id.rs:32-38) in its serde form (SocketAddr Display)."""
        def sa(ip, port):
            return f"[{ip}]:{port}" if ip.version == 6 else f"{ip}:{port}"
        return {"orig": sa(*self.src), "resp": sa(*self.dst), "proto": self.proto}


class Burst:
    """The results of one Subscription.run over a burst of n frames (host copies)."""

    def __init__(self, sub: "Subscription", out: pc.PCOutputs, core_id: int):
        self.core_id = core_id
        self._d = out.decode()
        self.n = out.n
        self._stmts = sub.callback_sites
        self.stats = out.stats_host() if out.counters is not None else None

    def continue_packet(self, i: int) -> int:
        """Actions.data of frame i (PacketContinue or nothing, at this layer: datatypes.rs:618-638)."""
        return PACKET_CONTINUE if self._d["pc"][i] else 0

    def process_packets(self):
        """(frame index, L4Context) of every frame that reaches conn_tracker.process, in order."""
        l4 = self._d["l4"]
        a6 = self._d.get("addr6")
        for j in range(len(l4)):
            r = l4[j]
            if r["ver"] == 6:
                s = ipaddress.IPv6Address(bytes(a6[j, :16]))
                d = ipaddress.IPv6Address(bytes(a6[j, 16:]))
            else:
                s, d = ipaddress.IPv4Address(int(r["src_ip4"])), ipaddress.IPv4Address(int(r["dst_ip4"]))
            yield int(r["pkt_idx"]), L4Context((s, int(r["sport"])), (d, int(r["dport"])), int(r["proto"]),
                                               int(r["offset"]), int(r["length"]), int(r["seq_no"]),
                                               int(r["ack_no"]), int(r["flags"]))

    def packet_callbacks(self):
        """(frame index, [(subscription index, callback, "ZcFrame" | "Payload"), ...]) for every
        frame with packet-level callbacks, frames in order, callbacks in the order the generated
        code calls them."""
        if "dlv" not in self._d:
            return
        for row in self._d["dlv"]:
            calls = []
            for k, site in enumerate(self._stmts):
                if (int(row[1 + k // 64]) >> (k % 64)) & 1:
                    calls.append(site)
            yield int(row[0]), calls


class Subscription:
    """One compiled subscription set loaded on one GPU (see the module docstring)."""

    def __init__(self, spec: str, device: int = 0):
        self.program = pc.Program.from_spec(spec)
        self.ctx = pc.PacketContinue(self.program, device)
        self.device = device
        self.stats = {k: 0 for k in STAT_NAMES}
        subs, pay = self.program.deliver_table()
        names = self.program.deliver_callbacks()
        self.callback_sites = [(int(s), cb, "Payload" if p else "ZcFrame") for s, p, cb in zip(subs, pay, names)]

    def run(self, slab, stride: int, data_len, n: int | None = None, ext=None, stream=None,
            core_id: int = 0) -> Burst:
        """One burst through the packet stage; `slab`/`data_len`/`ext` are device tensors in the
        layout of include/retina_pc.h. Synchronizes `stream` and accumulates `stats`."""
        import torch

        n = int(data_len.numel()) if n is None else n
        out = self.ctx.alloc_outputs(max(n, 1), addr6=True, counters=True)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.ctx.run(slab, stride, data_len, n, out, stream=s, core_id=core_id, ext=ext)
        s.synchronize()
        b = Burst(self, out, core_id)
        st = out.counters_host()[3]
        if st:
            raise pc.RetinaError(-22, f"frames whose headers do not fit their slots (status {int(st):#x})")
        for k, v in b.stats.items():
            self.stats[k] += v
        return b

