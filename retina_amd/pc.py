"""ctypes binding of the C ABI in include/retina_pc.h (libretina_pc.so, built in-tree).

This is the host-side mirror used by tests, bench.py and the Python Subscription shim; the
product path is the HIP kernel behind rtn_pc_run. There is no CPU fallback: if the shared
library or a GPU is missing, these calls raise.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path

import numpy as np

_LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libretina_pc.so"
_lib = None

RTN_OK = 0


class RetinaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class FilterError(RetinaError):
    """The subscription/filter would be rejected by the reference's filtergen."""


class _Batch(C.Structure):
    _fields_ = [("slab", C.c_void_p), ("stride", C.c_uint64), ("data_len", C.c_void_p),
                ("n", C.c_uint32), ("core_id", C.c_uint32), ("ext", C.c_void_p), ("flags", C.c_uint32),
                ("ext_rows", C.c_uint32), ("ext_chunk", C.c_void_p)]


BATCH_DL_LE64 = 1          # RTN_BATCH_DL_LE64
BATCH_EXT_COMPACT = 2      # RTN_BATCH_EXT_COMPACT
STATUS_EXT_ROWS = 4        # RTN_STATUS_EXT_ROWS
STATUS_HDR_PAST_SLOT = 1   # RTN_STATUS_HDR_PAST_SLOT
STATUS_DL_PAST_SLOT = 2    # RTN_STATUS_DL_PAST_SLOT
COUNTERS_BYTES = 64        # RTN_COUNTERS_BYTES
MAX_FRAMES = 1 << 31       # RTN_MAX_FRAMES


class _Out(C.Structure):
    _fields_ = [("pc_bitmap", C.c_void_p), ("fwd_bitmap", C.c_void_p), ("l4", C.c_void_p),
                ("addr6", C.c_void_p), ("dlv_bitmap", C.c_void_p), ("dlv_records", C.c_void_p),
                ("counters", C.c_void_p), ("conn", C.c_void_p), ("conn_dlv", C.c_void_p), ("seqack", C.c_void_p)]


class _PcapStats(C.Structure):
    _fields_ = [("frames", C.c_uint64), ("skipped_mtu", C.c_uint64), ("packed", C.c_uint64), ("bytes", C.c_uint64)]


class _StageSlab(C.Structure):
    _fields_ = [("head", C.c_void_p), ("ext", C.c_void_p), ("ext_chunk", C.c_void_p), ("data_len", C.c_void_p),
                ("cap", C.c_uint32), ("ext_cap", C.c_uint32)]


class _Info(C.Structure):
    _fields_ = [("n_subscriptions", C.c_uint32), ("n_deliver_stmts", C.c_uint32),
                ("deliver_words", C.c_uint32), ("tree_size", C.c_uint32), ("n_conn_stmts", C.c_uint32),
                ("conn_words", C.c_uint32), ("conn_tree_size", C.c_uint32), ("n_pd_stmts", C.c_uint32),
                ("n_pd_facts", C.c_uint32), ("pd_tree_size", C.c_uint32)]


class _FlowItem(C.Structure):
    _fields_ = [("item_type", C.c_uint32), ("size", C.c_uint32), ("spec", C.c_uint8 * 40), ("mask", C.c_uint8 * 40)]


class _FlowRule(C.Structure):
    _fields_ = [("group", C.c_uint32), ("priority", C.c_uint32), ("action", C.c_uint32),
                ("jump_group", C.c_uint32), ("pattern", C.c_uint32), ("n_items", C.c_uint32),
                ("items", _FlowItem * 4)]


_FLOW_VALIDATE = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.POINTER(_FlowRule))

EXPORTS = {
    "rtn_last_error": (C.c_char_p, []),
    "rtn_program_compile": (C.c_int32, [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "rtn_program_compile_filter": (C.c_int32, [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "rtn_program_info": (C.c_int32, [C.c_void_p, C.POINTER(_Info)]),
    "rtn_program_tree": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_rust": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_source": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_deliver_table": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "rtn_program_deliver_callback": (C.c_size_t, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]),
    "rtn_program_hw_filter": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_conn_tree": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_conn_rust": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_conn_table": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "rtn_program_tree_json": (C.c_size_t, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]),
    "rtn_program_pd_json": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_pd_rust": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "rtn_program_code_object": (C.c_int32, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "rtn_program_destroy": (None, [C.c_void_p]),
    "rtn_pc_create": (C.c_int32, [C.c_char_p, C.c_size_t, C.c_int, C.POINTER(C.c_void_p)]),
    "rtn_pc_create_from_program": (C.c_int32, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "rtn_pc_run": (C.c_int32, [C.c_void_p, C.POINTER(_Batch), C.POINTER(_Out), C.c_void_p]),
    "rtn_pc_set_grid": (C.c_int32, [C.c_void_p, C.c_uint32]),
    "rtn_pc_kernel_info": (C.c_int32, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]),
    "rtn_pc_take_status": (C.c_int32, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "rtn_pc_index": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rtn_pc_destroy": (C.c_int32, [C.c_void_p]),
    "rtn_out_bitmap_bytes": (C.c_size_t, [C.c_uint32]),
    "rtn_out_l4_bytes": (C.c_size_t, [C.c_uint32]),
    "rtn_out_addr6_bytes": (C.c_size_t, [C.c_uint32]),
    "rtn_out_dlv_bytes": (C.c_size_t, [C.c_uint32, C.c_uint32]),
    "rtn_out_conn_bytes": (C.c_size_t, [C.c_uint32]),
    "rtn_out_conn_dlv_bytes": (C.c_size_t, [C.c_uint32, C.c_uint32]),
    "rtn_out_seqack_bytes": (C.c_size_t, [C.c_uint32]),
    # include/retina_ct.h
    "rtn_ct_create": (C.c_int32, [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p)]),
    "rtn_ct_destroy": (C.c_int32, [C.c_void_p]),
    "rtn_ct_process": (C.c_int32, [C.c_void_p, C.POINTER(_Out), C.c_uint32, C.c_void_p, C.c_void_p]),
    "rtn_ct_remove": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "rtn_ct_rebuild": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "rtn_ct_stats": (C.c_int32, [C.c_void_p, C.c_void_p]),
    "rtn_ct_table": (C.c_void_p, [C.c_void_p]),
    "rtn_out_ct_bytes": (C.c_size_t, [C.c_uint32]),
    # include/retina_pd.h
    "rtn_pd_run": (C.c_int32, [C.c_void_p, C.POINTER(_Out), C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                               C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rtn_out_pd_counts_bytes": (C.c_size_t, [C.c_uint32, C.c_uint32]),
    "rtn_program_pd_replay": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.POINTER(C.c_uint32)]),
    # include/retina_hw.h
    "rtn_hw_rules": (C.c_int32, [C.c_char_p, _FLOW_VALIDATE, C.c_void_p, C.POINTER(_FlowRule), C.c_uint32,
                                 C.POINTER(C.c_uint32)]),
    "rtn_program_hw_rules": (C.c_int32, [C.c_void_p, _FLOW_VALIDATE, C.c_void_p, C.POINTER(_FlowRule),
                                         C.c_uint32, C.POINTER(C.c_uint32)]),
    "rtn_hw_patterns": (C.c_size_t, [C.c_char_p, _FLOW_VALIDATE, C.c_void_p, C.c_char_p, C.c_size_t]),
    # include/retina_ingest.h
    "rtn_pcap_open": (C.c_int32, [C.c_char_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    "rtn_pcap_next_batch": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                        C.POINTER(C.c_uint32)]),
    "rtn_pcap_next_batch_split": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                              C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "rtn_pcap_stats": (C.c_int32, [C.c_void_p, C.POINTER(_PcapStats)]),
    "rtn_pcap_next_batch_gpu": (C.c_int32, [C.c_void_p, C.c_int, C.POINTER(_StageSlab), C.POINTER(C.c_uint32),
                                            C.c_void_p]),
    "rtn_pcap_gpu_window": (C.c_int32, [C.c_void_p, C.c_uint64]),
    "rtn_pcap_rewind": (C.c_int32, [C.c_void_p]),
    "rtn_pcap_close": (None, [C.c_void_p]),
    # include/retina_stage.h
    "rtn_stager_create": (C.c_int32, [C.c_uint32, C.c_void_p, C.POINTER(C.c_void_p)]),
    "rtn_stager_destroy": (None, [C.c_void_p]),
    "rtn_stage_mbufs": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                    C.POINTER(C.c_uint32), C.POINTER(C.c_uint16)]),
    "rtn_mbuf_pool_register": (C.c_int32, [C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_void_p)]),
    "rtn_mbuf_pool_destroy": (C.c_int32, [C.c_void_p]),
    "rtn_stage_gather_ext_rows": (C.c_uint32, [C.c_uint32]),
    "rtn_stage_gather": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                     C.c_void_p]),
    "rtn_mbuf_pool_take_status": (C.c_int32, [C.c_void_p, C.POINTER(C.c_uint32)]),
}


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise RetinaError(-2, f"{_LIB_PATH} not built (run __graft_entry__.build())")
        L = C.CDLL(str(_LIB_PATH))
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != RTN_OK:
        msg = lib().rtn_last_error().decode(errors="replace")
        raise (FilterError if rc == -74 else RetinaError)(rc, msg)


def _text(fn, h) -> str:
    n = fn(h, None, 0)
    buf = C.create_string_buffer(n + 1)
    fn(h, buf, n + 1)
    return buf.value.decode()


# rtn_l4ctx_t (include/retina_pc.h), 16 bytes: w0/w1 = IPv4 addresses, or an IPv6 record's source
# address bytes 0..7 (the rest of its addresses in addr6, 24 B); TCP seq/ack in the seqack side
# stream
L4_DTYPE = np.dtype([("w0", "<u4"), ("w1", "<u4"), ("ports", "<u4"), ("meta", "<u4")])
# what PCOutputs.decode() returns per forwarded frame: the record's fields unpacked, plus the
# frame index its position implies
L4_DECODED = np.dtype([("pkt_idx", "<u8"), ("src_ip4", "<u4"), ("dst_ip4", "<u4"), ("sport", "<u4"),
                       ("dport", "<u4"), ("seq_no", "<u4"), ("ack_no", "<u4"), ("offset", "<u4"),
                       ("length", "<u4"), ("proto", "<u4"), ("flags", "<u4"), ("ver", "<u4")])


def decode_l4(raw: np.ndarray, frames: np.ndarray, seqack: np.ndarray | None = None, n: int | None = None) -> np.ndarray:
    """Unpack rtn_l4ctx_t records (the RTN_L4_* accessors of retina_pc.h) of the forwarded frames
    `frames` (ascending); `seqack` is the run's seqack side stream (uint64) for the TCP records'
    seq/ack (left 0 when None), n the batch size. IPv6 addresses: PCOutputs.decode()."""
    out = np.zeros(len(raw), L4_DECODED)
    out["pkt_idx"] = frames
    m = raw["meta"]
    v6, udp = (m & 0x80) != 0, (m & 0x40) != 0
    out["src_ip4"] = np.where(v6, 0, raw["w0"])
    out["dst_ip4"] = np.where(v6, 0, raw["w1"])
    tcp = ~udp
    if seqack is not None and tcp.any():
        t = seqack[_rec_index(np.asarray(frames, np.int64)[tcp], n)]
        out["seq_no"][tcp] = (t & 0xFFFFFFFF).astype(np.uint32)
        out["ack_no"][tcp] = (t >> 32).astype(np.uint32)
    out["sport"] = raw["ports"] & 0xFFFF
    out["dport"] = raw["ports"] >> 16
    out["offset"] = ((m & 0x3F) << 2) | 2
    out["proto"] = np.where(m & 0x40, 17, 6)
    out["ver"] = np.where(m & 0x80, 6, 4)
    out["flags"] = (m >> 8) & 0xFF
    out["length"] = m >> 16
    return out


class Program:
    """A compiled subscription set (the output of filtergen for the packet stage)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @classmethod
    def from_spec(cls, toml_text: str) -> "Program":
        h = C.c_void_p()
        b = toml_text.encode()
        _check(lib().rtn_program_compile(b, len(b), C.byref(h)))
        return cls(h.value)

    @classmethod
    def from_filter(cls, filter_str: str, datatypes=("ConnRecord",), callback: str = "cb") -> "Program":
        h = C.c_void_p()
        _check(lib().rtn_program_compile_filter(filter_str.encode(), ",".join(datatypes).encode(),
                                                callback.encode(), C.byref(h)))
        return cls(h.value)

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rtn_program_destroy(self._h)
            self._h = C.c_void_p()

    @property
    def info(self) -> dict:
        i = _Info()
        _check(lib().rtn_program_info(self._h, C.byref(i)))
        return {f: getattr(i, f) for f, _ in _Info._fields_}

    @property
    def tree(self) -> str:
        return _text(lib().rtn_program_tree, self._h)

    @property
    def rust(self) -> str:
        return _text(lib().rtn_program_rust, self._h)

    @property
    def source(self) -> str:
        return _text(lib().rtn_program_source, self._h)

    def deliver_callbacks(self) -> list[str]:
        """Callback name of every packet-level statement, in statement order."""
        out = []
        for k in range(self.info["n_deliver_stmts"]):
            m = lib().rtn_program_deliver_callback(self._h, k, None, 0)
            buf = C.create_string_buffer(m + 1)
            lib().rtn_program_deliver_callback(self._h, k, buf, m + 1)
            out.append(buf.value.decode())
        return out

    def deliver_table(self) -> tuple[np.ndarray, np.ndarray]:
        n = self.info["n_deliver_stmts"]
        subs = np.zeros(max(n, 1), np.uint32)
        pay = np.zeros(max(n, 1), np.uint8)
        _check(lib().rtn_program_deliver_table(self._h, subs.ctypes.data, pay.ctypes.data, max(n, 1)))
        return subs[:n], pay[:n]

    @property
    def hw_filter(self) -> str:
        """The NIC keep/drop filter string (FilterFactory.filter_str)."""
        return _text(lib().rtn_program_hw_filter, self._h)

    @property
    def conn_tree(self) -> str:
        """The collapsed FilterLayer::Packet tree (the first-packet `packet_filter`)."""
        return _text(lib().rtn_program_conn_tree, self._h)

    @property
    def conn_rust(self) -> str:
        return _text(lib().rtn_program_conn_rust, self._h)

    def conn_table(self) -> tuple[np.ndarray, np.ndarray]:
        """First-packet statement k -> (subscription index, RTN_STMT_* kind)."""
        n = self.info["n_conn_stmts"]
        subs = np.zeros(max(n, 1), np.uint32)
        kinds = np.zeros(max(n, 1), np.uint8)
        _check(lib().rtn_program_conn_table(self._h, subs.ctypes.data, kinds.ctypes.data, max(n, 1)))
        return subs[:n], kinds[:n]

    @property
    def pd_rust(self) -> str:
        """The generated packet_deliver as filtergen would emit it (FilterLayer::PacketDeliver)."""
        return _text(lib().rtn_program_pd_rust, self._h)

    def pd_program(self) -> dict:
        """The packet_deliver filter's facts and statements (include/retina_pd.h)."""
        import json

        return json.loads(_text(lib().rtn_program_pd_json, self._h))

    def pd_replay(self, counts_row, facts_row) -> list[int]:
        """rtn_program_pd_replay: one frame's callback sequence from its counts and facts."""
        c = np.ascontiguousarray(counts_row, np.uint32)
        f = np.ascontiguousarray(facts_row, np.uint32)
        n = C.c_uint32()
        lib().rtn_program_pd_replay(self._h, c.ctypes.data, f.ctypes.data if f.size else None, None, 0, C.byref(n))
        out = np.zeros(max(n.value, 1), np.uint32)
        _check(lib().rtn_program_pd_replay(self._h, c.ctypes.data, f.ctypes.data if f.size else None,
                                           out.ctypes.data, n.value, C.byref(n)))
        return out[:n.value].tolist()

    def tree_json(self, layer: int) -> dict:
        """Collapsed tree of layer 0 (PacketContinue), 1 (Packet) or 2 (PacketDeliver) as nested dicts."""
        import json

        L = lib()
        n = L.rtn_program_tree_json(self._h, layer, None, 0)
        buf = C.create_string_buffer(n + 1)
        L.rtn_program_tree_json(self._h, layer, buf, n + 1)
        return json.loads(buf.value.decode())

    def code_object(self) -> bytes:
        p = C.c_void_p()
        n = C.c_size_t()
        _check(lib().rtn_program_code_object(self._h, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value)


@dataclass
class PCOutputs:
    """Device-side output buffers (torch tensors) of one rtn_pc_run."""
    n: int
    pc_bitmap: object
    fwd_bitmap: object
    l4: object
    addr6: object
    dlv_bitmap: object
    dlv_records: object
    counters: object
    deliver_words: int
    conn: object = None
    conn_dlv: object = None
    conn_words: int = 0
    seqack: object = None

    def counters_host(self) -> np.ndarray:
        """[pc, fwd, dlv, status] (uint32)."""
        return self.counters.cpu().numpy().view(np.uint32)[:4]

    def stats_host(self) -> dict:
        """The counters block under the reference's stats names (core/src/stats/mod.rs:9-27), as
        rx_core.rs:127-139 and Subscription::process_packet (subscription/mod.rs:102-111) would
        have counted this batch."""
        w = self.counters.cpu().numpy().view(np.uint32)
        q = w.view(np.uint64)
        return {"TOTAL_PKT": int(self.n), "TOTAL_BYTE": int(q[2]),
                "IGNORED_BY_PACKET_FILTER_PKT": int(self.n) - int(w[0]), "IGNORED_BY_PACKET_FILTER_BYTE": int(q[3]),
                "TCP_PKT": int(w[8]), "UDP_PKT": int(w[9]), "TCP_BYTE": int(q[5]), "UDP_BYTE": int(q[6])}

    def byte_counters_host(self) -> tuple[int, int]:
        """(data_len sum of all frames, data_len sum of the frames not accepted)."""
        b = self.counters.cpu().numpy().view(np.uint64)
        return int(b[2]), int(b[3])

    def decode(self) -> dict:
        """Bring results to the host in frame order (numpy)."""
        n = self.n
        pc_bm = self.pc_bitmap.cpu().numpy().view(np.uint64)
        fwd_bm = self.fwd_bitmap.cpu().numpy().view(np.uint64)
        pc = np.unpackbits(pc_bm.view(np.uint8), bitorder="little")[:n].astype(bool)
        fwd = np.unpackbits(fwd_bm.view(np.uint8), bitorder="little")[:n].astype(bool)
        recs_all = self.l4.cpu().numpy().view(L4_DTYPE)
        idx = _fwd_index(fwd_bm, n)
        t4 = self.seqack.cpu().numpy().view(np.uint64) if self.seqack is not None else None
        recs = decode_l4(recs_all[idx], np.nonzero(fwd)[0], t4, n)
        out = {"pc": pc, "fwd": fwd, "l4": recs}
        if self.addr6 is not None:
            # src | dst (32 B) per record: source bytes 0..7 from the record, the other 24 B from
            # addr6, dense per chunk over the chunk's forwarded IPv6 frames
            a6 = self.addr6.cpu().numpy().view(np.uint8).reshape(-1, 24)
            v6 = recs["ver"] == 6
            rows = np.zeros((len(recs), 32), np.uint8)
            r6 = recs_all[idx][v6]
            rows[v6, :8] = np.stack([r6["w0"], r6["w1"]], axis=1).astype("<u4").view(np.uint8).reshape(-1, 8)
            rows[v6, 8:] = a6[_rank_index(recs["pkt_idx"][v6].astype(np.int64))]
            out["addr6"] = rows
        if self.conn is not None:
            c = self.conn.cpu().numpy().view(np.uint32).reshape(-1, 2)[idx]
            out["conn_hash"] = c[:, 0].copy()
            out["conn_info"] = c[:, 1].copy()
            if self.conn_words:
                cd = self.conn_dlv.cpu().numpy().view(np.uint64).reshape(-1, self.conn_words)
                out["conn_dlv"] = cd[idx]
        if self.deliver_words:
            dbm = self.dlv_bitmap.cpu().numpy().view(np.uint64)
            recs_d = self.dlv_records.cpu().numpy().view(np.uint64).reshape(-1, self.deliver_words)
            di = _segment_index(dbm)
            # rows of (frame index, statement mask words): the index is the bit's position
            frames = np.nonzero(np.unpackbits(dbm.view(np.uint8), bitorder="little")[:n])[0].astype(np.uint64)
            out["dlv"] = np.column_stack([frames, recs_d[di]]) if len(frames) else np.zeros((0, 1 + self.deliver_words), np.uint64)
        return out


CHUNK_FRAMES = 256  # RTN_CHUNK_FRAMES (include/retina_pc.h)


def _rank_index(frames: np.ndarray) -> np.ndarray:
    """Record-array index of each of `frames` (ascending frame indices of one record stream):
    records are dense per chunk of CHUNK_FRAMES frames, starting at chunk * CHUNK_FRAMES."""
    if frames.size == 0:
        return np.zeros(0, np.int64)
    chunk = frames // CHUNK_FRAMES
    # rank within the chunk = number of the stream's frames of the same chunk before it
    first = np.searchsorted(chunk, chunk, side="left")
    return chunk * CHUNK_FRAMES + (np.arange(frames.size, dtype=np.int64) - first)


def _segment_index(bm: np.ndarray) -> np.ndarray:
    """Index of every set bit of `bm` in a chunk-dense stream (addr6 / dlv_records), frame order."""
    bits = np.unpackbits(bm.view(np.uint8), bitorder="little").astype(np.int64)
    return _rank_index(np.nonzero(bits)[0])


REC_BLOCK = 64  # RTN_REC_BLOCK (include/retina_pc.h)


def _rec_index(frames: np.ndarray, n: int) -> np.ndarray:
    """RTN_REC_INDEX of each forwarded frame (ascending frame indices): the l4 / conn / conn_dlv /
    rtn_ct_entry_t / PacketDeliver-counts slot. Block k // 64 of chunk c sits at block slot
    (k // 64) * nchunks + c."""
    dense = _rank_index(frames)
    chunk = dense // CHUNK_FRAMES
    k = dense - chunk * CHUNK_FRAMES
    nch = (n + CHUNK_FRAMES - 1) // CHUNK_FRAMES
    return ((k // REC_BLOCK) * nch + chunk) * REC_BLOCK + k % REC_BLOCK


def _fwd_index(bm: np.ndarray, n: int) -> np.ndarray:
    """RTN_REC_INDEX of every set bit of the forwarded bitmap `bm`, in frame order."""
    bits = np.unpackbits(bm.view(np.uint8), bitorder="little").astype(np.int64)
    return _rec_index(np.nonzero(bits)[0], n)


class PacketContinue:
    """A Program loaded on one GPU: batch version of Subscription::continue_packet plus the
    L4Context gate of process_packet (core/src/subscription/mod.rs:94-127)."""

    def __init__(self, program: Program, device: int = 0):
        self.program = program
        self.device = device
        h = C.c_void_p()
        _check(lib().rtn_pc_create_from_program(program._h, device, C.byref(h)))
        self._h = h
        self.deliver_words = program.info["deliver_words"]
        self.conn_words = program.info["conn_words"]

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rtn_pc_destroy(self._h)
            self._h = C.c_void_p()

    def kernel_info(self, layout: int, conn: bool = False) -> dict:
        """rtn_pc_kernel_info: registers, LDS, occupancy and chunks per wave of one kernel instance
        (layout 0 monolithic, 1 64-byte slots, 2 split, 3 compact split)."""
        w = (C.c_uint32 * 5)()
        _check(lib().rtn_pc_kernel_info(self._h, layout, 1 if conn else 0, C.byref(w)))
        return dict(zip(("regs", "lds_bytes", "threads", "waves_per_simd", "chunks_per_wave"), list(w)))

    def set_grid(self, blocks: int) -> None:
        _check(lib().rtn_pc_set_grid(self._h, blocks))

    def take_status(self) -> int:
        """RTN_STATUS_* bits raised by runs without counters since the last call (synchronizes)."""
        st = C.c_uint32()
        _check(lib().rtn_pc_take_status(self._h, C.byref(st)))
        return int(st.value)

    def index(self, bitmap, n: int, chunk_base: bool = True, stream=None):
        """rtn_pc_index: (idx, chunk_base) device tensors for a device bitmap of n frames: idx = the
        frame indices of the set bits in frame order (accepted_idx), chunk_base = set bits before
        each chunk (+ the total). Synchronizes to read n_set."""
        import torch

        dev = bitmap.device
        idx = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        n_set = torch.zeros(1, dtype=torch.int32, device=dev)
        cb = torch.empty((n + CHUNK_FRAMES - 1) // CHUNK_FRAMES + 1, dtype=torch.int32, device=dev) if chunk_base else None
        s = stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        _check(lib().rtn_pc_index(self._h, C.c_void_p(bitmap.data_ptr()), n, C.c_void_p(idx.data_ptr()),
                                  C.c_void_p(n_set.data_ptr()), C.c_void_p(cb.data_ptr() if cb is not None else 0),
                                  C.c_void_p(s)))
        k = int(n_set.item())
        return idx[:k], cb

    def alloc_outputs(self, n: int, addr6: bool = True, counters: bool = True, conn: bool = False,
                      seqack: bool = True) -> PCOutputs:
        import torch

        dev = torch.device("cuda", self.device)
        L = lib()
        u8 = lambda nbytes: torch.empty(nbytes, dtype=torch.uint8, device=dev)  # noqa: E731
        dw = self.deliver_words
        return PCOutputs(
            n=n,
            pc_bitmap=u8(L.rtn_out_bitmap_bytes(n)),
            fwd_bitmap=u8(L.rtn_out_bitmap_bytes(n)),
            l4=u8(L.rtn_out_l4_bytes(n)),
            addr6=u8(L.rtn_out_addr6_bytes(n)) if addr6 else None,
            dlv_bitmap=u8(L.rtn_out_bitmap_bytes(n)) if dw else None,
            dlv_records=u8(L.rtn_out_dlv_bytes(n, dw)) if dw else None,
            counters=torch.zeros(COUNTERS_BYTES, dtype=torch.uint8, device=dev) if counters else None,
            deliver_words=dw,
            conn=u8(L.rtn_out_conn_bytes(n)) if conn else None,
            conn_dlv=u8(L.rtn_out_conn_dlv_bytes(n, self.conn_words)) if conn and self.conn_words else None,
            conn_words=self.conn_words if conn else 0,
            seqack=u8(L.rtn_out_seqack_bytes(n)) if seqack else None,
        )

    def run(self, slab, stride: int, data_len, n: int | None = None, out: PCOutputs | None = None,
            stream=None, core_id: int = 0, ext=None, dl_le64: bool = False, ext_chunk=None) -> PCOutputs:
        """One rtn_pc_run. `ext` (device uint8, 64 B per frame) selects the split layout: `slab`
        then holds bytes [0, 64) of every frame (stride 64) and `ext` bytes [64, 128).
        dl_le64 asserts that every data_len is <= 64 (RTN_BATCH_DL_LE64), which 64-byte slots
        without ext need unless `out` has counters (include/retina_pc.h). `ext_chunk` (device
        uint32, one per CHUNK_FRAMES-frame chunk) selects the compact split layout: `ext` then holds rows
        only for the frames rtn_ext_needed() names (split_slab(..., compact=True))."""
        import torch

        if n is None:
            n = int(data_len.numel())
        if out is None or out.n < n:
            out = self.alloc_outputs(n)
        flags = (BATCH_DL_LE64 if dl_le64 else 0) | (BATCH_EXT_COMPACT if ext_chunk is not None else 0)
        rows = int(ext.numel()) // 64 if ext is not None else 0
        b = _Batch(slab.data_ptr(), stride, data_len.data_ptr(), n, core_id,
                   ext.data_ptr() if ext is not None else None, flags, rows,
                   ext_chunk.data_ptr() if ext_chunk is not None else None)
        o = _out_struct(out)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(lib().rtn_pc_run(self._h, C.byref(b), C.byref(o), C.c_void_p(s.cuda_stream)))
        out.n = n
        return out


PD_ACTIVE = 1  # RTN_PD_ACTIVE (include/retina_pd.h)


def pd_run(pc: "PacketContinue", pc_out: PCOutputs, ct_entries, data_len, state, counts=None, bitmap=None,
           stream=None):
    """rtn_pd_run: the packet_deliver filter over a batch, after ConnTable.process. `state` is the
    device uint32 [slots][1 + n_pd_facts] per-connection table. Returns (counts, bitmap) device
    tensors: counts [record][n_pd_stmts] uint32 (valid where the bitmap is set)."""
    import torch

    if pc_out.addr6 is None or pc_out.conn is None:
        raise RetinaError(-22, "pd_run needs outputs allocated with addr6=True and conn=True")
    n = pc_out.n
    L = lib()
    dev = torch.device("cuda", pc.device)
    ns = pc.program.info["n_pd_stmts"]
    nf = pc.program.info["n_pd_facts"]
    if state.numel() % (1 + nf) != 0:
        raise RetinaError(-22, f"state must hold rows of 1 + {nf} uint32")
    if counts is None:
        counts = torch.empty(L.rtn_out_pd_counts_bytes(max(n, 1), ns) // 4, dtype=torch.int32, device=dev)
    if bitmap is None:
        bitmap = torch.empty(L.rtn_out_bitmap_bytes(max(n, 1)), dtype=torch.uint8, device=dev)
    o = _out_struct(pc_out)
    s = stream if stream is not None else torch.cuda.current_stream(pc.device)
    _check(L.rtn_pd_run(pc._h, C.byref(o), C.c_void_p(ct_entries.data_ptr()), C.c_void_p(data_len.data_ptr()), n,
                        C.c_void_p(state.data_ptr()), int(state.numel() // (1 + nf)), C.c_void_p(counts.data_ptr()),
                        C.c_void_p(bitmap.data_ptr()), C.c_void_p(s.cuda_stream)))
    return counts, bitmap


def decode_pd(counts, bitmap, pc_out: PCOutputs, n_stmts: int) -> tuple[np.ndarray, np.ndarray]:
    """(frame indices with a delivery, their per-statement counts) in frame order."""
    n = pc_out.n
    fwd_bm = pc_out.fwd_bitmap.cpu().numpy().view(np.uint64)
    fwd = np.nonzero(np.unpackbits(fwd_bm.view(np.uint8), bitorder="little")[:n])[0]
    rec = _rec_index(fwd, n)
    bm = bitmap.cpu().numpy().view(np.uint64)
    hit = np.unpackbits(bm.view(np.uint8), bitorder="little")[:n].astype(bool)
    sel = hit[fwd]
    c = counts.cpu().numpy().view(np.uint32).reshape(-1, max(n_stmts, 1))[:, :n_stmts]
    return fwd[sel], c[rec[sel]]


def pd_replay(pd: dict, counts_row, facts_row) -> list[int]:
    """The callback sequence (statement indices) the reference runs for one frame. A session loop
    runs its body once per matching session (deliver_filter.rs:123-151), i.e. facts_row[fact]
    times, so the statements of one loop body repeat as a block; a statement fires in a pass iff
    its count is non-zero (its packet and service conditions do not depend on the session)."""
    stmts = pd["stmts"]

    def rec(idx: list[int], depth: int) -> list[int]:
        out: list[int] = []
        i = 0
        while i < len(idx):
            loops = stmts[idx[i]]["loops"]
            if len(loops) == depth:
                if counts_row[idx[i]]:
                    out.append(idx[i])
                i += 1
                continue
            node, fact = loops[depth]
            j = i
            while j < len(idx) and len(stmts[idx[j]]["loops"]) > depth and stmts[idx[j]]["loops"][depth][0] == node:
                j += 1
            out += rec(idx[i:j], depth + 1) * int(facts_row[fact])
            i = j
        return out

    return rec(list(range(len(stmts))), 0)


class MappedHost:
    """A pinned host tensor (torch `pin_memory()`) seen through its device address, for output
    buffers the kernel writes straight into host memory over PCIe (no D2H copy): the C ABI takes
    plain pointers, and hipHostGetDevicePointer gives the one the GPU may use. Raises if the
    memory is not mapped for the device."""

    def __init__(self, host_tensor):
        if not host_tensor.is_pinned():
            raise RetinaError(-22, "MappedHost needs a pinned host tensor")
        hip = C.CDLL("libamdhip64.so")
        hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
        hip.hipHostGetDevicePointer.restype = C.c_int
        p = C.c_void_p()
        rc = hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(host_tensor.data_ptr()), 0)
        if rc != 0 or not p.value:
            raise RetinaError(-19, f"hipHostGetDevicePointer failed ({rc})")
        self.host = host_tensor
        self._dptr = int(p.value)

    def data_ptr(self) -> int:
        return self._dptr

    def numel(self) -> int:
        return self.host.numel()

    def cpu(self):
        return self.host


def _out_struct(out: PCOutputs) -> _Out:
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    return _Out(ptr(out.pc_bitmap), ptr(out.fwd_bitmap), ptr(out.l4), ptr(out.addr6), ptr(out.dlv_bitmap),
                ptr(out.dlv_records), ptr(out.counters), ptr(out.conn), ptr(out.conn_dlv), ptr(out.seqack))


class _CtStats(C.Structure):
    _fields_ = [("capacity", C.c_uint32), ("live", C.c_uint32), ("epoch", C.c_uint32),
                ("max_connections", C.c_uint32)]


CT_HIT, CT_NEW, CT_MISS, CT_NEW_DROPPED, CT_FULL, CT_COLLISION, CT_PRIOR = 1, 2, 3, 4, 5, 6, 0x100
CT_NO_SLOT = 0xFFFFFFFF


class ConnTable:
    """GPU connection lookup (include/retina_ct.h): the ConnTracker table step for whole batches,
    on a table resident in HBM. process() takes the PCOutputs of rtn_pc_run (with conn=True)."""

    def __init__(self, device: int = 0, capacity_log2: int = 20, max_connections: int | None = None):
        self.device = device
        h = C.c_void_p()
        cap = 1 << capacity_log2
        _check(lib().rtn_ct_create(device, capacity_log2, max_connections if max_connections is not None else cap,
                                   C.byref(h)))
        self._h = h
        self.capacity = cap

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rtn_ct_destroy(self._h)
            self._h = C.c_void_p()

    def process(self, pc_out: PCOutputs, out=None, stream=None):
        """Returns a device uint8 tensor of rtn_ct_entry_t (slot, status) indexed like pc_out.l4."""
        import torch

        if pc_out.conn is None or pc_out.addr6 is None:
            raise RetinaError(-22, "ConnTable.process needs outputs allocated with conn=True and addr6=True")
        n = pc_out.n
        if out is None:
            out = torch.empty(lib().rtn_out_ct_bytes(max(n, 1)), dtype=torch.uint8, device=torch.device("cuda", self.device))
        o = _out_struct(pc_out)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(lib().rtn_ct_process(self._h, C.byref(o), n, C.c_void_p(out.data_ptr()), C.c_void_p(s.cuda_stream)))
        return out

    def remove(self, slots, stream=None) -> None:
        """slots: device int32/uint32 tensor of connection handles."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(lib().rtn_ct_remove(self._h, C.c_void_p(slots.data_ptr()), int(slots.numel()), C.c_void_p(s.cuda_stream)))

    def rebuild(self, stream=None):
        """Compact tombstones; returns the device old-slot -> new-slot map (uint32 view in int32)."""
        import torch

        m = torch.empty(self.capacity, dtype=torch.int32, device=torch.device("cuda", self.device))
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(lib().rtn_ct_rebuild(self._h, C.c_void_p(m.data_ptr()), C.c_void_p(s.cuda_stream)))
        return m

    def stats(self) -> dict:
        st = _CtStats()
        _check(lib().rtn_ct_stats(self._h, C.byref(st)))
        return {f: getattr(st, f) for f, _ in _CtStats._fields_}


def decode_ct(entries, pc_out: PCOutputs) -> np.ndarray:
    """rtn_ct_entry_t of the forwarded frames in frame order: (slot, status) uint32 pairs."""
    fwd_bm = pc_out.fwd_bitmap.cpu().numpy().view(np.uint64)
    e = entries.cpu().numpy().view(np.uint32).reshape(-1, 2)
    return e[_fwd_index(fwd_bm, pc_out.n)]


def ext_needed(head: np.ndarray, dlen: np.ndarray) -> np.ndarray:
    """rtn_ext_needed (include/retina_pc.h) for every frame: head = [n, >= 64] first bytes."""
    h = head.astype(np.int64)
    et = (h[:, 12] << 8) | h[:, 13]
    q = et == 0x8100
    inner = np.where(q, (h[:, 16] << 8) | h[:, 17], et)
    ihl4 = (np.where(q, h[:, 18], h[:, 14]) & 0xF) << 2
    l4 = np.where(q, 18, 14) + np.where(inner == 0x86DD, 40, ihl4)
    ip = (inner == 0x0800) | (inner == 0x86DD)
    return ip & (dlen.astype(np.int64) > 64) & (l4 + 20 > 64)


def split_slab(slab: np.ndarray, stride: int, dlen: np.ndarray | None = None, compact: bool = False):
    """Monolithic slots of `stride` >= 128 -> the split layout (64-B head slots, 64-B ext slots):
    (head, ext). compact=True (needs dlen) keeps ext rows only for the frames that need them
    (RTN_BATCH_EXT_COMPACT) and returns (head, ext, ext_chunk)."""
    b = slab.reshape(-1, stride)
    head = np.ascontiguousarray(b[:, :64]).reshape(-1)
    if not compact:
        return head, np.ascontiguousarray(b[:, 64:128]).reshape(-1)
    need = ext_needed(b, dlen)
    ext = np.ascontiguousarray(b[need, 64:128]).reshape(-1)
    n = len(dlen)
    per = np.add.reduceat(need.astype(np.int64), np.arange(0, max(n, 1), CHUNK_FRAMES)) if n else np.zeros(0, np.int64)
    ext_chunk = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint32)
    if ext.size == 0:
        ext = np.zeros(64, np.uint8)  # (a valid pointer; no row is read)
    return head, ext, ext_chunk


def pack_frames(frames, stride: int = 128) -> tuple[np.ndarray, np.ndarray]:
    """Lay frames out as a header slab (slot = first min(len, stride) bytes) + u16 data_len."""
    n = len(frames)
    slab = np.zeros((n, stride), np.uint8)
    dlen = np.zeros(n, np.uint16)
    for i, f in enumerate(frames):
        b = np.frombuffer(bytes(f), np.uint8)
        k = min(len(b), stride)
        slab[i, :k] = b[:k]
        dlen[i] = len(b)
    return slab.reshape(-1), dlen


class PcapReader:
    """Offline ingest (include/retina_ingest.h): a libpcap/pcapng capture packed into the slot
    layout rtn_pc_run reads, with the reference's offline-runtime rules (offline.rs:64-82)."""

    def __init__(self, path, mtu: int = 9702):
        h = C.c_void_p()
        _check(lib().rtn_pcap_open(str(path).encode(), mtu, C.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rtn_pcap_close(self._h)
            self._h = C.c_void_p()

    def next_batch(self, slab: np.ndarray, stride: int, data_len: np.ndarray) -> int:
        """Fill host arrays slab (uint8, >= cap*stride) and data_len (uint16[cap]); returns frames packed."""
        cap = len(data_len)
        assert slab.dtype == np.uint8 and data_len.dtype == np.uint16 and slab.size >= cap * stride
        n = C.c_uint32()
        _check(lib().rtn_pcap_next_batch(self._h, slab.ctypes.data, stride, data_len.ctypes.data, cap, C.byref(n)))
        return n.value

    def next_batch_split(self, head: np.ndarray, ext: np.ndarray, ext_chunk: np.ndarray,
                         data_len: np.ndarray) -> tuple[int, int]:
        """The compact split layout (RTN_BATCH_EXT_COMPACT): head (uint8, cap*64), ext (uint8,
        rows*64), ext_chunk (uint32, ceil(cap/CHUNK_FRAMES)), data_len (uint16[cap]) -> (frames, ext rows)."""
        cap = len(data_len)
        assert head.size >= cap * 64 and ext.size % 64 == 0 and ext_chunk.size >= (cap + CHUNK_FRAMES - 1) // CHUNK_FRAMES
        n, rows = C.c_uint32(), C.c_uint32()
        _check(lib().rtn_pcap_next_batch_split(self._h, head.ctypes.data, ext.ctypes.data, ext.size // 64,
                                               ext_chunk.ctypes.data, data_len.ctypes.data, cap, C.byref(n),
                                               C.byref(rows)))
        return n.value, rows.value

    def next_batch_gpu(self, head, ext, ext_chunk, dlen_out, device: int = 0, stream=None) -> int:
        """rtn_pcap_next_batch_gpu: the capture walk on the GPU into device tensors in the gather
        layout (head: uint8 cap*64, ext: uint8 >= gather_ext_rows(cap)*64, ext_chunk: int32/uint32
        ceil(cap/CHUNK_FRAMES), dlen_out: int16/uint16 cap); returns the frames of the batch. The
        packing runs on `stream` (default: the current torch stream)."""
        import torch

        cap = dlen_out.numel()
        slab = _StageSlab(_addr(head), _addr(ext), _addr(ext_chunk), _addr(dlen_out), cap, ext.numel() // 64)
        s = stream if stream is not None else torch.cuda.current_stream(device)
        n = C.c_uint32()
        _check(lib().rtn_pcap_next_batch_gpu(self._h, device, C.byref(slab), C.byref(n), s.cuda_stream))
        return n.value

    def gpu_window(self, nbytes: int) -> None:
        _check(lib().rtn_pcap_gpu_window(self._h, nbytes))

    def rewind(self) -> None:
        _check(lib().rtn_pcap_rewind(self._h))

    def stats(self) -> dict:
        st = _PcapStats()
        _check(lib().rtn_pcap_stats(self._h, C.byref(st)))
        return {f: getattr(st, f) for f, _ in _PcapStats._fields_}

    def read_all(self, stride: int = 128, batch: int = 1 << 16) -> tuple[np.ndarray, np.ndarray]:
        slabs, lens = [], []
        while True:
            s = np.zeros(batch * stride, np.uint8)
            d = np.zeros(batch, np.uint16)
            k = self.next_batch(s, stride, d)
            if k == 0:
                break
            slabs.append(s[:k * stride])
            lens.append(d[:k])
        if not slabs:
            return np.zeros(0, np.uint8), np.zeros(0, np.uint16)
        return np.concatenate(slabs), np.concatenate(lens)


# ----------------------------------------------------------------------------------------------
# Hardware-assist filter (include/retina_hw.h): the rte_flow rules Retina installs on each port.

def _rule_dict(r: "_FlowRule") -> dict:
    items = [(it.item_type, it.size, bytes(it.spec), bytes(it.mask)) for it in r.items[:r.n_items]]
    return {"group": r.group, "priority": r.priority, "action": r.action, "jump_group": r.jump_group,
            "pattern": r.pattern, "items": items}


def _validator(validate):
    """A Python device model (rule dict -> bool) as an rtn_flow_validate_fn (NULL for None)."""
    if validate is None:
        return _FLOW_VALIDATE()
    return _FLOW_VALIDATE(lambda _user, rule: 1 if validate(_rule_dict(rule.contents)) else 0)


def hw_rules(filter_str: str | None = None, validate=None, program: "Program | None" = None) -> list[dict]:
    """rtn_hw_rules / rtn_program_hw_rules: rules as dicts {group, priority, action, jump_group,
    pattern, items: [(type, size, spec, mask)]}; `validate` models rte_flow_validate."""
    cb = _validator(validate)
    n = C.c_uint32(0)
    L = lib()
    call = (lambda buf, cap: L.rtn_program_hw_rules(program._h, cb, None, buf, cap, C.byref(n))) if program \
        else (lambda buf, cap: L.rtn_hw_rules(filter_str.encode(), cb, None, buf, cap, C.byref(n)))
    rc = call(None, 0)
    if rc not in (RTN_OK, -34):
        _check(rc)
    buf = (_FlowRule * max(n.value, 1))()
    _check(call(buf, n.value))
    return [_rule_dict(buf[k]) for k in range(n.value)]


def hw_patterns(filter_str: str, validate=None) -> str:
    """HardwareFilter's patterns, one flat pattern per line (rtn_hw_patterns)."""
    cb = _validator(validate)
    L = lib()
    need = L.rtn_hw_patterns(filter_str.encode(), cb, None, None, 0)
    buf = C.create_string_buffer(need + 1)
    L.rtn_hw_patterns(filter_str.encode(), cb, None, buf, need + 1)
    return buf.value.decode()


# ----------------------------------------------------------------------------------------------
# Staging DPDK RX bursts (include/retina_stage.h): mbuf data pointers -> the compact split layout.

STATUS_BAD_MBUF = 8  # RTN_STATUS_BAD_MBUF


def _addr(x) -> int:
    """Address of a numpy array or a torch tensor (or a MappedHost)."""
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    return x.data_ptr()


class Stager:
    """rtn_stage_mbufs: host worker threads gather mbufs (by data pointer = buf_addr + data_off)
    into the compact split layout in host memory: head slots, data_len, exactly compact ext rows
    and ext_chunk (the layout rtn_pc_run reads with RTN_BATCH_EXT_COMPACT)."""

    def __init__(self, threads: int = 0, cpus=None):
        h = C.c_void_p()
        arr = (C.c_int32 * len(cpus))(*cpus) if cpus else None
        _check(lib().rtn_stager_create(threads, arr, C.byref(h)))
        self._h = h
        self.threads = threads

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rtn_stager_destroy(self._h)
            self._h = C.c_void_p()

    def stage(self, ptrs: np.ndarray, data_len: np.ndarray, head, ext, ext_chunk, dlen_out, n: int | None = None,
              cap: int | None = None, ext_cap: int | None = None) -> tuple[int, int]:
        """ptrs: uint64[n] data pointers; data_len: uint16[n]. head / ext / ext_chunk / dlen_out:
        host buffers (numpy arrays or pinned torch tensors) sized for cap frames / ext_cap rows.
        Returns (rows, dl_max)."""
        n = len(ptrs) if n is None else n
        cap = (head.nbytes if isinstance(head, np.ndarray) else head.numel()) // 64 if cap is None else cap
        if ext_cap is None:
            ext_cap = (ext.nbytes if isinstance(ext, np.ndarray) else ext.numel()) // 64
        slab = _StageSlab(_addr(head), _addr(ext), _addr(ext_chunk), _addr(dlen_out), cap, ext_cap)
        rows, mx = C.c_uint32(), C.c_uint16()
        _check(lib().rtn_stage_mbufs(self._h, C.c_void_p(_addr(ptrs)), C.c_void_p(_addr(data_len)), n,
                                     C.byref(slab), C.byref(rows), C.byref(mx)))
        return rows.value, mx.value


def gather_ext_rows(n: int) -> int:
    """Ext rows rtn_stage_gather writes for n frames (256 per chunk)."""
    return int(lib().rtn_stage_gather_ext_rows(n))


class MbufPool:
    """rtn_mbuf_pool_register: a host memory range holding mbuf buffers, mapped for the GPU
    (hipHostRegister), from which rtn_stage_gather pulls frames over PCIe. `host` is a numpy
    array or a torch CPU tensor that stays alive while the pool exists."""

    def __init__(self, host, device: int = 0):
        self.host = host
        nbytes = host.nbytes if isinstance(host, np.ndarray) else host.numel() * host.element_size()
        self.base = _addr(host)
        self.nbytes = nbytes
        h = C.c_void_p()
        _check(lib().rtn_mbuf_pool_register(C.c_void_p(self.base), nbytes, device, C.byref(h)))
        self._h = h
        self.device = device

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rtn_mbuf_pool_destroy(self._h)
            self._h = C.c_void_p()

    def gather(self, ptrs, data_len, n: int, head, ext, ext_chunk, dlen_out, status=None, stream=None) -> None:
        """rtn_stage_gather on `stream`: ptrs (uint64) and data_len (uint16) device-readable
        (device or pinned host tensors); outputs device tensors. Asynchronous."""
        import torch

        slab = _StageSlab(_addr(head), _addr(ext), _addr(ext_chunk), _addr(dlen_out), head.numel() // 64,
                          ext.numel() // 64)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(lib().rtn_stage_gather(self._h, C.c_void_p(_addr(ptrs)), C.c_void_p(_addr(data_len)), n,
                                      C.byref(slab), C.c_void_p(_addr(status) if status is not None else 0),
                                      C.c_void_p(s.cuda_stream)))

    def take_status(self) -> int:
        st = C.c_uint32()
        _check(lib().rtn_mbuf_pool_take_status(self._h, C.byref(st)))
        return int(st.value)


def mbuf_pool(slab: np.ndarray, dlen: np.ndarray, stride: int, buf: int = 2176, headroom: int = 128,
              seed: int = 1, alloc=None):
    """A DPDK-shaped mbuf pool holding the frames of a slot slab: one `buf`-byte buffer per frame
    (RTE_MBUF_DEFAULT_BUF_SIZE 2176, headroom 128, core/src/memory/mempool.rs:26-29), in a
    shuffled order as a mempool hands them out after some churn. Buffer b receives its frame's
    slot bytes at headroom. Returns (pool uint8 array, data pointers uint64[n]).
    `alloc(nbytes)` may supply the (e.g. pinned) backing array."""
    n = len(dlen)
    raw = alloc(n * buf + 4096) if alloc is not None else np.zeros(n * buf + 4096, np.uint8)
    off = (-_addr(raw)) % 4096  # page-aligned pool (hipHostRegister pins whole pages), 128-B buffers
    pool = raw[off:off + n * buf]
    perm = np.random.default_rng(seed).permutation(n)
    pool.reshape(n, buf)[perm, headroom:headroom + stride] = slab.reshape(n, stride)
    ptrs = (_addr(pool) + perm.astype(np.uint64) * buf + headroom).astype(np.uint64)
    return pool, ptrs
