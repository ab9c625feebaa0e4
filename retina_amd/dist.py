"""Multi-GPU sharding for the packet stage.

Packets are independent at this stage, so ranks never exchange packet data on the data path:
rank r filters its own shard of the frame stream on its own GPU (weak scaling). The only
collectives are the reduction of per-rank totals and timings, once, outside the timed region --
SURVEY §8e's `allreduce(sum)` of {packets, accepted, forwarded, delivered} plus a max of the
per-rank times -- a gather of the per-rank kernel times for the report, and, for RSS shards only,
an all-to-all of the generated frames at setup (each rank generates 1/world of the stream and
sends every frame to the rank its RSS queue belongs to). The same functions run over RCCL
("nccl") on GPUs and over gloo in the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    start: int  # index of the rank's first frame in the global stream
    count: int  # frames per rank (weak scaling: fixed per rank)


def env_rank() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(frames_per_rank: int, rank: int, world: int) -> Shard:
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return Shard(rank, world, rank * frames_per_rank, frames_per_rank)


# Retina's symmetric RSS key (core/src/port/mod.rs:22-28) and redirection table size (:28, 156-165)
SYMMETRIC_RSS_KEY = bytes([0x6D, 0x5A] * 26)
RSS_RETA_SIZE = 512


def _toeplitz_tables(key: bytes = SYMMETRIC_RSS_KEY, nbytes: int = 36) -> np.ndarray:
    """T[p][v] = the Toeplitz hash contribution of byte value v at input byte p: the XOR of the
    32-bit key windows starting at every set bit of v (bit 7 of byte 0 first)."""
    kbits = int.from_bytes(key, "big")
    klen = 8 * len(key)
    win = np.array([(kbits >> (klen - 32 - i)) & 0xFFFFFFFF for i in range(8 * nbytes)], np.uint64)
    t = np.zeros((nbytes, 256), np.uint64)
    for p in range(nbytes):
        for b in range(8):
            on = (np.arange(256) >> (7 - b)) & 1
            t[p] ^= np.where(on == 1, win[8 * p + b], 0).astype(np.uint64)
    return t.astype(np.uint32)


_TT = None


def rss_hash(slab: np.ndarray, stride: int, dlen: np.ndarray) -> np.ndarray:
    """The NIC's RSS hash of each frame under Retina's port configuration
    (core/src/port/mod.rs:320-331: rss_hf = ETH_RSS_IP | ETH_RSS_TCP | ETH_RSS_UDP, symmetric
    key): Toeplitz over src addr | dst addr [| src port | dst port] for IPv4 / IPv6 with TCP or
    UDP, over the addresses only for other IP frames, 0 for non-IP frames. The headers are located
    with the packet parsers' rules (Ethernet / one 802.1Q tag / IPv4 IHL / IPv6 without extension
    headers). With the symmetric key both directions of a connection hash alike, so a connection's
    frames all land on one rank."""
    global _TT
    if _TT is None:
        _TT = _toeplitz_tables()
    b = np.ascontiguousarray(slab, np.uint8).reshape(-1, stride)
    n = len(dlen)
    rows = np.arange(n)
    et = (b[:, 12].astype(np.int64) << 8) | b[:, 13]
    vl = et == 0x8100
    l3 = np.where(vl, 18, 14)
    inner = np.where(vl, (b[:, 16].astype(np.int64) << 8) | b[:, 17], et)
    dl = dlen.astype(np.int64)
    v4 = (inner == 0x0800) & (l3 + 20 <= dl)
    v6 = (inner == 0x86DD) & (l3 + 40 <= dl)
    col = lambda off: b[rows, np.minimum(off, stride - 1)]  # noqa: E731
    proto = np.where(v4, col(l3 + 9), col(l3 + 6)).astype(np.int64)
    l4 = l3 + np.where(v4, (col(l3) & 15).astype(np.int64) * 4, 40)
    ports = (v4 | v6) & ((proto == 6) | (proto == 17)) & (l4 + 4 <= np.minimum(dl, stride))
    h = np.zeros(n, np.uint32)
    # IPv4: src(4) dst(4) [sport dport]; IPv6: src(16) dst(16) [ports]
    for p in range(8):
        h ^= np.where(v4, _TT[p][col(l3 + 12 + p)], 0).astype(np.uint32)
    for p in range(4):
        h ^= np.where(v4 & ports, _TT[8 + p][col(l4 + p)], 0).astype(np.uint32)
    for p in range(32):
        h ^= np.where(v6, _TT[p][col(l3 + 8 + p)], 0).astype(np.uint32)
    for p in range(4):
        h ^= np.where(v6 & ports, _TT[32 + p][col(l4 + p)], 0).astype(np.uint32)
    return h


def rss_rank(hashes: np.ndarray, world: int) -> np.ndarray:
    """Queue / GPU of each frame: RETA[hash % 512] with the RETA filled round-robin over the
    queues (port/mod.rs:156-165), one queue per rank."""
    return ((hashes.astype(np.int64) % RSS_RETA_SIZE) % world).astype(np.int64)


def reduce_totals(totals, times):
    """Sum the per-rank totals (int64 tensor) and take the max of the per-rank times (float64
    tensor) over all ranks, in place, whenever a process group is up (one rank included, so the
    RCCL path runs even at N=1 under torch.distributed.run). Returns (totals, times)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        host = dist.get_backend() == "gloo" and totals.is_cuda  # gloo reduces host tensors
        t, m = (totals.cpu(), times.cpu()) if host else (totals, times)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        if host:
            totals.copy_(t)
            times.copy_(m)
    return totals, times


def aggregate_mpps(frames_per_rank: int, world: int, steps: int, max_wall_s: float) -> float:
    """Whole-job throughput: every rank's frames over the slowest rank's time."""
    return frames_per_rank * world * steps / max_wall_s / 1e6


def gather_rows(row, device=None) -> np.ndarray:
    """Every rank's float64 row (same length on all ranks) as a [world, k] array, on every rank;
    the row itself when no process group is up. Outside any timed region."""
    import torch
    import torch.distributed as dist

    r = np.asarray(row, np.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return r[None, :]
    on_dev = dist.get_backend() == "nccl"
    t = torch.from_numpy(r.copy())
    if on_dev:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return np.stack([o.cpu().numpy() for o in out])


_HOST_GROUP = None


def _host_group():
    """A gloo group over all ranks (host memory, blocking waits), created once."""
    import torch.distributed as dist

    global _HOST_GROUP
    if _HOST_GROUP is None:
        _HOST_GROUP = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
    return _HOST_GROUP


def host_barrier() -> None:
    """A barrier whose waiting ranks block in a socket read (gloo) instead of polling the GPU
    stream: rank 0 times the CPU baseline on the host cores while the others wait here."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=_host_group())


def exchange(parts: list) -> list:
    """All-to-all of byte arrays: parts[d] (uint8) goes to rank d; returns, by source rank, the
    arrays every rank sent this one. Setup only (RSS shards): it runs over a gloo group on host
    memory whatever the main backend is, so the same code path runs here and on the GPU node."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    g = _host_group()
    sizes = torch.tensor([int(p.size) for p in parts], dtype=torch.int64)
    got = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(got, sizes, group=g)
    send = torch.from_numpy(np.concatenate([np.ascontiguousarray(p, np.uint8).reshape(-1) for p in parts]))
    recv = torch.empty(int(got.sum()), dtype=torch.uint8)
    dist.all_to_all_single(recv, send, got.tolist(), sizes.tolist(), group=g)
    r = recv.numpy()
    offs = np.concatenate([[0], np.cumsum(got.numpy())])
    return [r[offs[k]:offs[k + 1]] for k in range(world)]


def rss_shard(gen, stride: int, total: int, rank: int, world: int, chunk: int = 1 << 21):
    """This rank's frames of the global stream [0, total) under Retina's symmetric RSS (rss_hash,
    rss_rank), in stream order. `gen(k, start)` returns (slab, dlen) of frames [start, start + k).
    Rank r generates only the stream's chunks r, r + world, ... (1/world of the stream), hashes
    them, and sends every frame to its queue's rank (exchange); chunks are then reassembled in
    stream order from the per-chunk counts, so the result equals filtering the whole stream."""
    nch = (total + chunk - 1) // chunk
    counts = np.zeros((world, nch), np.int64)  # frames of my chunks per destination
    slabs = [[] for _ in range(world)]
    dls = [[] for _ in range(world)]
    for c in range(rank, nch, world):
        s0 = c * chunk
        k = min(chunk, total - s0)
        sl, dl = gen(k, s0)
        q = rss_rank(rss_hash(sl, stride, dl), world)
        rows = sl.reshape(k, stride)
        for d in range(world):
            sel = q == d
            counts[d, c] = int(sel.sum())
            slabs[d].append(rows[sel].reshape(-1))
            dls[d].append(dl[sel])
    cat = lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt)  # noqa: E731
    if world == 1:
        return cat(slabs[0], np.uint8), cat(dls[0], np.uint16)
    rc = [x.view(np.int64) for x in exchange([counts[d].view(np.uint8) for d in range(world)])]
    rs = exchange([cat(slabs[d], np.uint8) for d in range(world)])
    rd = [x.view(np.uint16) for x in exchange([cat(dls[d], np.uint16).view(np.uint8) for d in range(world)])]
    n = int(sum(int(x.sum()) for x in rc))
    slab = np.empty(n * stride, np.uint8)
    dlen = np.empty(n, np.uint16)
    off = [0] * world
    at = 0
    for c in range(nch):  # chunk c came from rank c % world
        src = c % world
        k = int(rc[src][c])
        slab[at * stride:(at + k) * stride] = rs[src][off[src] * stride:(off[src] + k) * stride]
        dlen[at:at + k] = rd[src][off[src]:off[src] + k]
        off[src] += k
        at += k
    return slab, dlen
