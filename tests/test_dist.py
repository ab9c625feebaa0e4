"""The multi-GPU path's host logic on CPU: world_size-2 gloo ranks shard the seeded frame stream,
filter their shards (oracle as the stand-in for each rank's GPU) and reduce totals/timings with
the same retina_amd.dist functions bench.py uses over RCCL; the reduced totals must equal one
process filtering the whole stream."""
import os
import socket

import numpy as np
import pytest

from golden.filter_sets import SETS

N_PER_RANK = 1 << 14


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank: int, world: int, port: int, cfg: str, q) -> None:
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root), str(root / "tests")]
    import torch
    import torch.distributed as dist

    import helpers
    from retina_amd import dist as rdist
    from retina_amd import synth

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = rdist.shard(N_PER_RANK, rank, world)
        slab, dlen = getattr(synth, cfg)(sh.count, start=sh.start)
        stride = len(slab) // len(dlen)
        r = helpers.oracle_run(SETS[cfg], slab, stride, dlen)
        totals = torch.tensor([sh.count, int(r["pc"].sum()), int(r["fwd"].sum()),
                               int((r["dm"] != 0).any(1).sum()) if r["dm"].size else 0], dtype=torch.int64)
        times = torch.tensor([0.5 + rank, 1.0 * rank], dtype=torch.float64)
        rdist.reduce_totals(totals, times)
        rows = rdist.gather_rows([float(rank), 2.0 * rank + 0.5])  # bench.py's per-rank report
        rdist.host_barrier()  # where bench.py parks the ranks during rank 0's CPU baseline
        q.put((rank, totals.tolist(), times.tolist(), rows.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_two_rank_shards_reduce_to_single_process(cfg):
    import multiprocessing as mp

    import helpers
    from retina_amd import dist as rdist
    from retina_amd import synth

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    slab, dlen = getattr(synth, cfg)(N_PER_RANK * world, start=0)
    stride = len(slab) // len(dlen)
    r = helpers.oracle_run(SETS[cfg], slab, stride, dlen)
    exp = [N_PER_RANK * world, int(r["pc"].sum()), int(r["fwd"].sum()),
           int((r["dm"] != 0).any(1).sum()) if r["dm"].size else 0]
    for rank, totals, times, rows in got:
        assert totals == exp, (rank, totals, exp)
        assert times == [0.5 + world - 1, 1.0 * (world - 1)]
        assert rows == [[float(r), 2.0 * r + 0.5] for r in range(world)]
    assert rdist.aggregate_mpps(N_PER_RANK, world, 10, 1.0) == N_PER_RANK * world * 10 / 1e6


def test_shard_bounds():
    from retina_amd import dist as rdist

    s = rdist.shard(100, 3, 4)
    assert (s.start, s.count) == (300, 100)
    with pytest.raises(ValueError):
        rdist.shard(100, 4, 4)


def test_toeplitz_known_answers_and_symmetry():
    """retina_amd.dist's Toeplitz hash reproduces the published RSS verification vectors (the
    Microsoft RSS key, IPv4 with ports) and, under Retina's symmetric key
    (core/src/port/mod.rs:22-28), hashes both directions of a connection alike."""
    import ipaddress

    import helpers
    from retina_amd import dist as rdist
    from retina_amd import pc

    ms_key = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
    t = rdist._toeplitz_tables(ms_key, 12)
    for src, dst, sp, dp, want in (("66.9.149.187", "161.142.100.80", 2794, 1766, 0x51CCC178),
                                   ("199.92.111.2", "65.69.140.83", 14230, 4739, 0xC626B0EA),
                                   ("24.19.198.95", "12.22.207.184", 12898, 38024, 0x5C2B394A)):
        inp = ipaddress.IPv4Address(src).packed + ipaddress.IPv4Address(dst).packed + sp.to_bytes(2, "big") + dp.to_bytes(2, "big")
        h = 0
        for p, v in enumerate(inp):
            h ^= int(t[p][v])
        assert h == want
    rng = np.random.default_rng(3)
    frames = []
    for _ in range(300):
        v6 = bool(rng.random() < 0.3)
        a, b = int(rng.integers(0, 1 << 32)), int(rng.integers(0, 1 << 32))
        pa, pb = int(rng.integers(1, 65536)), int(rng.integers(1, 65536))
        pr = 6 if rng.random() < 0.5 else 17
        frames += [helpers.build_frame(v6, a, b, pa, pb, pr, 0x02), helpers.build_frame(v6, b, a, pb, pa, pr, 0x12)]
    slab, dlen = pc.pack_frames(frames, 128)
    h = rdist.rss_hash(slab, 128, dlen)
    assert (h[0::2] == h[1::2]).all() and len(set(h.tolist())) > 290
    ranks = rdist.rss_rank(h, 8)
    assert set(ranks.tolist()) == set(range(8))


def _rss_rank_main(rank: int, world: int, port: int, n: int, chunk: int, q) -> None:
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root), str(root / "tests")]
    import torch.distributed as dist

    import bench
    from retina_amd import dist as rdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d = bench.gen_rss_shard("cfg3", n, rank, world, chunk=chunk)
        rdist.host_barrier()
        q.put((rank, s, d))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk", [(4, 1 << 12), (3, 5000), (2, 1 << 21)])
def test_rss_shards_partition_the_stream(world, chunk):
    """bench.py --shard rss: each rank generates 1/world of the stream (chunks r, r + world, ...)
    and sends every frame to the rank of its RSS queue (an all-to-all over gloo); the ranks' frames
    then partition the global stream (every frame on exactly one rank, stream order kept), exactly
    as filtering the whole stream per rank would, and the per-rank counts are near even."""
    import multiprocessing as mp

    import bench
    from retina_amd import dist as rdist

    n = 1 << 14
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rss_rank_main, args=(r, world, port, n, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = dict((r, (s, d)) for r, s, d in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, fd = bench.gen_frames("cfg3", world * n, 0)
    assert sum(len(d) for _, d in parts.values()) == world * n
    rk = rdist.rss_rank(rdist.rss_hash(full, 128, fd), world)
    for r, (s, d) in parts.items():
        assert np.array_equal(d, fd[rk == r])
        assert np.array_equal(s.reshape(-1, 128), full.reshape(-1, 128)[rk == r])
        assert abs(len(d) - n) < n * 0.1


@pytest.mark.gpu
def test_rccl_process_group_one_rank(gpu):
    """The RCCL path bench.py takes under torch.distributed.run: a 1-rank "nccl" process group bound
    to cuda:0, the totals / times reduction on device tensors (reduce_totals), and a barrier."""
    import torch
    import torch.distributed as dist

    from retina_amd import dist as rdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        tot = torch.tensor([5, 7, 11], dtype=torch.int64, device="cuda")
        tim = torch.tensor([0.25, 1.5], dtype=torch.float64, device="cuda")
        rdist.reduce_totals(tot, tim)
        dist.barrier()
        torch.cuda.synchronize()
        assert tot.tolist() == [5, 7, 11] and tim.tolist() == [0.25, 1.5]
        assert dist.get_backend() == "nccl"
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("shard", ["contiguous", "rss"])
def test_bench_under_torchrun_rccl(gpu, shard, tmp_path):
    """bench.py as the driver launches it for N GPUs (python -m torch.distributed.run ... bench.py
    --gpus N), here N = 1 on one card with RCCL: it prints one JSON line with the reduced totals."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(root / "bench.py"), "--gpus", "1", "--steps", "3",
           "--warmup", "1", "--frames", str(1 << 20), "--no-cpu", "--no-e2e", "--no-conn", "--shard", shard]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["verified"]["ok"]
    assert line["config"]["shard"]["frames_total"] == 1 << 20
