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
        q.put((rank, totals.tolist(), times.tolist()))
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
    for rank, totals, times in got:
        assert totals == exp, (rank, totals, exp)
        assert times == [0.5 + world - 1, 1.0 * (world - 1)]
    assert rdist.aggregate_mpps(N_PER_RANK, world, 10, 1.0) == N_PER_RANK * world * 10 / 1e6


def test_shard_bounds():
    from retina_amd import dist as rdist

    s = rdist.shard(100, 3, 4)
    assert (s.start, s.count) == (300, 100)
    with pytest.raises(ValueError):
        rdist.shard(100, 4, 4)
