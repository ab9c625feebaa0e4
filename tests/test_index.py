"""accepted_idx / n_accepted through rtn_pc_index: the frame indices of a bitmap's
set bits in frame order, their count and each chunk's base, against numpy on random bitmaps
(ragged n, garbage bits past n, empty and full), and tied to the packet kernel's own records:
the record at RTN_REC_INDEX(n, c, k) is frame idx[chunk_base[c] + k]."""
from __future__ import annotations

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from retina_amd import pc, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gpu):  # torch's HIP runtime first (the gpu fixture), then the library's context
    return pc.PacketContinue(pc.Program.from_spec(SETS["cfg2"]), gpu)


def _expect(words: np.ndarray, n: int):
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(np.int64)
    idx = np.flatnonzero(bits)
    per = np.add.reduceat(bits, np.arange(0, n, pc.CHUNK_FRAMES)) if n else np.zeros(0, np.int64)
    base = np.concatenate([[0], np.cumsum(per)])
    return idx, base


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 256, 257, 4097, 100_003, (1 << 20) + 37, 4096 * 64 * 3 + 5])
@pytest.mark.parametrize("density", [0.0, 0.03, 0.5, 1.0])
def test_index_vs_numpy(ctx, n, density):
    import torch

    rng = np.random.default_rng(n * 7 + int(density * 100))
    nw = (n + 63) // 64
    bits = (rng.random(nw * 64) < density).astype(np.uint8)
    bits[n:] = rng.integers(0, 2, nw * 64 - n)  # garbage past n: not frames
    words = np.packbits(bits, bitorder="little").view(np.uint64)
    got_idx, got_base = ctx.index(torch.from_numpy(words.view(np.int64)).cuda(), n)
    want_idx, want_base = _expect(words, n)
    assert np.array_equal(got_idx.cpu().numpy().astype(np.int64), want_idx)
    assert np.array_equal(got_base.cpu().numpy().astype(np.int64), want_base)


def test_index_empty_batch(ctx):
    import torch

    idx, base = ctx.index(torch.zeros(1, dtype=torch.int64, device="cuda"), 0)
    assert idx.numel() == 0 and int(base[0]) == 0


def test_index_ties_records_to_frames(ctx):
    """On a synthetic cfg3 batch run through the packet kernel: every forwarded record sits at the
    RTN_REC_INDEX the chunk bases give, and idx equals the oracle's forwarded frames."""
    import torch

    spec = SETS["cfg3"]
    slab, dlen = synth.cfg3((1 << 16) + 77)
    got = helpers.gpu_run(spec, slab, 128, dlen)
    ora = helpers.oracle_run(spec, slab, 128, dlen)
    n = len(dlen)
    fwd = np.asarray(got["fwd"], dtype=bool)[:n]
    assert np.array_equal(fwd, np.asarray(ora["fwd"], dtype=bool))
    nw = (n + 63) // 64
    fwd_words = np.packbits(np.pad(fwd, (0, nw * 64 - n)).astype(np.uint8), bitorder="little").view(np.uint64)
    idx, base = ctx.index(torch.from_numpy(fwd_words.view(np.int64)).cuda(), n)
    idx = idx.cpu().numpy().astype(np.int64)
    base = base.cpu().numpy().astype(np.int64)
    assert np.array_equal(idx, np.flatnonzero(ora["fwd"]))
    # (chunk, rank) of every forwarded frame from the chunk bases -> RTN_REC_INDEX == the decoder's
    chunk = idx // pc.CHUNK_FRAMES
    k = np.arange(idx.size) - base[chunk]
    nch = (n + pc.CHUNK_FRAMES - 1) // pc.CHUNK_FRAMES
    rec = ((k // pc.REC_BLOCK) * nch + chunk) * pc.REC_BLOCK + k % pc.REC_BLOCK
    assert np.array_equal(rec, pc._rec_index(idx, n))
