"""Byte-mutation fuzz of the HIP path against the oracle at 2^20 frames: valid IMIX / 1500-B
frames (synth.cfg3 / cfg4) with 1-4 header bytes in [12, 96) overwritten at random and, for a
quarter of the frames, data_len cut to a random value. The mutations reach every branch the
adversarial corpus names (EtherType, 802.1Q/802.1ad tags, IHL, protocol / next header, TCP data
offset, length fields, truncation at any byte) in combinations no hand-written corpus holds, in
all three slot layouts. Bit-exact: accept set, forwarded set, every L4Context field and the
packet-level statement masks."""
from __future__ import annotations

import zlib

import numpy as np
import pytest

import helpers
import test_range_runs
from golden.filter_sets import SETS
from retina_amd import synth

pytestmark = pytest.mark.gpu


def mutate(slab: np.ndarray, dlen: np.ndarray, stride: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(seed)
    rows = slab.reshape(-1, stride).copy()
    n = len(dlen)
    for _ in range(4):
        hit = rng.random(n) < 0.6
        pos = rng.integers(12, 96, n)
        # bias toward the bytes the parse branches on: EtherType / tag, IHL, protocol, doff
        hot = np.array([12, 13, 14, 16, 17, 18, 23, 27, 20, 46, 50, 58, 66])
        pos = np.where(rng.random(n) < 0.5, hot[rng.integers(0, len(hot), n)], pos)
        val = rng.integers(0, 256, n).astype(np.uint8)
        # half the tag / EtherType writes pick a meaningful value instead of a random one
        et = np.array([0x81, 0x00, 0x88, 0xA8, 0x86, 0xDD, 0x08, 0x45, 0x06, 0x11, 0x4F, 0x60], np.uint8)
        val = np.where(rng.random(n) < 0.5, et[rng.integers(0, len(et), n)], val)
        i = np.nonzero(hit)[0]
        rows[i, pos[i]] = val[i]
    dl = dlen.astype(np.int64).copy()
    cut = rng.random(n) < 0.25
    dl[cut] = rng.integers(0, np.maximum(dl[cut], 1) + 1)
    return rows.reshape(-1), dl.astype(dlen.dtype)


CASES = [("cfg3", synth.cfg3, SETS["cfg3"]), ("cfg4", synth.cfg4, SETS["cfg4"]),
         ("quirks", synth.cfg3, SETS["quirks"]), ("ranges", synth.cfg4, test_range_runs.SPEC)]


@pytest.mark.parametrize("layout", [False, True, "compact"])
@pytest.mark.parametrize("name,gen,spec", CASES, ids=[c[0] for c in CASES])
def test_mutation_fuzz(name, gen, spec, layout, gpu):
    n = (1 << 20) + 11
    slab, dlen = gen(n, start=7 << 20)
    slab, dlen = mutate(slab, dlen, 128, seed=zlib.crc32(name.encode()))
    helpers.assert_same(helpers.gpu_run(spec, slab, 128, dlen, split=layout),
                        helpers.oracle_run(spec, slab, 128, dlen), f"fuzz {name}/{layout}")
