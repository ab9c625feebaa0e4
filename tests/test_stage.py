"""Staging DPDK RX bursts (include/retina_stage.h): mbuf data pointers -> the compact split layout
rtn_pc_run reads, by host worker threads (rtn_stage_mbufs; CPU tests against the numpy packer) and
by the GPU pulling frames out of a registered host mbuf pool (rtn_stage_gather; GPU tests, then
rtn_pc_run against the oracle). The mbufs are DPDK-shaped (2176-B buffers, 128-B headroom,
core/src/memory/mempool.rs:26-29) and handed out in shuffled order; the reference reads each
header in place at buf_addr + data_off + offset (core/src/memory/mbuf.rs:125-141) after rx_burst
(core/src/lcore/rx_core.rs:57-73)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import helpers
from golden.filter_sets import SETS
from retina_amd import pc, synth

GOLD = Path(__file__).resolve().parent / "golden"


def corpus(name: str, n: int):
    """(slab, dlen, stride, filter set) of a named corpus, n frames (0 = all)."""
    if name in ("traces", "adversarial"):
        t = np.load(GOLD / ("traces.npz" if name == "traces" else "corpus_adversarial.npz"))
        slab, dlen = t["slab"], t["dlen"]
        if n:
            slab, dlen = slab[:n * 128], dlen[:n]
        return slab, dlen, 128, "cfg3"
    if name == "cfg2":
        s, d = synth.cfg2(n, start=11)
        return s, d, 64, "cfg2"
    s, d = getattr(synth, name)(n, start=7)
    return s, d, 128, name


def expected(slab, dlen, stride):
    """The compact split layout of the same frames (pc.split_slab, the packer the parity tests
    already hold to the monolithic slots): head slots, exact ext rows, ext_chunk."""
    n = len(dlen)
    if stride == 64:
        return slab.copy(), np.zeros(0, np.uint8), np.zeros((n + 255) // 256, np.uint32)
    head, ext, chunk = pc.split_slab(slab, stride, dlen, compact=True)
    rows = int(pc.ext_needed(slab.reshape(-1, stride), dlen).sum())
    return head, ext[:rows * 64], chunk


def _buf(nbytes: int, off: int) -> np.ndarray:
    """nbytes zero bytes starting `off` bytes past a 64-B boundary (0: the streaming-store copy;
    otherwise the plain one)."""
    raw = np.zeros(nbytes + 128, np.uint8)
    a = (-raw.ctypes.data) % 64 + off
    return raw[a:a + nbytes]


def host_stage(stager, ptrs, dlen, n, ext_cap=None, off=0):
    head = _buf(max(n, 1) * 64, off)
    ext = _buf(max(n if ext_cap is None else ext_cap, 1) * 64, off)
    chunk = np.zeros(max((n + 255) // 256, 1), np.uint32)
    dl = np.zeros(max(n, 1), np.uint16)
    rows, mx = stager.stage(ptrs, dlen, head, ext, chunk, dl, n=n, ext_cap=ext_cap)
    return head[:n * 64], ext[:rows * 64], chunk[:(n + 255) // 256], dl[:n], rows, mx


@pytest.mark.parametrize("threads", [0, 3, 8])
@pytest.mark.parametrize("name,n", [("cfg3", 20000 + 37), ("cfg2", 9000 + 5), ("cfg4", 12345), ("traces", 0),
                                    ("adversarial", 0), ("cfg3", 255), ("cfg3", 1)])
def test_host_stage_matches_packer(name, n, threads):
    slab, dlen, stride, _ = corpus(name, n)
    n = len(dlen)
    pool, ptrs = pc.mbuf_pool(slab, dlen, stride, seed=n)
    st = pc.Stager(threads)
    head, ext, chunk, dl, rows, mx = host_stage(st, ptrs, dlen, n)
    eh, ee, ec = expected(slab, dlen, stride)
    assert np.array_equal(dl, dlen)
    assert mx == int(dlen.max())
    assert rows * 64 == ee.size, (rows, ee.size // 64)
    assert np.array_equal(chunk, ec)
    assert np.array_equal(head, eh)
    assert np.array_equal(ext, ee)


@pytest.mark.parametrize("off", [0, 16, 1])
def test_host_stage_slab_alignment(off):
    """Aligned slabs take streaming stores, others a plain copy: same bytes either way."""
    slab, dlen, stride, _ = corpus("cfg3", 9000)
    n = len(dlen)
    pool, ptrs = pc.mbuf_pool(slab, dlen, stride, seed=3)
    head, ext, chunk, dl, rows, mx = host_stage(pc.Stager(4), ptrs, dlen, n, off=off)
    eh, ee, ec = expected(slab, dlen, stride)
    assert np.array_equal(head, eh) and np.array_equal(ext, ee) and np.array_equal(chunk, ec)


def test_host_stage_empty_and_errors():
    slab, dlen, stride, _ = corpus("cfg3", 3000)
    pool, ptrs = pc.mbuf_pool(slab, dlen, stride)
    st = pc.Stager(2)
    assert host_stage(st, ptrs, dlen, 0)[4:] == (0, 0)
    need = int(pc.ext_needed(slab.reshape(-1, stride), dlen).sum())
    assert need > 10
    with pytest.raises(pc.RetinaError) as e:  # fewer ext rows than the frames need
        host_stage(st, ptrs, dlen, len(dlen), ext_cap=need - 1)
    assert e.value.code == -34
    head = np.zeros(64 * 10, np.uint8)
    with pytest.raises(pc.RetinaError) as e:  # more frames than the slab holds
        st.stage(ptrs, dlen, head, np.zeros(64, np.uint8), np.zeros(1, np.uint32), np.zeros(10, np.uint16), n=11,
                 cap=10)
    assert e.value.code == -34
    # exactly enough rows
    out = host_stage(st, ptrs, dlen, len(dlen), ext_cap=need)
    assert out[4] == need


# ---------------------------------------------------------------------------------------------
# GPU


def _pinned(nbytes: int) -> np.ndarray:
    import torch

    return torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy()


def _gather(name, n, pinned_pool: bool, ptr_on_device: bool = False, bad=None):
    """Gather the corpus from a registered mbuf pool; returns everything the checks need."""
    import torch

    slab, dlen, stride, fset = corpus(name, n)
    n = len(dlen)
    dev = torch.device("cuda", 0)
    pool, ptrs = pc.mbuf_pool(slab, dlen, stride, seed=n + 1, alloc=_pinned if pinned_pool else None)
    mp = pc.MbufPool(pool, 0)
    if bad is not None:  # pointers outside the pool: never dereferenced, data_len 0, status raised
        ptrs = ptrs.copy()
        lo, hi = mp.base, mp.base + mp.nbytes
        for k, i in enumerate(bad):
            ptrs[i] = [0, lo - 64, hi - 100, hi, (1 << 64) - 64][k % 5]
    h_ptrs = torch.from_numpy(ptrs.view(np.int64)).pin_memory()
    h_dl = torch.from_numpy(dlen.view(np.int16)).pin_memory()
    if ptr_on_device:
        h_ptrs, h_dl = h_ptrs.to(dev), h_dl.to(dev)
    rows = pc.gather_ext_rows(max(n, 1))
    head = torch.zeros(max(n, 1) * 64, dtype=torch.uint8, device=dev)
    ext = torch.zeros(rows * 64, dtype=torch.uint8, device=dev)
    chunk = torch.zeros(max((n + 255) // 256, 1), dtype=torch.int32, device=dev)
    dl = torch.zeros(max(n, 1), dtype=torch.int16, device=dev)
    mp.gather(h_ptrs, h_dl, n, head, ext, chunk, dl)
    torch.cuda.synchronize()
    status = mp.take_status()
    return dict(slab=slab, dlen=dlen, stride=stride, fset=fset, n=n, pool=pool, mp=mp, head=head, ext=ext,
                chunk=chunk, dl=dl, status=status, rows=rows)


def _run_and_check(g, dlen_expected, what):
    import torch

    prog = pc.Program.from_spec(SETS[g["fset"]])
    ctx = pc.PacketContinue(prog, 0)
    n = g["n"]
    out = ctx.run(g["head"], 64, g["dl"], n, out=ctx.alloc_outputs(max(n, 1)), ext=g["ext"], ext_chunk=g["chunk"])
    torch.cuda.synchronize()
    got = helpers.canonical(prog, out, dlen_expected)
    assert got["counters"][3] == 0, got["counters"]
    ora = helpers.oracle_run(SETS[g["fset"]], g["slab"], g["stride"], dlen_expected)
    helpers.assert_same(got, ora, what)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("cfg3", (1 << 16) + 77), ("cfg4", 30000), ("cfg2", 40000 + 3), ("traces", 0),
                                    ("adversarial", 0), ("cfg3", 1), ("cfg3", 300)])
def test_gather_layout_and_parity(gpu, name, n):
    g = _gather(name, n, pinned_pool=False)
    n, dlen, slab, stride = g["n"], g["dlen"], g["slab"], g["stride"]
    assert g["status"] == 0
    assert np.array_equal(g["dl"].cpu().numpy().view(np.uint16)[:n], dlen)
    eh, ee, ec = expected(slab, dlen, stride)
    assert np.array_equal(g["head"].cpu().numpy()[:n * 64], eh)
    nch = (n + 255) // 256
    assert np.array_equal(g["chunk"].cpu().numpy().view(np.uint32)[:nch], np.arange(nch, dtype=np.uint32) * 256)
    # ext: chunk c's rows are the exact rows of its needing frames, at c*256 + rank
    ext = g["ext"].cpu().numpy().reshape(-1, 64)
    ee = ee.reshape(-1, 64)
    counts = np.diff(np.append(ec.astype(np.int64), len(ee)))
    for c in range(nch):
        k = int(counts[c])
        assert np.array_equal(ext[c * 256:c * 256 + k], ee[ec[c]:ec[c] + k]), f"chunk {c}"
    _run_and_check(g, dlen, f"gather {name}")


@pytest.mark.gpu
def test_gather_pinned_pool_and_device_pointers(gpu):
    """A pool pinned by its allocator (hipHostMalloc: mapped as it is) and the pointer array in
    device memory give the same batch."""
    g = _gather("cfg3", 20000, pinned_pool=True, ptr_on_device=True)
    assert g["status"] == 0
    _run_and_check(g, g["dlen"], "gather (pinned pool, device pointers)")


@pytest.mark.gpu
def test_gather_bad_pointers_are_never_read(gpu):
    """Pointers outside the registered pool (NULL, below it, straddling or past its end) are not
    dereferenced: their frames get data_len 0 (dropped, as an empty frame) and the status bit."""
    bad = [0, 5, 255, 256, 1000, 4095, 9999]
    g = _gather("cfg3", 10000, pinned_pool=False, bad=bad)
    assert g["status"] == pc.STATUS_BAD_MBUF
    d = g["dlen"].copy()
    d[bad] = 0
    assert np.array_equal(g["dl"].cpu().numpy().view(np.uint16)[:g["n"]], d)
    _run_and_check(g, d, "gather with bad pointers")
    assert g["mp"].take_status() == 0  # cleared


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg3", "cfg2", "adversarial"])
def test_host_stage_then_gpu_parity(gpu, name):
    """Form (a): host threads stage into pinned memory, H2D, rtn_pc_run: the oracle's results."""
    import torch

    slab, dlen, stride, fset = corpus(name, 50000 if name != "adversarial" else 0)
    n = len(dlen)
    pool, ptrs = pc.mbuf_pool(slab, dlen, stride, seed=3)
    head, ext, chunk, dl, rows, mx = host_stage(pc.Stager(4), ptrs, dlen, n)
    dev = torch.device("cuda", 0)
    g = dict(fset=fset, n=n, slab=slab, stride=stride,
             head=torch.from_numpy(head).to(dev), ext=torch.from_numpy(ext if rows else np.zeros(64, np.uint8)).to(dev),
             chunk=torch.from_numpy(chunk.view(np.int32)).to(dev), dl=torch.from_numpy(dl.view(np.int16)).to(dev))
    _run_and_check(g, dlen, f"host stage {name}")
