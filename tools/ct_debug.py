"""Connection-table accounting probe (experiments only): tests/test_ct.py's batches-with-removals
scenario, printing per batch the live counter, the live slots found by scanning the table, and the
number of keys held by more than one slot.

    python tools/ct_debug.py
"""
from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tools")]


def table_host(ct, cap: int) -> np.ndarray:
    from retina_amd import pc

    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipDeviceSynchronize()
    out = np.zeros(cap * 16, np.uint32)
    ptr = pc.lib().rtn_ct_table(ct._h)
    assert hip.hipMemcpy(out.ctypes.data, ptr, cap * 64, 2) == 0  # hipMemcpyDeviceToHost
    return out.reshape(cap, 16)


def main() -> None:
    import torch

    torch.cuda.init()  # torch's HIP runtime first, then the library's (as the tests do)
    import test_ct as T
    import helpers
    from oracle import conn as oconn
    from retina_amd import pc

    import os

    if os.environ.get("CT_VARIANT"):  # a tools/ct_variants.py variant through the experiments build
        import ct_variants

        pc._LIB_PATH = pc._LIB_PATH.with_name("libretina_pc_exp.so")
        os.environ["RTN_CT_TEMPLATE"] = str(ct_variants.write(os.environ["CT_VARIANT"], ROOT / "tools" / "_ab" / "ct"))
    pc.lib().rtn_ct_table.restype = C.c_void_p
    rng = np.random.default_rng(7)
    pool = helpers.flow_pool(rng, 1500)
    r = T._Run()
    model = oconn.TableModel()
    ids, owner = {}, {}
    for b in range(4):
        frames = helpers.flow_frames(rng, pool, 6000 + 37 * b)
        exp = model.process(T._model_frames(frames, r.pf))
        got = r.batch(frames)
        T._check(got, exp, ids, owner)
        tab = table_host(r.ct, r.ct.capacity)
        tags = tab[:, 0].astype(np.uint64) | (tab[:, 1].astype(np.uint64) << 32)
        live_slots = np.nonzero(tags > 1)[0]
        u, cnt = np.unique(tags[live_slots], return_counts=True)
        dup = u[cnt > 1]
        print(f"batch {b}: counter {r.ct.stats()['live']} scanned {len(live_slots)} model {len(model.present)} "
              f"duplicate keys {len(dup)}", flush=True)
        # live slots no model connection owns: print them and the batch's frames of the same key
        orphans = [int(x) for x in live_slots if int(x) not in owner]
        mf = T._model_frames(frames, r.pf)
        for sl in orphans[:5]:
            w = tab[sl, 4:14].tolist()
            print("   orphan slot", sl, "epoch/first", tab[sl, 2:4].tolist(), "key", w, flush=True)
            for i, ((key, opens, drops), (mid, est), (gs, gst)) in enumerate(zip(mf, exp, got)):
                ver, mx, mn, proto = key
                if ver == 4 and mx[0] == w[0] and mn[0] == w[4] and ((mx[1] << 16) | mn[1]) == w[8]:
                    print(f"      frame {i} opens {opens} drops {drops} model ({mid}, {est}) gpu ({int(gs)}, {int(gst)})",
                          flush=True)
        for d in dup[:5]:
            sl = live_slots[tags[live_slots] == d]
            print("   dup", hex(int(d)), "slots", sl.tolist(), "epoch/first", [tab[s, 2:4].tolist() for s in sl],
                  "key", [tab[s, 4:14].tolist() for s in sl][:1], flush=True)
        live = list(model.present.items())
        drop = [live[i] for i in rng.choice(len(live), size=len(live) // 5, replace=False)]
        slots = np.array([ids[mid] for _, (mid, _) in drop], np.uint32)
        r.ct.remove(r.torch.from_numpy(slots.view(np.int32)).to("cuda:0"))
        model.remove([k for k, _ in drop])
        for _, (mid, _) in drop:
            owner.pop(ids.pop(mid), None)
        print(f"   after removal: counter {r.ct.stats()['live']} model {len(model.present)}", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def churn() -> None:
    """tests/test_ct.py::test_ct_churn_reuses_removed_slots, printing the table around any FULL."""
    import torch

    torch.cuda.init()
    import test_ct as T
    import helpers
    from oracle import conn as oconn
    from retina_amd import pc

    pc.lib().rtn_ct_table.restype = C.c_void_p
    rng = np.random.default_rng(23)
    r = T._Run(cap_log2=10, max_conn=900)
    model = oconn.TableModel(max_connections=900)
    ids, owner = {}, {}
    for b in range(14):
        pool = helpers.flow_pool(rng, 300)
        frames = helpers.flow_frames(rng, pool, 900, p_syn=0.9)
        exp = model.process(T._model_frames(frames, r.pf))
        got = r.batch(frames)
        tab = table_host(r.ct, r.ct.capacity)
        tags = tab[:, 0].astype(np.uint64) | (tab[:, 1].astype(np.uint64) << 32)
        print(f"batch {b}: live {r.ct.stats()['live']} empty {(tags == 0).sum()} removed {(tags == 1).sum()} "
              f"used {(tags > 1).sum()} FULL {int((got[:, 1] & 0xFF == pc.CT_FULL).sum())}", flush=True)
        if (got[:, 1] & 0xFF == pc.CT_FULL).any():
            bad = np.nonzero(got[:, 1] & 0xFF == pc.CT_FULL)[0][:3]
            for i in bad:
                print("   FULL frame", int(i), "model", exp[i], flush=True)
            break
        T._check(got, exp, ids, owner)
        live = list(model.present.items())
        slots = np.array([ids[mid] for _, (mid, _) in live], np.uint32)
        r.ct.remove(r.torch.from_numpy(slots.view(np.int32)).to("cuda:0"))
        model.remove([k for k, _ in live])
        for _, (mid, _) in live:
            owner.pop(ids.pop(mid), None)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "churn":
    churn()
