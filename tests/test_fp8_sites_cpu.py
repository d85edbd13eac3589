"""fp8 scale-site bookkeeping (ops/fp8.py) on the CPU: object keys are unique per live object
(never a recycled id()), a dead object's sites go back to the pool, and a reused row starts
with no amax history (a fresh bootstrap)."""
import gc

import torch

from p2p_pytorch_amd.ops import fp8


class _Obj:
    pass


def test_obj_key_stable_and_unique():
    a, b = _Obj(), _Obj()
    ka, kb = fp8.obj_key(a), fp8.obj_key(b)
    assert ka == fp8.obj_key(a) and kb == fp8.obj_key(b) and ka != kb
    w = torch.zeros(3, requires_grad=True)            # tensors (weights) carry keys too
    assert fp8.obj_key(w) == fp8.obj_key(w) != ka


def test_dead_object_sites_recycled_and_reset(monkeypatch):
    pool = fp8._Pool("cpu")
    monkeypatch.setitem(fp8._pools, "cpu-test", pool)
    a = _Obj()
    ka = fp8.obj_key(a)
    i1 = pool.site((ka, "x", 1))
    i2 = pool.site((ka, "gy", 1))
    other = _Obj()
    j = pool.site((fp8.obj_key(other), "x", 1))
    pool.fresh.discard(i1)
    pool.sites[i1] = torch.tensor([7, 7, 7, 7], dtype=torch.int32)   # an amax history
    del a
    gc.collect()
    assert (ka, "x", 1) not in pool.index and (ka, "gy", 1) not in pool.index
    assert sorted(pool.free) == sorted([i1, i2]) and j in pool.index.values()
    b = _Obj()                     # may even get a's id(): it must not inherit a's sites
    kb = fp8.obj_key(b)
    assert kb != ka
    r = pool.site((kb, "x", 1))
    assert r in (i1, i2) and r in pool.fresh
    assert int(pool.sites[r].abs().sum()) == 0       # zeroed before reuse
    assert pool.high == 3                            # no new row was needed


def test_pool_capacity_counts_rows_not_keys(monkeypatch):
    pool = fp8._Pool("cpu")
    monkeypatch.setitem(fp8._pools, "cpu-test", pool)
    for _ in range(50):            # short-lived weights (a test's per-run clones) never leak rows
        o = _Obj()
        pool.site((fp8.obj_key(o), "x", 1))
        del o
        gc.collect()
    assert pool.high == 1 and len(pool.index) == 0
