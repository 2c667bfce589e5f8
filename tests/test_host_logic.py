"""Host-side logic that needs no GPU: the sharded lookup autograd node's
forward-generation guard (modelzoo._ShardedLookupFn) and the capture-safe
deferred release queue (kv_variable_ops)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deeprec-1_amd"))


class _FakeEngine(object):
    """Stands in for a row-sharded engine: forward returns a [B, D] tensor,
    backward records the gradient it was handed."""

    def __init__(self):
        self.seen = []

    def forward(self, ids, need_grad=False):
        return ids.float().unsqueeze(1).repeat(1, 2)

    def backward(self, g):
        self.seen.append(g.clone())


def test_sharded_backward_refuses_after_second_forward():
    from deeprec_amd import modelzoo as mz
    eng = _FakeEngine()
    anchor = torch.zeros(1, requires_grad=True)
    ids = torch.arange(4)
    out1 = mz._sharded_lookup(anchor, eng, ids)
    out1.sum().backward()                       # the latest forward: fine
    assert len(eng.seen) == 1
    out2 = mz._sharded_lookup(anchor, eng, ids)
    out3 = mz._sharded_lookup(anchor, eng, ids)  # overwrites out2's routing state
    with pytest.raises(RuntimeError, match="another forward ran"):
        out2.sum().backward()
    out3.sum().backward()
    assert len(eng.seen) == 2
    out4 = mz._sharded_lookup(anchor, eng, ids)
    with torch.no_grad():                       # an eval pass in between
        mz._sharded_lookup(anchor, eng, ids)
    with pytest.raises(RuntimeError, match="another forward ran"):
        out4.sum().backward()


def test_deferred_release_queue_is_lock_free_for_del():
    """__del__ may run (cyclic GC) inside the locked flush on the same thread:
    queueing must not take the flush's lock."""
    from deeprec_amd import kv_variable_ops as kvo
    n0 = len(kvo._DEFERRED)
    acquired = kvo._DEFERRED_LOCK.acquire(timeout=5)
    assert acquired
    try:
        kvo._release_engine("dr_sharded_destroy", None)   # would deadlock on a held Lock
        assert len(kvo._DEFERRED) == n0 + 1
    finally:
        kvo._DEFERRED.pop()
        kvo._DEFERRED_LOCK.release()
