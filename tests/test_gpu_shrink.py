"""Save-time eviction EmbeddingVar::Shrink (embedding_var.h:264-313) as DumpEv
runs it before a save (save_restore_v2_ops.cc:117-133).

Global-step form: the timeline of embedding_variable_ops_test.py:478-497
(testEmbeddingVariableForShrinkNone: steps_to_live 5, id 2*i trained at
step i for i < 10) -- its expected survivors are derived here from the rule
gs - version > steps_to_live, since that test only prints.  L2 form: keys
whose 0.5 * |row|^2 is below the threshold, computed with numpy on the same
rows.  Integer outcomes (which keys survive, Size) are exact."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    deeprec_amd.set_validate(True)
    return deeprec_amd


def test_shrink_by_global_step_timeline(dr):
    ev = dr.EmbeddingVariable("shrink_gs", 3, 1.0, steps_to_live=5)
    opt = dr.GradientDescentOptimizer(0.1)
    for i in range(10):
        ev.sparse_read(T([2 * i]))
        ev.pending_grads.append(dr.IndexedSlices(T(np.full((1, 3), 2.0, np.float32)),
                                                 T([2 * i])))
        opt.apply_gradients([ev], global_step=i)
    assert int(ev.total_count()[0]) == 10
    removed = ev.shrink(10)            # 10 - i > 5  <=>  i < 5
    assert removed == 5
    keys, vals, vers, _ = ev.export()
    assert keys.tolist() == [10, 12, 14, 16, 18]
    assert vers.tolist() == [5, 6, 7, 8, 9]
    np.testing.assert_allclose(vals.cpu().numpy(), np.full((5, 3), 0.8, np.float32), rtol=1e-6)
    assert int(ev.total_count()[0]) == 5
    # an evicted key comes back as a fresh default row (LookupOrCreate)
    np.testing.assert_array_equal(ev.sparse_read(T([0, 12])).cpu().numpy(),
                                  np.array([[1.0] * 3, [0.8] * 3], np.float32))
    assert int(ev.total_count()[0]) == 6


def test_shrink_version_minus_one_becomes_global_step(dr):
    ev = dr.EmbeddingVariable("shrink_m1", 2, 0.0, steps_to_live=3)
    keys = T(np.arange(6, dtype=np.int64))
    vals = T(np.ones((6, 2), np.float32))
    vers = T(np.array([-1, -1, 0, 1, 7, 8], np.int64))
    ev.insert(keys, vals, vers, T(np.zeros(6, np.int64)))
    assert ev.shrink(8) == 2           # versions 0 and 1: 8 - v > 3
    k, _, v, _ = ev.export()
    assert k.tolist() == [0, 1, 4, 5]
    assert v.tolist() == [8, 8, 7, 8]


def test_shrink_by_l2_weight(dr):
    rng = np.random.default_rng(5)
    n, D, thr = 500, 8, 1.5
    rows = (rng.standard_normal((n, D)) * 0.6).astype(np.float32)
    ev = dr.EmbeddingVariable("shrink_l2", D, 0.0, l2_weight_threshold=thr)
    acc = ev.slot("Adagrad", 0.1)
    ev.insert(T(np.arange(n, dtype=np.int64) * 7), T(rows))
    l2 = np.zeros(n, np.float32)
    for j in range(D):                  # the reference's ascending fp32 sum
        l2 = (l2 + rows[:, j] * rows[:, j]).astype(np.float32)
    l2 = (l2 * np.float32(0.5)).astype(np.float32)
    want = (np.arange(n, dtype=np.int64) * 7)[l2 >= thr]
    assert ev.shrink() == n - want.shape[0]
    k, v, _, _ = ev.export()
    assert k.tolist() == want.tolist()
    np.testing.assert_array_equal(v.cpu().numpy(), rows[l2 >= thr])
    assert int(ev.total_count()[0]) == want.shape[0]
    # the slot EV shares the key space: its export shrinks with it
    assert acc.export()[0].tolist() == [] or set(acc.export()[0].tolist()) <= set(want.tolist())


def test_shrink_noop_without_eviction_config(dr):
    ev = dr.EmbeddingVariable("shrink_none", 4, 0.5)
    ev.sparse_read(T([1, 2, 3]))
    assert ev.shrink(100) == 0
    assert ev.export()[0].tolist() == [1, 2, 3]


def test_save_applies_shrink(dr, tmp_path):
    from deeprec_amd import checkpoint as ck
    ev = dr.EmbeddingVariable("shrink_save", 2, 0.0, steps_to_live=2)
    ev.insert(T(np.arange(4, dtype=np.int64)), T(np.ones((4, 2), np.float32)),
              T(np.array([0, 1, 5, 6], np.int64)), T(np.zeros(4, np.int64)))
    prefix = str(tmp_path / "model.ckpt-6")
    ck.save(prefix, {"emb": ev}, global_step=6)
    r = ck.BundleReader(prefix)
    assert sorted(r.lookup_rows("emb-keys", 0, 2).tolist()) == [2, 3]


def test_shrink_empty_ev(dr):
    ev = dr.EmbeddingVariable("shrink_empty", 4, 0.0, steps_to_live=3)
    assert ev.shrink(10) == 0
    assert int(ev.total_count()[0]) == 0
    assert ev.export()[0].numel() == 0
