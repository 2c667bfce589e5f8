"""dr_embedding_lookup_sparse -- the embedding_lookup_sparse / safe_embedding_
lookup_sparse composition as ONE C call (embedding_ops.py:480-675 and
:1209-1344), through ops.embedding_lookup_sparse_c -- against the oracle's
compositions (oracle.embedding_lookup_sparse / safe_embedding_lookup_sparse):
EVs with and without a Counter filter, dense tables (OOB ids latch), every
combiner, weights, max_norm, prune + fill with default_id None / given, empty
rows and ragged bags.  Bit-exact (same association order) except where the
reference's own arithmetic order is not fixed: the clip_by_norm L2 reduction
(an Eigen tree reduction in TF) and the weighted chain's divides, compared
at north_star's 1e-5 relative (atol 1e-6), as test_gpu_parity.py does."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(x):
    return torch.as_tensor(np.asarray(x), device=DEV)


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd as dr
    dr.load()
    dr.set_validate(True)
    return dr


def _sparse(rng, B, max_h, vocab, allow_empty):
    lens = rng.integers(0 if allow_empty else 1, max_h + 1, B)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(l) for l in lens]) if lens.sum() else np.zeros(0, np.int64)
    ind = np.stack([rows, cols], 1).astype(np.int64)
    return ind, rng.integers(0, vocab, rows.shape[0]).astype(np.int64)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("max_norm", [None, 1.5])
def test_ev_lookup_sparse_one_call(dr, orc, comb, weighted, max_norm):
    from deeprec_amd import ops
    rng = np.random.default_rng(hash((comb, weighted, max_norm)) % 1000)
    B, D = 211, 16
    ev = dr.EmbeddingVariable("lsc_%s_%d_%s" % (comb, weighted, max_norm), D, 0.25)
    oev = orc.EV(D, 0.25)
    keys = np.arange(0, 200, dtype=np.int64)
    vals = rng.standard_normal((200, D)).astype(np.float32)
    ev.insert(T(keys), T(vals))
    oev.insert(keys, vals)
    ind, v = _sparse(rng, B, 6, 260, allow_empty=False)      # ~25 % new keys
    w = rng.uniform(0.1, 2.0, v.shape[0]).astype(np.float32) if weighted else None
    out = ops.embedding_lookup_sparse_c(ev, T(ind), T(v), B, None if w is None else T(w),
                                        comb, max_norm)
    ref = orc.embedding_lookup_sparse(oev, ind, v, B, w, comb, max_norm)
    if max_norm is None and not weighted:
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    else:
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    assert int(ev.total_count()[0]) == oev.size()


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("safe", [False, True])
def test_bf16_ev_lookup_sparse_one_call(dr, orc, comb, weighted, safe):
    """bf16 EVs (BASELINE configs[4]) through the single entry: the rows are
    widened to float32 and pooled in the reference order into an fp32 output
    (embedding_ops.py:606-607), against oracle.EV(bf16=True)."""
    from deeprec_amd import ops
    rng = np.random.default_rng(31 + 3 * weighted + safe + len(comb))
    B, D = 173, 24
    ev = dr.EmbeddingVariable("lscbf_%s_%d_%d" % (comb, weighted, safe), D, 0.3,
                              value_dtype=torch.bfloat16)
    oev = orc.EV(D, 0.3, bf16=True)
    keys = np.arange(0, 150, dtype=np.int64)
    vals = orc.bf16_round(rng.standard_normal((150, D)).astype(np.float32))
    ev.insert(T(keys), T(vals).to(torch.bfloat16))
    oev.insert(keys, vals)
    ind, v = _sparse(rng, B, 5, 200, allow_empty=safe)
    if safe:
        v[::9] = -2
    w = rng.uniform(0.1, 2.0, v.shape[0]).astype(np.float32) if weighted else None
    out = ops.embedding_lookup_sparse_c(ev, T(ind), T(v), B, None if w is None else T(w), comb,
                                        None, safe=safe, default_id=None)
    assert out.dtype == torch.float32
    if safe:
        ref = orc.safe_embedding_lookup_sparse(oev, ind, v, (B, 5), w, comb, None)
    else:
        ref = orc.embedding_lookup_sparse(oev, ind, v, B, w, comb)
    if weighted:
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    else:
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert int(ev.total_count()[0]) == oev.size()


@pytest.mark.parametrize("default_id", [None, 3])
@pytest.mark.parametrize("weighted", [False, True])
def test_safe_lookup_one_call(dr, orc, default_id, weighted):
    from deeprec_amd import ops
    rng = np.random.default_rng(7 + (default_id or 0) + 10 * weighted)
    B, D = 150, 8
    ev = dr.EmbeddingVariable("slc_%s_%d" % (default_id, weighted), D, 0.5)
    oev = orc.EV(D, 0.5)
    ind, v = _sparse(rng, B, 5, 60, allow_empty=True)
    v[::7] = -3                                   # pruned ids
    w = rng.uniform(-0.5, 2.0, v.shape[0]).astype(np.float32) if weighted else None
    out = ops.embedding_lookup_sparse_c(ev, T(ind), T(v), B, None if w is None else T(w),
                                        "mean", None, safe=True, default_id=default_id)
    ref = orc.safe_embedding_lookup_sparse(oev, ind, v, (B, 5), w, "mean", default_id)
    if weighted:
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)
    else:
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert int(ev.total_count()[0]) == oev.size()


def test_counter_filter_ev_one_call(dr, orc):
    """Counter filter: UniqueWithCounts -> KvResourceGatherV1 with counts;
    the admission timeline over three calls equals the oracle's, in the
    plain and the safe (device-count, one host read) forms."""
    from deeprec_amd import ops
    rng = np.random.default_rng(41)
    B, D = 90, 4
    for safe in (False, True):
        ev = dr.EmbeddingVariable("cf_lsc%d" % safe, D, 0.0,
                                  ev_option=dr.EmbeddingVariableOption(
                                      filter_option=dr.CounterFilter(3)))
        oev = orc.EV(D, 0.0, filter_freq=3)
        ins = rng.integers(0, 30, (30, D)).astype(np.float32)
        for step in range(3):
            ind, v = _sparse(rng, B, 3, 30, allow_empty=safe)
            if safe:
                out = ops.embedding_lookup_sparse_c(ev, T(ind), T(v), B, None, "sum", None,
                                                    safe=True)
                ref = orc.safe_embedding_lookup_sparse(oev, ind, v, (B, 3), None, "sum")
            else:
                out = ops.embedding_lookup_sparse_c(ev, T(ind), T(v), B, None, "sum")
                ref = orc.embedding_lookup_sparse(oev, ind, v, B, None, "sum")
            np.testing.assert_array_equal(out.cpu().numpy(), ref)
        del ins


@pytest.mark.parametrize("safe", [False, True])
def test_dense_table_one_call(dr, orc, safe):
    from deeprec_amd import ops
    from deeprec_amd._lib import DeepRecError
    rng = np.random.default_rng(5 + safe)
    B, R, D = 120, 80, 32
    table = rng.standard_normal((R, D)).astype(np.float32)
    ind, v = _sparse(rng, B, 4, R, allow_empty=safe)
    if safe:
        v[::5] = -1
        out = ops.embedding_lookup_sparse_c(T(table), T(ind), T(v), B, None, "sqrtn", 2.0,
                                            safe=True, default_id=None)
        ref = orc.safe_embedding_lookup_sparse(table, ind, v, (B, 4), None, "sqrtn", None, 2.0)
    else:
        out = ops.embedding_lookup_sparse_c(T(table), T(ind), T(v), B, None, "sqrtn", 2.0)
        ref = orc.embedding_lookup_sparse(table, ind, v, B, None, "sqrtn", 2.0)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)   # max_norm
    bad = v.copy()
    bad[3] = R + 5                                     # OOB dense id latches InvalidArgument
    with pytest.raises(DeepRecError):
        ops.embedding_lookup_sparse_c(T(table), T(ind), T(bad), B, None, "sum")
        dr.status_check()
    dr.status_check()


def test_empty_and_unsorted(dr):
    from deeprec_amd import ops
    from deeprec_amd._lib import DeepRecError
    ev = dr.EmbeddingVariable("lsc_empty", 8, 1.0)
    e = torch.zeros((0, 2), dtype=torch.int64, device=DEV)
    out = ops.embedding_lookup_sparse_c(ev, e, torch.zeros(0, dtype=torch.int64, device=DEV), 5)
    assert out.shape == (5, 8) and not bool(out.any())
    out = ops.embedding_lookup_sparse_c(ev, e, torch.zeros(0, dtype=torch.int64, device=DEV), 5,
                                        safe=True, default_id=None)
    assert not bool(out.any())
    out = ops.embedding_lookup_sparse_c(ev, e, torch.zeros(0, dtype=torch.int64, device=DEV), 5,
                                        safe=True, default_id=2)
    assert bool((out == 1.0).all())                    # id 2's first touch: the default row
    # rows not sorted / out of range: INVALID_ARGUMENT latched, and the pool
    # behind the offsets (no host sync in between) reads only valid positions
    for bad in ([[3, 0], [1, 0]], [[-5, 0], [0, 0]], [[0, 0], [9, 0]]):
        with pytest.raises(DeepRecError):
            ops.embedding_lookup_sparse_c(ev, T(np.array(bad, np.int64)),
                                          T(np.array([1, 2], np.int64)), 5)
            dr.status_check()
        dr.status_check()
