"""GPU parity for the partitioned lookups and the weighted / max_norm backward:

* FusedEmbeddingSparsePreLookUp / PostLookUp / PostLookUpGrad against the
  reference KATs (fused_embedding_ops_test.cc:59-97, 129-196, 217-290) and the
  oracle, and fused_embedding_lookup_sparse over partitioned tables;
* embedding_lookup_sparse backward with sp_weights and max_norm
  (embedding_ops.py:609-651, _clip) against the oracle's chain rule: weighted
  grads bit-exact, clipped grads within 1e-5 relative (row norms are summed in
  wave order on the GPU);
* partitioned EmbeddingVariables (ids % 1000 % np, embedding_ops.py:207-299):
  forward equals the single EV, a training step updates each partition as
  the single EV would be updated, and filter counts reach every partition.
"""
import json
import os
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda:0"
RTOL = 1e-5


def load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    deeprec_amd.set_validate(True)
    assert torch.cuda.is_available()
    return deeprec_amd


@pytest.fixture(scope="module")
def ops(dr):
    from deeprec_amd import ops
    return ops


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


def H(t):
    return t.detach().cpu().numpy()


def _sparse(rng, B, M, vocab, allow_empty=False):
    lens = rng.integers(0 if allow_empty else 1, M + 1, B)
    r = np.repeat(np.arange(B), lens)
    c = np.concatenate([np.sort(rng.choice(M, n, replace=False)) for n in lens]) \
        if lens.sum() else np.zeros(0, np.int64)
    ind = np.stack([r, c], 1).astype(np.int64)
    vals = rng.integers(0, vocab, r.shape[0]).astype(np.int64)
    return ind, vals


# ---- PreLookUp / PostLookUp / PostLookUpGrad --------------------------------
def test_pre_lookup_kat(ops):
    g = load("pre_lookup_partition")
    ind = np.asarray(g["sp_indices"], np.int64).reshape(-1, 2)
    pv, pi = ops.fused_embedding_sparse_pre_look_up([(r, 8) for r in g["partition_rows"]],
                                                    T(g["sp_values"]), T(ind))
    assert len(pv) == len(g["expected"])
    for v, i, exp in zip(pv, pi, g["expected"]):
        assert H(v).tolist() == exp["values"]
        assert H(i).ravel().tolist() == exp["indices"]


def test_pre_lookup_matches_oracle_random(ops, orc):
    rng = np.random.default_rng(3)
    for rows in ([5], [100, 1, 37], [1] * 20, [0, 50, 0, 9]):
        n = int(rng.integers(0, 3000))
        vals = rng.integers(0, sum(rows), n).astype(np.int64) if sum(rows) else \
            np.zeros(0, np.int64)
        ind = np.stack([np.arange(n), rng.integers(0, 7, n)], 1).astype(np.int64)
        pv, pi = ops.fused_embedding_sparse_pre_look_up([(r, 4) for r in rows], T(vals), T(ind))
        ref = orc.fused_pre_lookup(vals, rows)
        for v, i, (rv, rpos) in zip(pv, pi, ref):
            np.testing.assert_array_equal(H(v), rv)
            np.testing.assert_array_equal(H(i), ind[rpos])


def test_pre_lookup_rejects_out_of_range(dr, ops):
    with pytest.raises(dr.InvalidArgumentError):
        ops.fused_embedding_sparse_pre_look_up([(3, 4), (2, 4)], T([0, 5, 1]),
                                               T([[0, 0], [0, 1], [1, 0]]))


def test_post_lookup_kat(ops):
    c = load("post_lookup")["forward"]
    D = c["dim"]
    shards = [T(np.asarray(s, np.float32).reshape(-1, D)) for s in c["shards"]]
    inds = [T(np.asarray(i, np.int64).reshape(-1, 2)) for i in c["indices"]]
    out, fnum = ops.fused_embedding_sparse_post_look_up(shards, inds, (c["batch"], c["cols"]),
                                                        combiner=c["combiner"],
                                                        max_norm=c["max_norm"])
    np.testing.assert_allclose(H(out).ravel(), c["expected"], atol=c["tol"], rtol=0)
    assert H(fnum).tolist() == c["feature_nums"]


def test_post_lookup_grad_kat(ops):
    c = load("post_lookup")["grad"]
    D = c["dim"]
    top = T(np.asarray(c["top_grad"], np.float32).reshape(c["batch"], D))
    shards = [T(np.asarray(s, np.float32).reshape(-1, D)) for s in c["shards"]]
    inds = [T(np.asarray(i, np.int64).reshape(-1, 2)) for i in c["indices"]]
    outs = ops.fused_embedding_sparse_post_look_up_grad(top, shards, inds, T(c["feature_nums"]),
                                                        combiner=c["combiner"],
                                                        max_norm=c["max_norm"])
    for o, e in zip(outs, c["expected"]):
        np.testing.assert_allclose(H(o).ravel(), e, atol=c["tol"], rtol=0)


@pytest.mark.parametrize("D", [8, 13, 64, 128])
@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_post_lookup_matches_oracle(ops, orc, D, comb):
    rng = np.random.default_rng(D)
    B, M, rows = 300, 9, [40, 7, 90]
    ind, vals = _sparse(rng, B, M, sum(rows), allow_empty=True)
    table = (rng.standard_normal((sum(rows), D)) * 2).astype(np.float32)
    acc = np.cumsum([0] + rows)
    parts = orc.fused_pre_lookup(vals, rows)
    shards = [table[acc[p] + v] for p, (v, _) in enumerate(parts)]
    inds = [ind[pos] for _, pos in parts]
    for mn in (None, 3.0):
        ref, rfn = orc.fused_post_lookup(shards, inds, B, M, comb, -1.0 if mn is None else mn)
        out, fnum = ops.fused_embedding_sparse_post_look_up([T(s) for s in shards],
                                                            [T(i) for i in inds], (B, M),
                                                            combiner=comb, max_norm=mn)
        assert H(fnum).tolist() == rfn.tolist()
        if mn is None:
            np.testing.assert_array_equal(H(out), ref)   # incl. NaN of empty mean/sqrtn bags
        else:
            np.testing.assert_allclose(H(out), ref, rtol=RTOL, atol=1e-6)
        top = rng.standard_normal((B, D)).astype(np.float32)
        gref = orc.fused_post_lookup_grad(top, shards, inds, rfn, comb, -1.0 if mn is None else mn)
        gout = ops.fused_embedding_sparse_post_look_up_grad(T(top), [T(s) for s in shards],
                                                            [T(i) for i in inds], fnum,
                                                            combiner=comb, max_norm=mn)
        for a, b in zip(gout, gref):
            if mn is None:
                np.testing.assert_array_equal(H(a), b)
            else:
                np.testing.assert_allclose(H(a), b, rtol=RTOL, atol=1e-6)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_fused_lookup_sparse_partitioned(dr, ops, orc, comb):
    """fused_embedding_lookup_sparse over 3 partitions == the local fused
    lookup on the whole table (bit-exact), and its backward == the local
    op's per-nnz grads summed per id (UnsortedSegmentSum order)."""
    rng = np.random.default_rng(11)
    B, M, D, rows = 200, 6, 16, [30, 5, 45]
    ind, vals = _sparse(rng, B, M, sum(rows))
    table = rng.standard_normal((sum(rows), D)).astype(np.float32)
    acc = np.cumsum([0] + rows)
    parts = [T(table[acc[p]:acc[p + 1]]).requires_grad_(True) for p in range(3)]
    sp = dr.SparseTensor(T(ind), T(vals), (B, M))
    out = dr.fused_embedding_lookup_sparse(parts, sp, combiner=comb)
    ref, off = orc.fused_local_lookup(table, vals, ind[:, 0], B, comb)
    np.testing.assert_array_equal(H(out), ref)
    top = rng.standard_normal((B, D)).astype(np.float32)
    out.backward(T(top))
    gl = orc.fused_local_lookup_grad(top, table, vals, off, comb)
    dense = orc.unsorted_segment_sum(gl, vals.astype(np.int32), sum(rows))
    for p in range(3):
        np.testing.assert_array_equal(H(parts[p].grad), dense[acc[p]:acc[p + 1]])


def test_fused_lookup_sparse_dense_tables_queue_slices(dr, orc):
    rng = np.random.default_rng(12)
    B, M, D, rows = 64, 4, 8, [20, 20]
    ind, vals = _sparse(rng, B, M, 40)
    table = rng.standard_normal((40, D)).astype(np.float32)
    tabs = [dr.DenseTable(T(table[:20])), dr.DenseTable(T(table[20:]))]
    out = dr.fused_embedding_lookup_sparse(tabs, dr.SparseTensor(T(ind), T(vals), (B, M)),
                                           combiner="mean", max_norm=2.5)
    ref, off = orc.fused_local_lookup(table, vals, ind[:, 0], B, "mean", 2.5)
    np.testing.assert_allclose(H(out), ref, rtol=RTOL, atol=1e-6)
    top = rng.standard_normal((B, D)).astype(np.float32)
    out.backward(T(top))
    gl = orc.fused_local_lookup_grad(top, table, vals, off, "mean", 2.5)
    dense = orc.unsorted_segment_sum(gl, vals.astype(np.int32), 40)
    for p, tab in enumerate(tabs):
        (sl,) = tab.pending_grads
        got = np.zeros((20, D), np.float32)
        np.add.at(got, H(sl.indices), H(sl.values))
        np.testing.assert_allclose(got, dense[20 * p:20 * (p + 1)], rtol=RTOL, atol=1e-5)


# ---- weighted / max_norm backward ------------------------------------------
def _slices_dense(sl, rows, D):
    n = sl.indices.numel() if sl.num_valid is None else int(sl.num_valid.item())
    idx, val = H(sl.indices[:n]), H(sl.values[:n])
    assert len(set(idx.tolist())) == n
    return dict(zip(idx.tolist(), val))


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
@pytest.mark.parametrize("case", ["weighted", "max_norm", "both"])
@pytest.mark.parametrize("holder", ["dense", "ev", "tensor"])
def test_weighted_max_norm_backward(dr, orc, comb, case, holder):
    rng = np.random.default_rng(zlib.crc32(("%s/%s/%s" % (comb, case, holder)).encode()))
    B, M, D, R = 150, 7, 24, 90
    ind, vals = _sparse(rng, B, M, R)
    table = (rng.standard_normal((R, D)) * 1.3).astype(np.float32)
    w = rng.uniform(0.1, 2.0, vals.shape[0]).astype(np.float32) if case != "max_norm" else None
    mn = 3.0 if case != "weighted" else None
    sp = dr.SparseTensor(T(ind), T(vals), (B, M))
    spw = None if w is None else dr.SparseTensor(T(ind), T(w), (B, M))
    if holder == "ev":
        params = dr.EmbeddingVariable("wmn_%s_%s" % (comb, case), D, 0.0)
        params.insert(T(np.arange(R)), T(table))
        oparams = orc.EV(D, 0.0)
        oparams.insert(np.arange(R, dtype=np.int64), table)
    elif holder == "dense":
        params = dr.DenseTable(T(table))
        oparams = table
    else:
        params = T(table).requires_grad_(True)
        oparams = table
    out = dr.embedding_lookup_sparse(params, sp, spw, combiner=comb, max_norm=mn)
    ref = orc.embedding_lookup_sparse(oparams, ind, vals, B, weights=w, combiner=comb,
                                      max_norm=mn)
    np.testing.assert_allclose(H(out), ref, rtol=RTOL, atol=1e-6)
    top = rng.standard_normal((B, D)).astype(np.float32)
    out.backward(T(top))
    uids, gref = orc.embedding_lookup_sparse_grad(oparams, ind, vals, B, top, w, comb, mn)
    if holder == "tensor":
        got = H(params.grad)[uids]
        other = np.setdiff1d(np.arange(R), uids)
        assert not H(params.grad)[other].any()
    else:
        (sl,) = params.pending_grads
        m = _slices_dense(sl, R, D)
        assert sorted(m) == sorted(uids.tolist())
        got = np.stack([m[u] for u in uids.tolist()])
    if mn is None:
        np.testing.assert_array_equal(got, gref)
    else:
        np.testing.assert_allclose(got, gref, rtol=RTOL, atol=1e-6)


# ---- partitioned EmbeddingVariables ----------------------------------------
@pytest.mark.parametrize("np_", [2, 3])
def test_partitioned_ev_lookup_and_train_step(dr, np_):
    """A fixed_size_partitioner EV (ids % 1000 % np) gives the single EV's
    forward, and one SGD step leaves every key's row where the single EV's
    step puts it (the ADVICE round-1 regression: no grads were queued)."""
    rng = np.random.default_rng(np_)
    B, M, D = 120, 5, 16
    ind, vals = _sparse(rng, B, M, 5000)
    vals = vals * 7 + 3                      # spread over id % 1000
    sp = dr.SparseTensor(T(ind), T(vals), (B, M))
    parts = dr.get_embedding_variable("pev%d" % np_, D, initializer=0.5, partitioner=np_)
    single = dr.EmbeddingVariable("pev_single%d" % np_, D, 0.5)
    opt = dr.GradientDescentOptimizer(0.1)
    top = T(rng.standard_normal((B, D)).astype(np.float32))
    for comb in ("mean", "sqrtn"):
        a = dr.embedding_lookup_sparse(parts, sp, combiner=comb)
        b = dr.embedding_lookup_sparse(single, sp, combiner=comb)
        np.testing.assert_array_equal(H(a), H(b))
        a.backward(top)
        b.backward(top)
        opt.apply_gradients(parts + [single], global_step=1)
    keys = np.unique(vals)
    got = np.zeros((keys.shape[0], D), np.float32)
    for p, ev in enumerate(parts):
        sel = keys[(keys % 1000) % np_ == p]
        got[np.searchsorted(keys, sel)] = H(ev.sparse_read(T(sel)))
        assert int(ev.total_count()[0]) == sel.shape[0]
    np.testing.assert_array_equal(got, H(single.sparse_read(T(keys))))


def test_partitioned_ev_counter_filter_counts(dr):
    """Counter admission sees each key's real batch frequency in every
    partition (counts dynamic-partitioned with the ids)."""
    D = 4
    opt = dr.EmbeddingVariableOption(filter_option=dr.CounterFilter(filter_freq=3))
    parts = dr.get_embedding_variable("pcf", D, initializer=1.0, ev_option=opt, partitioner=2)
    single = dr.EmbeddingVariable("pcf_single", D, 1.0, ev_option=opt)
    vals = np.array([1000, 1001, 1000, 1001, 1000, 7, 8, 8], np.int64)   # 1000 x3, 1001 x2
    ind = np.stack([np.arange(8), np.zeros(8)], 1).astype(np.int64)
    sp = dr.SparseTensor(T(ind), T(vals), (8, 1))
    with torch.no_grad():
        dr.embedding_lookup_sparse(parts, sp, combiner="sum")
        dr.embedding_lookup_sparse(single, sp, combiner="sum")
    for k in (1000, 1001, 7, 8):
        ev = parts[(k % 1000) % 2]
        fr, _, _ = ev.key_meta([k])
        sfr, _, _ = single.key_meta([k])
        assert fr.tolist() == sfr.tolist(), k


@pytest.mark.parametrize("strategy", ["mod", "div"])
def test_partitioned_dense_embedding_lookup(dr, strategy):
    rng = np.random.default_rng(4)
    rows, D = [11, 10, 10], 8
    R = sum(rows)
    full = rng.standard_normal((R, D)).astype(np.float32)
    ids = rng.integers(0, R, (37, 3)).astype(np.int64)
    if strategy == "mod":
        parts = [full[p::3] for p in range(3)]
    else:
        acc = np.cumsum([0] + rows)
        parts = [full[acc[p]:acc[p + 1]] for p in range(3)]
    tabs = [T(p).requires_grad_(True) for p in parts]
    out = dr.embedding_lookup(tabs, T(ids), partition_strategy=strategy)
    np.testing.assert_array_equal(H(out), full[ids])
    g = rng.standard_normal((37, 3, D)).astype(np.float32)
    out.backward(T(g))
    dense = np.zeros((R, D), np.float32)
    np.add.at(dense, ids.ravel(), g.reshape(-1, D))
    got = np.zeros_like(dense)
    if strategy == "mod":
        for p in range(3):
            got[p::3] = H(tabs[p].grad)
    else:
        acc = np.cumsum([0] + rows)
        for p in range(3):
            got[acc[p]:acc[p + 1]] = H(tabs[p].grad)
    np.testing.assert_allclose(got, dense, rtol=RTOL, atol=1e-6)
