"""GPU: the row-grouped lookup backward fused with the KV SGD update
(dr_ev_pool_grad_rows_apply_sgd, embedding_ops._RowsPending.apply_sgd).

When GradientDescentOptimizer.apply_gradients covers every EV of a lookup
whose gradient nothing else read, the backward runs fused with the update:
the same run sums (ascending positions; the same 8192-position pieces for
runs longer than that) and the same v -= lr * g roundings as forming the
IndexedSlices (dr_pool_grad_rows_grouped_ex) and applying them
(dr_ev_apply_grouped_ptr_rows), which is the reference composition
embedding_ops.py:592-675 -> KvResourceSparseApplyGradientDescent
(training_ali_ops.cc:1597-1678).  Every test runs the same steps both ways and
requires keys, values (and versions) bit-identical, and checks which path ran.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    deeprec_amd.set_validate(True)
    assert torch.cuda.is_available()
    return deeprec_amd


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


def H(t):
    return t.detach().cpu().numpy()


class _Fused(object):
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        from deeprec_amd import embedding_ops as eo
        self.old = eo._FUSED_SGD
        eo._FUSED_SGD = self.on

    def __exit__(self, *a):
        from deeprec_amd import embedding_ops as eo
        eo._FUSED_SGD = self.old


def _export(ev, versions=False):
    ex = ev.export()
    vals = ex[1].view(torch.int16) if ex[1].dtype == torch.bfloat16 else ex[1]
    k, v = H(ex[0]), H(vals)
    o = np.argsort(k)
    out = [k[o], v[o]]
    if versions:
        out.append(H(ex[2])[o])
    return out


def _onehot(ids):
    B = ids.size
    return np.stack([np.arange(B), np.zeros(B, np.int64)], 1), ids, (B, 1)


def _multihot(rng, B, H_, vocab):
    lens = rng.integers(0, H_ + 1, B)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(n) for n in lens]) if lens.sum() else np.zeros(0, np.int64)
    return (np.stack([rows, cols], 1).astype(np.int64),
            rng.integers(0, vocab, rows.shape[0]).astype(np.int64), (B, H_))


def _train(dr, fused, tag, batches, D, combiner, lr=0.05, dtype=torch.float32, stl=0,
           weighted=False, preinsert=0):
    from deeprec_amd.kv_variable_ops import PendingRowSlices
    F = len(batches[0][0])
    evs = [dr.EmbeddingVariable("%s_%d_%d" % (tag, int(fused), f), D, 0.05 * (f + 1),
                                steps_to_live=stl, value_dtype=dtype) for f in range(F)]
    # (preinsert: keys inserted one at a time, rows in key order; without it
    # parallel first-touch inserts number the rows in a racy order -- the
    # run sums do not depend on it, test_gpu_rows_deterministic.py)
    for e in evs:
        for k in range(preinsert):
            e.insert_synthetic(k, 1, seed=7)
    opt = dr.GradientDescentOptimizer(lr)
    outs = []
    with _Fused(fused):
        for step, (sps, g, ws) in enumerate(batches):
            st = [dr.SparseTensor(T(i), T(v), s) for i, v, s in sps]
            if weighted:
                assert F == 1
                i, v, s = sps[0]
                out = dr.embedding_lookup_sparse(evs[0], st[0],
                                                 sp_weights=dr.SparseTensor(T(i), T(ws[0]), s),
                                                 combiner=combiner)
            else:
                out = dr.embedding_lookup_sparse_multi(evs, st, combiner=combiner)
            out.backward(T(g[:, :out.shape[1]]))
            pend = [e.pending_grads[-1] for e in evs]
            # (unfused: formed eagerly, or launched on a side stream -- a
            # PendingRowSlices that is no longer fusable)
            assert all(isinstance(p, PendingRowSlices) and p.fusable() for p in pend) == fused
            opt.apply_gradients(evs, global_step=10 + step)
            if fused:   # ran fused: the IndexedSlices were never formed
                assert all(p._pending.applied and "indices" not in p.__dict__ for p in pend)
            assert all(not e.pending_grads for e in evs)
            outs.append(H(out.float()))
    torch.cuda.synchronize()
    dr.status_check()
    return outs, [_export(e, versions=stl != 0) for e in evs]


def _same(a, b):
    (o1, e1), (o2, e2) = a, b
    for x, y in zip(o1, o2):
        np.testing.assert_array_equal(x, y)
    for p, q in zip(e1, e2):
        for x, y in zip(p, q):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("D", [8, 16, 64, 128, 256, 1024])
def test_fused_sgd_onehot_sum_equals_unfused(dr, D):
    """One-hot sum over 3 tables, vocab small enough for many duplicate runs
    (and, D = 128, ids that repeat > 256 times: long runs, on EVs whose rows
    were numbered by racing first-touch inserts)."""
    rng = np.random.default_rng(D)
    B = 3000 if D < 1024 else 700
    vocab = 8 if D == 128 else 400
    batches = [([_onehot(rng.integers(0, vocab, B).astype(np.int64)) for _ in range(3)],
                rng.standard_normal((B, 3 * D)).astype(np.float32), None) for _ in range(3)]
    pre = 0
    _same(_train(dr, True, "fso%d" % D, batches, D, "sum", preinsert=pre),
          _train(dr, False, "fso%d" % D, batches, D, "sum", preinsert=pre))


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_fused_sgd_multihot_equals_unfused(dr, comb):
    """Multi-hot bags of 0..4 ids (empty bags, one-id bags of mean / sqrtn that
    go by address, longer bags that are scaled on the worklist)."""
    rng = np.random.default_rng(5)
    B, D = 700, 32
    batches = [([_multihot(rng, B, 4, 90) for _ in range(2)],
                rng.standard_normal((B, 2 * D)).astype(np.float32), None) for _ in range(3)]
    _same(_train(dr, True, "fsm" + comb, batches, D, comb),
          _train(dr, False, "fsm" + comb, batches, D, comb))


@pytest.mark.parametrize("comb", ["sum", "mean"])
def test_fused_sgd_weighted_equals_unfused(dr, comb):
    rng = np.random.default_rng(9)
    B, D = 400, 16
    batches = []
    for _ in range(3):
        sp = _multihot(rng, B, 5, 60)
        w = rng.uniform(0.5, 2.0, sp[1].size).astype(np.float32)
        batches.append(([sp], rng.standard_normal((B, D)).astype(np.float32), [w]))
    _same(_train(dr, True, "fsw" + comb, batches, D, comb, weighted=True),
          _train(dr, False, "fsw" + comb, batches, D, comb, weighted=True))


def test_fused_sgd_bf16_equals_unfused(dr):
    """bf16 EV rows: widened, updated in fp32, rounded to nearest even once."""
    rng = np.random.default_rng(17)
    B, D = 2000, 64
    batches = [([_onehot(rng.integers(0, 300, B).astype(np.int64)) for _ in range(2)],
                rng.standard_normal((B, 2 * D)).astype(np.float32), None) for _ in range(3)]
    _same(_train(dr, True, "fsb", batches, D, "sum", dtype=torch.bfloat16),
          _train(dr, False, "fsb", batches, D, "sum", dtype=torch.bfloat16))


def test_fused_sgd_stamps_versions(dr):
    """steps_to_live EVs: the fused update stamps version[row] = global_step
    as the apply does (LookupOrCreate with the global step)."""
    rng = np.random.default_rng(23)
    B, D = 500, 16
    batches = [([_onehot(rng.integers(0, 200 + 100 * s, B).astype(np.int64)) for _ in range(2)],
                rng.standard_normal((B, 2 * D)).astype(np.float32), None) for s in range(3)]
    a = _train(dr, True, "fsv", batches, D, "sum", stl=5)
    _same(a, _train(dr, False, "fsv", batches, D, "sum", stl=5))
    assert a[1][0][2].max() == 12


def test_fused_sgd_falls_back_when_gradient_is_read(dr):
    """Reading a pending gradient forms the IndexedSlices; the optimizer then
    applies them unfused, with the same result."""
    from deeprec_amd.kv_variable_ops import PendingRowSlices
    rng = np.random.default_rng(29)
    B, D = 600, 16
    sps = [_onehot(rng.integers(0, 100, B).astype(np.int64)) for _ in range(2)]
    g = rng.standard_normal((B, 2 * D)).astype(np.float32)
    res = []
    for peek in (True, False):
        evs = [dr.EmbeddingVariable("fsp_%d_%d" % (int(peek), f), D, 0.1) for f in range(2)]
        st = [dr.SparseTensor(T(i), T(v), s) for i, v, s in sps]
        out = dr.embedding_lookup_sparse_multi(evs, st, combiner="sum")
        out.backward(T(g))
        sl = evs[0].pending_grads[-1]
        assert isinstance(sl, PendingRowSlices)
        if peek:
            U = int(sl.num_valid.item())
            assert U == np.unique(sps[0][1]).size
            assert sl.values.shape == (B, D)
        dr.GradientDescentOptimizer(0.1).apply_gradients(evs)
        assert sl._pending.applied != peek
        torch.cuda.synchronize()
        res.append([_export(e) for e in evs])
    for p, q in zip(*res):
        for x, y in zip(p, q):
            np.testing.assert_array_equal(x, y)
    dr.status_check()


def test_fused_sgd_partial_var_list_and_shared_ev(dr):
    from deeprec_amd.kv_variable_ops import PendingRowSlices
    """apply_gradients over only some EVs of the group, and one EV used by
    two features of one lookup: both take the unfused path (the first forms
    the slices, the second applies them as sequential rounds)."""
    rng = np.random.default_rng(31)
    B, D = 300, 8
    ev_a = dr.EmbeddingVariable("fss_a", D, 0.1)
    ev_b = dr.EmbeddingVariable("fss_b", D, 0.1)
    sps = [_onehot(rng.integers(0, 50, B).astype(np.int64)) for _ in range(2)]
    st = [dr.SparseTensor(T(i), T(v), s) for i, v, s in sps]
    out = dr.embedding_lookup_sparse_multi([ev_a, ev_b], st, combiner="sum")
    out.backward(T(rng.standard_normal((B, 2 * D)).astype(np.float32)))
    sl = ev_a.pending_grads[-1]
    opt = dr.GradientDescentOptimizer(0.1)
    opt.apply_gradients([ev_a])
    assert not sl._pending.applied and not ev_a.pending_grads and ev_b.pending_grads
    opt.apply_gradients([ev_b])
    assert not ev_b.pending_grads
    ev_c = dr.EmbeddingVariable("fss_c", D, 0.1)
    out = dr.embedding_lookup_sparse_multi([ev_c, ev_c], st, combiner="sum")
    out.backward(T(rng.standard_normal((B, 2 * D)).astype(np.float32)))
    sl_c = ev_c.pending_grads[0]
    assert not (isinstance(sl_c, PendingRowSlices) and sl_c._pending.fusable())
    opt.apply_gradients([ev_c])
    torch.cuda.synchronize()
    dr.status_check()


def test_fused_sgd_graph_captured_equals_eager(dr):
    """Fused steps captured as one hipGraph and replayed = the same steps
    eager (the bench's train_step replays such a graph)."""
    rng = np.random.default_rng(37)
    B, D, F, S = 512, 32, 3, 4
    keys = [T(rng.integers(0, 3000, (F, B)).astype(np.int64)) for _ in range(S + 2)]
    ind = T(np.stack([np.arange(B), np.zeros(B, np.int64)], 1))
    ups = [T(rng.standard_normal((B, F * D)).astype(np.float32)) for _ in range(S + 2)]
    exports = []
    for graphed in (False, True):
        evs = [dr.EmbeddingVariable("fsg_%d_%d" % (int(graphed), f), D, 0.05, capacity=8192)
               for f in range(F)]
        opt = dr.GradientDescentOptimizer(0.1)

        def step(i):
            sps = [dr.SparseTensor(ind, keys[i][f], (B, 1)) for f in range(F)]
            out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
            out.backward(ups[i])
            opt.apply_gradients(evs, global_step=i)

        for i in range(2):
            step(i)
        torch.cuda.synchronize()
        if graphed:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(2, S + 2):
                    step(i)
            g.replay()
        else:
            for i in range(2, S + 2):
                step(i)
        torch.cuda.synchronize()
        dr.status_check()
        exports.append([_export(e) for e in evs])
    for p, q in zip(*exports):
        for x, y in zip(p, q):
            np.testing.assert_array_equal(x, y)


def test_lookup_table_order_flag_same_results(dr):
    """DR_LOOKUP_TABLE_ORDER (visit the feature-major ids table by table)
    gives the output order's outputs and row records bit for bit on the same
    EVs.  Each order runs first on one EV set (creating the new keys: the
    miss path) and second on the other (all hits)."""
    import ctypes as C
    from deeprec_amd._lib import LOOKUP_TABLE_ORDER, check, lib, ptr, stream_handle
    rng = np.random.default_rng(3)
    T_, B, D = 5, 3000, 32
    ids = T(rng.integers(0, 2600, (T_, B)).astype(np.int64))

    def run(evs, flags):
        out = torch.empty((B, T_ * D), device=DEV)
        rows = torch.empty(T_ * B, dtype=torch.int64, device=DEV)
        handles = (C.c_void_p * T_)(*[e.handle.value for e in evs])
        wsb = lib().dr_ev_lookup_onehot_workspace_size(T_, B)
        ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
        check(lib().dr_ev_lookup_onehot_ex(handles, T_, ptr(ids), 1, B, B, ptr(out), T_ * D, 0,
                                           flags, ptr(rows), ptr(ws), wsb, stream_handle(DEV)))
        torch.cuda.synchronize()
        dr.status_check()
        return H(out), H(rows)

    for first in (0, LOOKUP_TABLE_ORDER):
        evs = [dr.EmbeddingVariable("tord_%d_%d" % (first, t), D, 0.3) for t in range(T_)]
        for t, e in enumerate(evs):
            e.insert_synthetic(0, 2000, seed=40 + t)   # ids >= 2000 are new: misses
        o1, r1 = run(evs, first)
        o2, r2 = run(evs, LOOKUP_TABLE_ORDER - first)
        np.testing.assert_array_equal(o1, o2)
        np.testing.assert_array_equal(r1, r2)
