"""The registered op layer (torch.ops.deeprec.*) on the GPU: results equal the
package functions / the oracle, torch.library.opcheck passes (schema, fake
tensor and autograd registration), and a function built from the ops traces
into an FX graph of deeprec ops (make_fx, fake tensors)."""
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
    return deeprec_amd


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


def H(t):
    return t.detach().cpu().numpy()


def _sparse(rng, B, M, vocab):
    lens = rng.integers(1, M + 1, B)
    r = np.repeat(np.arange(B), lens)
    c = np.concatenate([np.arange(n) for n in lens])
    return np.stack([r, c], 1).astype(np.int64), rng.integers(0, vocab, r.shape[0]).astype(np.int64)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
@pytest.mark.parametrize("weighted", [False, True])
def test_embedding_lookup_sparse_op(dr, orc, comb, weighted):
    rng = np.random.default_rng(7)
    B, D, R = 90, 16, 60
    ind, vals = _sparse(rng, B, 5, R)
    table = rng.standard_normal((R, D)).astype(np.float32)
    w = rng.uniform(0.2, 2, vals.shape[0]).astype(np.float32) if weighted else None
    t = T(table).requires_grad_(True)
    out = torch.ops.deeprec.embedding_lookup_sparse(t, T(ind), T(vals), B,
                                                    None if w is None else T(w), comb, 2.5)
    ref = orc.embedding_lookup_sparse(table, ind, vals, B, weights=w, combiner=comb, max_norm=2.5)
    np.testing.assert_allclose(H(out), ref, rtol=1e-5, atol=1e-6)
    top = rng.standard_normal((B, D)).astype(np.float32)
    out.backward(T(top))
    uids, gu = orc.embedding_lookup_sparse_grad(table, ind, vals, B, top, w, comb, 2.5)
    np.testing.assert_allclose(H(t.grad)[uids], gu, rtol=1e-5, atol=1e-6)


def test_kv_ops_match_package(dr, orc):
    rng = np.random.default_rng(8)
    D = 8
    ev = dr.EmbeddingVariable("tops_kv", D, 0.25)
    keys = np.arange(0, 400, 3, dtype=np.int64)
    vals = rng.standard_normal((keys.shape[0], D)).astype(np.float32)
    torch.ops.deeprec.kv_resource_insert(ev.resource, T(keys), T(vals))
    q = np.concatenate([keys[:50], np.array([1, 2, 1000], np.int64)])
    got = torch.ops.deeprec.kv_resource_gather(ev.resource, T(q), D)
    np.testing.assert_array_equal(H(got), H(ev.sparse_read(T(q))))
    acc = ev.slot("Adagrad", 0.1)
    oev = orc.EV(D, 0.25)
    oev.insert(keys, vals)
    oev.gather(np.array([1, 2, 1000], np.int64))
    oacc = oev.create_slot(1, np.full(D, 0.1, np.float32))
    uq = np.unique(q)
    gq = rng.standard_normal((uq.shape[0], D)).astype(np.float32)
    torch.ops.deeprec.kv_resource_sparse_apply_adagrad(ev.resource, acc.resource, 0.1,
                                                       T(gq), T(uq), 3)
    oev.apply_adagrad(oacc, np.float32(0.1), gq, uq, 3)
    np.testing.assert_allclose(H(ev.sparse_read(T(uq))), oev.gather(uq), rtol=1e-5, atol=1e-7)


def test_opcheck(dr):
    from torch.library import opcheck
    rng = np.random.default_rng(9)
    utils = ("test_schema", "test_faketensor", "test_autograd_registration")
    data = T(rng.standard_normal((12, 6)).astype(np.float32)).requires_grad_(True)
    idx = T(np.array([0, 3, 3, 7, 11, 2], np.int32))
    seg = T(np.array([0, 0, 1, 1, 3, 3], np.int32))
    opcheck(torch.ops.deeprec.sparse_segment_reduce.default, (data, idx, seg, 4, "mean"),
            test_utils=utils)
    opcheck(torch.ops.deeprec.unsorted_segment_sum.default, (data, T(np.arange(12) % 5, torch.int32), 5),
            test_utils=utils)
    opcheck(torch.ops.deeprec.resource_gather.default, (data, T(np.array([1, 5, 5, 0]))),
            test_utils=utils)
    emb = T(rng.standard_normal((5, 4, 8)).astype(np.float32)).requires_grad_(True)
    opcheck(torch.ops.deeprec.fm_second_order.default, (emb,), test_utils=utils)
    opcheck(torch.ops.deeprec.dot_interaction.default, (emb,), test_utils=utils)
    ind, vals = _sparse(rng, 10, 4, 12)
    opcheck(torch.ops.deeprec.embedding_lookup_sparse.default,
            (data, T(ind), T(vals), 10, None, "sqrtn", -1.0), test_utils=utils)


def test_trace_to_fx_graph(dr):
    from torch.fx.experimental.proxy_tensor import make_fx
    rng = np.random.default_rng(10)
    ind, vals = _sparse(rng, 16, 3, 40)
    table = T(rng.standard_normal((40, 8)).astype(np.float32))

    def model(tab, ind, vals):
        e = torch.ops.deeprec.embedding_lookup_sparse(tab, ind, vals, 16, None, "mean", -1.0)
        x = torch.stack([e, e * 2.0, e + 1.0], 1)
        return torch.ops.deeprec.dot_interaction(x)

    gm = make_fx(model, tracing_mode="fake")(table, T(ind), T(vals))
    targets = [str(n.target) for n in gm.graph.nodes if n.op == "call_function"]
    assert "deeprec.embedding_lookup_sparse.default" in targets
    assert "deeprec.dot_interaction.default" in targets
    np.testing.assert_array_equal(H(gm(table, T(ind), T(vals))), H(model(table, T(ind), T(vals))))


def test_ev_lookup_op_matches_oracle(dr, orc):
    """torch.ops.deeprec.kv_embedding_lookup_sparse -- the EV-backed hot-path
    op (EmbeddingVariable.sparse_read -> KvResourceGather inside
    embedding_lookup_sparse, kv_variable_ops.py:644-664) in one C call --
    equals the oracle's composition, and its grad op equals the reference
    SparseSegment*Grad IndexedSlices."""
    rng = np.random.default_rng(12)
    B, D = 128, 16
    ev = dr.EmbeddingVariable("tops_evl", D, 0.25)
    oev = orc.EV(D, 0.25)
    keys = np.arange(0, 90, dtype=np.int64)
    vals0 = rng.standard_normal((90, D)).astype(np.float32)
    ev.insert(T(keys), T(vals0))
    oev.insert(keys, vals0)
    ind, vals = _sparse(rng, B, 4, 120)
    for comb in ("sum", "mean", "sqrtn"):
        out = torch.ops.deeprec.kv_embedding_lookup_sparse(ev.resource, T(ind), T(vals), B, D,
                                                           None, comb)
        ref = orc.embedding_lookup_sparse(oev, ind, vals, B, None, comb)
        np.testing.assert_array_equal(H(out), ref)
        g = rng.standard_normal((B, D)).astype(np.float32)
        u, gr, nu = torch.ops.deeprec.kv_embedding_lookup_sparse_grad(T(ind), T(vals), B, T(g),
                                                                      None, comb)
        U = int(nu.item())
        uids, gref = orc.embedding_lookup_sparse_grad(oev, ind, vals, B, g, None, comb)
        assert H(u[:U]).tolist() == uids.tolist()
        np.testing.assert_array_equal(H(gr[:U]), gref)


def _np_prune_fill(ind, v, w, B, comb, default_id, prune=True):
    """_prune_invalid_ids [/ _prune_invalid_weights] + sparse_fill_empty_rows
    (embedding_ops.py:1289-1310) in numpy: (ind, ids, weights, empty rows)."""
    keep = v >= 0 if prune else np.ones(v.shape, bool)
    if prune and w is not None and comb != "sum":
        keep &= w > 0
    ind, v = ind[keep], v[keep]
    w = None if w is None else w[keep]
    empty = np.ones(B, bool)
    empty[ind[:, 0]] = False
    fill = np.nonzero(empty)[0]
    ind2 = np.concatenate([ind, np.stack([fill, np.zeros_like(fill)], 1)])
    v2 = np.concatenate([v, np.full(fill.size, default_id or 0, np.int64)])
    o = np.argsort(ind2[:, 0], kind="stable")
    w2 = None if w is None else np.concatenate([w, np.ones(fill.size, np.float32)])[o]
    return ind2[o], v2[o], w2, empty


@pytest.mark.parametrize("safe,default_id", [(False, -1), (True, -1), (True, 2)])
@pytest.mark.parametrize("max_norm", [-1.0, 0.9])
@pytest.mark.parametrize("weighted", [False, True])
def test_ev_lookup_grad_op_safe_and_max_norm(dr, orc, safe, default_id, max_norm, weighted):
    """The registered grad op takes the forward's safe / default_id / prune /
    max_norm: pruned ids get no gradient, the filled id gets its rows'
    gradient (zeroed rows when default_id is None), and the max_norm clip's
    chain rule is applied at the EV's rows -- against the oracle's gradient
    of the same pruned / filled lookup."""
    rng = np.random.default_rng(100 + 7 * safe + int(max_norm > 0) + 3 * weighted + default_id)
    B, D, comb = 96, 8, "mean"
    ev = dr.EmbeddingVariable("tops_sg_%d_%d_%d_%d" % (safe, default_id, max_norm > 0, weighted),
                              D, 0.2)
    oev = orc.EV(D, 0.2)
    keys = np.arange(0, 60, dtype=np.int64)
    vals0 = rng.standard_normal((60, D)).astype(np.float32)
    ev.insert(T(keys), T(vals0))
    oev.insert(keys, vals0)
    lens = rng.integers(0 if safe else 1, 5, B)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(l) for l in lens])
    ind = np.stack([rows, cols], 1).astype(np.int64)
    v = rng.integers(0, 80, rows.shape[0]).astype(np.int64)
    if safe:
        v[::6] = -1
    w = rng.uniform(-0.3, 2.0, v.shape[0]).astype(np.float32) if weighted else None
    if weighted and not safe:
        w = np.abs(w) + 0.1
    Wt = None if w is None else T(w)
    out = torch.ops.deeprec.kv_embedding_lookup_sparse(ev.resource, T(ind), T(v), B, D, Wt, comb,
                                                       max_norm, safe, default_id)
    did = None if default_id < 0 else default_id
    mn = None if max_norm < 0 else max_norm
    if safe:
        ref = orc.safe_embedding_lookup_sparse(oev, ind, v, (B, 5), w, comb, did, mn)
    else:
        ref = orc.embedding_lookup_sparse(oev, ind, v, B, w, comb, mn)
    np.testing.assert_allclose(H(out), ref, rtol=1e-5, atol=1e-6)
    g = rng.standard_normal((B, D)).astype(np.float32)
    u, gr, nu = torch.ops.deeprec.kv_embedding_lookup_sparse_grad(
        T(ind), T(v), B, T(g), Wt, comb, ev.resource, max_norm, safe, default_id)
    U = int(nu.item())
    if safe:
        ind2, v2, w2, empty = _np_prune_fill(ind, v, w, B, comb, did)
        g2 = g.copy()
        if did is None:
            g2[empty] = 0.0
    else:
        ind2, v2, w2, g2 = ind, v, w, g
    uids, gref = orc.embedding_lookup_sparse_grad(oev, ind2, v2, B, g2, w2, comb, mn)
    assert H(u[:U]).tolist() == uids.tolist()
    assert (H(u[:U]) >= 0).all()                    # pruned ids never reach the slices
    if mn is None and not weighted:
        np.testing.assert_array_equal(H(gr[:U]), gref)
    else:
        np.testing.assert_allclose(H(gr[:U]), gref, rtol=1e-5, atol=1e-6)


def test_compile_keeps_stateful_order(dr, orc):
    """Under torch.compile (aot_eager: functionalization of the custom ops),
    a lookup -> grad -> SGD apply -> lookup chain on one EV keeps every
    stateful op, in program order: the second lookup sees the update, bit for
    bit what eager execution gives, and the traced graph holds one apply
    between the two lookups."""
    rng = np.random.default_rng(13)
    B, D, lr = 64, 8, 0.5
    ind, vals = _sparse(rng, B, 3, 50)
    g = T(rng.standard_normal((B, D)).astype(np.float32))
    def step(res, ind_t, vals_t, g):
        a = torch.ops.deeprec.kv_embedding_lookup_sparse(res, ind_t, vals_t, B, D, None, "sum")
        u, gr, nu = torch.ops.deeprec.kv_embedding_lookup_sparse_grad(ind_t, vals_t, B, g, None,
                                                                      "sum")
        torch.ops.deeprec.kv_resource_sparse_apply_gradient_descent(res, lr, gr, u, 1, nu)
        b = torch.ops.deeprec.kv_embedding_lookup_sparse(res, ind_t, vals_t, B, D, None, "sum")
        return a, b

    outs = []
    for mode in ("eager", "compiled"):
        ev = dr.EmbeddingVariable("tops_cmp_" + mode, D, 0.1)
        ev.insert(T(np.arange(50, dtype=np.int64)),
                  T(np.random.default_rng(3).standard_normal((50, D)).astype(np.float32)))
        fn = step if mode == "eager" else torch.compile(step, backend="aot_eager", fullgraph=True)
        a, b = fn(ev.resource, T(ind), T(vals), g)
        torch.cuda.synchronize()
        outs.append((H(a), H(b)))
        assert not np.array_equal(H(a), H(b))          # the apply ran before the 2nd lookup
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    # the same chain captured by make_fx keeps one apply between two lookups
    from torch.fx.experimental.proxy_tensor import make_fx
    ev = dr.EmbeddingVariable("tops_cmp_fx", D, 0.1)
    gm = make_fx(step, tracing_mode="real")(ev.resource, T(ind), T(vals), g)
    seq = [str(n.target) for n in gm.graph.nodes if n.op == "call_function"
           and "deeprec.kv_" in str(n.target)]
    assert seq == ["deeprec.kv_embedding_lookup_sparse.default",
                   "deeprec.kv_embedding_lookup_sparse_grad.default",
                   "deeprec.kv_resource_sparse_apply_gradient_descent.default",
                   "deeprec.kv_embedding_lookup_sparse.default"], seq
