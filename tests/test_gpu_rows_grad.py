"""GPU: the row-grouped training backward (dr_pool_grad_rows_grouped) and the
by-address EV applies (dr_ev_apply_grouped_ptr / _ftrl_grouped_ptr).

The training forward of filter-free EVs skips the Unique and the backward
regroups by the resolved rows.  It must give the IndexedSlices the Unique
path gives -- unique ids in first-occurrence order (Unique's order, bit-exact
vs the oracle), U_t, and the SparseSegment*Grad values (bit-exact for runs of
<= 256 positions) -- and the optimizer reading the gradient rows by address
must leave the EVs bit-identical to the value-block apply.
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


class _Path(object):
    """Select the training path of embedding_ops for a block."""

    def __init__(self, rows):
        self.rows = rows

    def __enter__(self):
        from deeprec_amd import embedding_ops as eo
        self.old = eo._ROWS_GRAD
        eo._ROWS_GRAD = self.rows

    def __exit__(self, *a):
        from deeprec_amd import embedding_ops as eo
        eo._ROWS_GRAD = self.old


def _sparse(rng, B, H_, vocab, allow_empty=False):
    lo = 0 if allow_empty else 1
    lens = rng.integers(lo, H_ + 1, B)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(n) for n in lens]) if lens.sum() else np.zeros(0, np.int64)
    ind = np.stack([rows, cols], 1).astype(np.int64)
    v = rng.integers(0, vocab, rows.shape[0]).astype(np.int64)
    return ind, v, (B, H_)


def _feature_set(dr, rng, tag, F, B, D, onehot, vocab, shared_keys):
    evs, sps, raw = [], [], []
    for f in range(F):
        evs.append(dr.EmbeddingVariable("%s_%d" % (tag, f), D, 0.1 * (f + 1)))
        if onehot:
            ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
            v = (shared_keys if shared_keys is not None else
                 rng.integers(0, vocab, B).astype(np.int64))
            shape = (B, 1)
        else:
            ind, v, shape = _sparse(rng, B, 5, vocab, allow_empty=True)
        sps.append(dr.SparseTensor(T(ind), T(v), shape))
        raw.append((ind, v))
    return evs, sps, raw


@pytest.mark.parametrize("D", [32, 1, 18])
@pytest.mark.parametrize("onehot", [True, False])
@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_rows_backward_matches_segment_grad(dr, orc, onehot, comb, D):
    """Grouped rows path vs the oracle Unique + SparseSegment*Grad: indices
    (first-occurrence order), U and values bit-exact.  Every feature inserts
    the same keys in the same order, so equal rows recur across tables (the
    regrouping must split runs at table boundaries)."""
    # D = 1 / 18: unaligned rows (wide tables; every run through the
    # worklist, one-position runs on its single-row path)
    rng = np.random.default_rng(101 + int(onehot))
    B, F = 300, 4
    shared = rng.integers(0, 90, B).astype(np.int64) if onehot else None
    evs, sps, raw = _feature_set(dr, rng, "rbw_%d_%s_%d" % (int(onehot), comb, D), F, B, D,
                                 onehot, 120, shared)
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner=comb)
    g = rng.standard_normal((B, F * D)).astype(np.float32)
    out.backward(T(g))
    for f in range(F):
        sl = evs[f].pending_grads.pop()
        assert sl.grad_ptr is not None          # the rows path ran
        U = int(sl.num_valid.item())
        uids, idx = orc.unique(raw[f][1])
        assert U == uids.size
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        ref = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g[:, f * D:(f + 1) * D]), idx,
                                             raw[f][0][:, 0].astype(np.int32), U, comb)
        np.testing.assert_array_equal(H(sl.values[:U]), ref)


@pytest.mark.parametrize("D", [16, 1])
def test_rows_backward_single_feature_weighted(dr, orc, D):
    """One EV feature with weights (embedding_lookup_sparse, not the multi
    API) through the rows path: the weighted grad is materialised (D = 1:
    formed in the emit pass, no worklist)."""
    rng = np.random.default_rng(7)
    B = 80
    for comb in ("sum", "mean", "sqrtn"):
        ev = dr.EmbeddingVariable("rw_%s_%d" % (comb, D), D, 0.2)
        ind, v, shape = _sparse(rng, B, 6, 50)
        w = rng.uniform(0.5, 2.0, v.size).astype(np.float32)
        out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), shape),
                                         sp_weights=dr.SparseTensor(T(ind), T(w), shape),
                                         combiner=comb)
        g = rng.standard_normal((B, D)).astype(np.float32)
        out.backward(T(g))
        sl = ev.pending_grads.pop()
        U = int(sl.num_valid.item())
        got = H(sl.values[:U])
        keys = H(sl.indices[:U])
        # the same lookup on the Unique path is the reference of this check
        ev2 = dr.EmbeddingVariable("rw2_%s_%d" % (comb, D), D, 0.2)
        with _Path(False):
            out2 = dr.embedding_lookup_sparse(ev2, dr.SparseTensor(T(ind), T(v), shape),
                                              sp_weights=dr.SparseTensor(T(ind), T(w), shape),
                                              combiner=comb)
            out2.backward(T(g))
        sl2 = ev2.pending_grads.pop()
        assert sl2.grad_ptr is None
        U2 = int(sl2.num_valid.item())
        assert U == U2 and keys.tolist() == H(sl2.indices[:U]).tolist()
        np.testing.assert_array_equal(got, H(sl2.values[:U]))
        np.testing.assert_array_equal(H(out), H(out2))


@pytest.mark.parametrize("walker", ["1", "0", "2"])
@pytest.mark.parametrize("D", [18, 32, 1])
def test_rows_backward_long_runs(dr, orc, D, walker):
    """Hot ids on the rows path: runs of 5000 / 256 / 257 / 768 / 200 / 511 /
    8192 / 8193 / 20000 / 21846 / 65536 positions.  Every run is ONE serial
    chain in ascending position order, one piece per run, through each
    walker (DR_GRAD_SERIAL_PLAIN 1: rows_serial_plain_kernel, the default;
    0: rows_serial_kernel; 2: rows_serial_dma_kernel): bit-equal to the
    reference's serial sum at any length."""
    import os
    os.environ["DR_GRAD_SERIAL_PLAIN"] = walker
    try:
        _long_runs_case(dr, orc, D, walker)
    finally:
        del os.environ["DR_GRAD_SERIAL_PLAIN"]


def _long_runs_case(dr, orc, D, walker):
    rng = np.random.default_rng(41)
    runs = {0: 5000, 1: 256, 2: 257, 3: 768, 4: 200, 5: 511, 6: 8192, 7: 8193, 8: 20000,
            9: 21846, 10: 65536}
    v = np.concatenate([np.full(n, k, np.int64) for k, n in runs.items()] +
                       [rng.integers(11, 400, 3000).astype(np.int64)])
    rng.shuffle(v)
    B = v.size
    evs, sps = [], []
    for f in range(3):
        evs.append(dr.EmbeddingVariable("rlong_%d_%d_%s" % (D, f, walker), D, 0.1,
                                        capacity=1024))
        ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
        sps.append(dr.SparseTensor(T(ind), T(v), (B, 1)))
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
    g = rng.standard_normal((B, 3 * D)).astype(np.float32)
    out.backward(T(g))
    uids, idx = orc.unique(v)
    seg = np.arange(B, dtype=np.int32)
    for f in range(3):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        gf = np.ascontiguousarray(g[:, f * D:(f + 1) * D])
        ref = orc.sparse_segment_reduce_grad(gf, idx, seg, U, "sum")
        np.testing.assert_array_equal(H(sl.values[:U]), ref)
    dr.status_check()


def _repeated_terms(rng, n, D):
    """n gradient rows in blocks of identical rows (lengths 1..259) whose
    values stress the closed-form walk: normals over six decades, dyadic
    integers (exact sums, rounding ties later), odd multiples of 2^(e-24)
    (ties against sums of binade e), tiny and huge values, zeros of both
    signs, and sign flips that drive the sum through zero."""
    rows = np.empty((n, D), np.float32)
    i = 0
    prev = np.zeros(D, np.float32)
    while i < n:
        m = min(int(rng.integers(1, 260)), n - i)
        kind = int(rng.integers(0, 8))
        if kind == 0:
            r = rng.standard_normal(D) * 10.0 ** rng.uniform(-3, 3)
        elif kind == 1:
            r = rng.integers(-64, 65, D) * 2.0 ** -12
        elif kind == 2:
            r = (2 * rng.integers(-40, 40, D) + 1) * 2.0 ** (rng.integers(-10, 10, D) - 24)
        elif kind == 3:
            r = rng.choice([1e-30, -1e-30, 0.0, -0.0, 1e6, -1e6], D)
        elif kind == 4:
            r = -prev * rng.integers(1, 4, D)
        else:
            r = rng.standard_normal(D).astype(np.float32)
        prev = np.asarray(r, np.float32)
        rows[i:i + m] = prev
        i += m
    return rows


def _seg_env(monkeypatch, seg):
    """"4096": segment scan, wave-rounds walk (DR_GRAD_SEG_ROUNDS=1, opt-in);
    "4096/r0": segment scan, one rep_add per segment (round 5's walk); "0": no
    scan, the plain walk (the default)."""
    s, _, r = seg.partition("/")
    monkeypatch.setenv("DR_GRAD_SEG_SCAN", s)
    monkeypatch.setenv("DR_GRAD_SEG_ROUNDS", "0" if r == "r0" else "1")


@pytest.mark.parametrize("seg", ["4096", "4096/r0", "0"])
@pytest.mark.parametrize("D", [18, 32, 1])
def test_rows_backward_repeated_terms(dr, orc, D, seg, monkeypatch):
    """Long runs whose terms come in blocks of identical rows (DIN's padding
    id: every padded position of a sample carries that sample's his_sum
    gradient).  With the segment scan on (DR_GRAD_SEG_SCAN=4096, opt-in) a
    run of such blocks is walked one block at a time in closed form
    (rows_serial_seg_kernel + rep_add); off (0, the default), position by
    position.
    Both bit-equal to the reference's serial sum; a long run without
    repeats rides along (scanned, then walked plainly).  Round 6: the
    segments walked by a whole wave in rounds (wave_rounds_walk, DR_GRAD_SEG_ROUNDS=1),
    the round-5 walk one segment at a time ("4096/r0")."""
    _seg_env(monkeypatch, seg)
    rng = np.random.default_rng(61 + D)
    v = np.concatenate([np.zeros(60000, np.int64), np.ones(5000, np.int64),
                        rng.integers(2, 300, 4000).astype(np.int64)])
    rng.shuffle(v)
    B = v.size
    g = rng.standard_normal((B, 3 * D)).astype(np.float32)
    pos0 = np.nonzero(v == 0)[0]
    for f in range(3):
        g[pos0, f * D:(f + 1) * D] = _repeated_terms(rng, pos0.size, D)
    evs, sps = [], []
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    for f in range(3):
        evs.append(dr.EmbeddingVariable("rrep_%d_%d_%s" % (D, f, seg.replace("/", "")), D, 0.1,
                                        capacity=1024))
        sps.append(dr.SparseTensor(T(ind), T(v), (B, 1)))
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
    out.backward(T(g))
    uids, idx = orc.unique(v)
    segs = np.arange(B, dtype=np.int32)
    for f in range(3):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        gf = np.ascontiguousarray(g[:, f * D:(f + 1) * D])
        ref = orc.sparse_segment_reduce_grad(gf, idx, segs, U, "sum")
        np.testing.assert_array_equal(H(sl.values[:U]).view(np.uint32), ref.view(np.uint32))
    dr.status_check()


def test_rows_sgd_repeated_terms_seg_equals_plain(dr, monkeypatch):
    """The fused SGD backward (dr_ev_pool_grad_rows_apply_sgd, 16-B rows)
    over blocks of repeated terms: the segment walk and the plain walk leave
    bit-identical EVs after two steps."""
    rng = np.random.default_rng(67)
    D, B = 32, 40000
    v = np.concatenate([np.zeros(36000, np.int64), rng.integers(1, 200, B - 36000)])
    rng.shuffle(v)
    gs = []
    for _ in range(2):
        g = rng.standard_normal((B, D)).astype(np.float32)
        g[np.nonzero(v == 0)[0]] = _repeated_terms(rng, int((v == 0).sum()), D)
        gs.append(g)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    res = []
    for seg in ("4096", "4096/r0", "0"):
        _seg_env(monkeypatch, seg)
        ev = dr.EmbeddingVariable("rrep_sgd_%s" % seg.replace("/", ""), D, 0.1, capacity=1024)
        opt = dr.GradientDescentOptimizer(0.05)
        for step, g in enumerate(gs):
            out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 1)),
                                             combiner="sum")
            out.backward(T(g))
            opt.apply_gradients([ev], global_step=step)
        torch.cuda.synchronize()
        res.append(_export(ev))
    (k1, v1) = res[0]
    for k2, v2 in res[1:]:
        np.testing.assert_array_equal(k1, k2)
        np.testing.assert_array_equal(v1.view(np.uint32), v2.view(np.uint32))


@pytest.mark.parametrize("seg", ["4096", "0"])
def test_rows_backward_din_padding_chain(dr, orc, seg, monkeypatch):
    """DIN's padding id at configs[3]'s size: ~4 000 samples, each adding its
    his_sum gradient row at every padded position (1..99 identical terms,
    normal values of both signs -- the running sum walks through zero and
    across binades), 2 x 10^5 positions in one run, D = 18: the wave-rounds
    segment walk (opt-in) and the plain walk bit-equal to the reference's
    serial sum."""
    _seg_env(monkeypatch, seg)
    rng = np.random.default_rng(2024)
    D, S = 18, 4000
    k = rng.integers(1, 100, S)
    terms = (rng.standard_normal((S, D)) * 10.0 ** rng.uniform(-6, -3, (S, 1))).astype(np.float32)
    n0 = int(k.sum())
    g0 = np.repeat(terms, k, axis=0)
    other = rng.integers(1, 5000, 30000).astype(np.int64)
    v = np.concatenate([np.zeros(n0, np.int64), other])
    g = np.concatenate([g0, rng.standard_normal((other.size, D)).astype(np.float32)])
    B = v.size
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    # the mid / cat pair of DIN's item lookup: two EVs, one grouped lookup
    evs = [dr.EmbeddingVariable("rdin_%s_%d" % (seg, f), D, 0.1, capacity=8192) for f in range(2)]
    gg = np.concatenate([g, g[::-1].copy()], 1)
    out = dr.embedding_lookup_sparse_multi(
        evs, [dr.SparseTensor(T(ind), T(v), (B, 1)) for _ in range(2)], combiner="sum")
    out.backward(T(gg))
    uids, idx = orc.unique(v)
    for f in range(2):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        gf = np.ascontiguousarray(gg[:, f * D:(f + 1) * D])
        ref = orc.sparse_segment_reduce_grad(gf, idx, np.arange(B, dtype=np.int32), U, "sum")
        np.testing.assert_array_equal(H(sl.values[:U]).view(np.uint32), ref.view(np.uint32))
    dr.status_check()


@pytest.mark.parametrize("side", [True, False])
def test_rows_backward_side_stream(dr, orc, side, monkeypatch):
    """Row-grouped backwards not fused into an SGD apply run on a side stream
    (DR_ROWS_SIDE_STREAM, default on), joined when their slices are first
    read: three separate lookups with long runs (D = 18, so no fused SGD),
    their backwards in flight together, the top gradient dropped and the
    allocator churned on the main stream before the slices are read --
    bit-equal to the reference's serial sums either way."""
    from deeprec_amd import embedding_ops
    monkeypatch.setattr(embedding_ops, "_SIDE_STREAM", side)
    rng = np.random.default_rng(43)
    D = 18
    runs = {0: 30000, 1: 257, 2: 9000, 3: 65536}
    v = np.concatenate([np.full(n, k, np.int64) for k, n in runs.items()] +
                       [rng.integers(4, 300, 5000).astype(np.int64)])
    rng.shuffle(v)
    B = v.size
    evs, outs = [], []
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    for f in range(3):
        ev = dr.EmbeddingVariable("rside_%d_%d" % (f, side), D, 0.1, capacity=1024)
        evs.append(ev)
        outs.append(dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 1)),
                                               combiner="sum"))
    g = rng.standard_normal((B, 3 * D)).astype(np.float32)
    gt = T(g)
    torch.cat(outs, 1).backward(gt)
    del gt, outs
    for _ in range(4):   # main-stream allocations that would reuse freed buffers
        torch.full((B, 3 * D), float("nan"), device="cuda").mul_(2.0)
    uids, idx = orc.unique(v)
    seg = np.arange(B, dtype=np.int32)
    for f in range(3):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        gf = np.ascontiguousarray(g[:, f * D:(f + 1) * D])
        ref = orc.sparse_segment_reduce_grad(gf, idx, seg, U, "sum")
        np.testing.assert_array_equal(H(sl.values[:U]), ref)
    dr.status_check()


@pytest.mark.parametrize("D", [18, 32])
def test_rows_backward_long_runs_zero_terms(dr, orc, D):
    """Long runs whose terms are mostly exact zeros (a padding id whose
    positions are masked out downstream: their gradients are +-0.0): with the
    zero scan on (DR_GRAD_ZERO_SKIP=1, opt-in) the serial walk skips the zero
    terms of a zero-started chain (rows_nz_kernel) -- bit-equal to the full
    serial sum, signs included: a run of only zero terms (+0.0 and -0.0) is
    +0.0, as 0 + (-0) + ... is in the reference's loop."""
    import os
    os.environ["DR_GRAD_ZERO_SKIP"] = "1"
    try:
        _zero_terms_case(dr, orc, D)
    finally:
        del os.environ["DR_GRAD_ZERO_SKIP"]


def _zero_terms_case(dr, orc, D):
    rng = np.random.default_rng(45)
    runs = {0: 30000, 1: 9000, 2: 40000, 3: 5000}
    v = np.concatenate([np.full(n, k, np.int64) for k, n in runs.items()] +
                       [rng.integers(4, 300, 2000).astype(np.int64)])
    rng.shuffle(v)
    B = v.size
    g = rng.standard_normal((B, 2 * D)).astype(np.float32)
    zero = (v == 0) & (rng.random(B) < 0.9)       # 90 % of run 0: zero rows
    g[zero] = 0.0
    g[zero & (rng.random(B) < 0.5)] = -0.0        # half of them -0.0
    g[v == 2] = np.where(rng.random((int((v == 2).sum()), 2 * D)) < 0.5, -0.0, 0.0)  # only zeros
    sel = np.flatnonzero(v == 1)[::7]
    g[sel, :D] = 0.0                                # partly zero rows stay in the walk
    evs, sps = [], []
    for f in range(2):
        evs.append(dr.EmbeddingVariable("rzero_%d_%d" % (D, f), D, 0.1, capacity=1024))
        ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
        sps.append(dr.SparseTensor(T(ind), T(v), (B, 1)))
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
    out.backward(T(g))
    uids, idx = orc.unique(v)
    seg = np.arange(B, dtype=np.int32)
    for f in range(2):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        gf = np.ascontiguousarray(g[:, f * D:(f + 1) * D])
        ref = orc.sparse_segment_reduce_grad(gf, idx, seg, U, "sum")
        got = H(sl.values[:U])
        np.testing.assert_array_equal(got.view(np.int32), ref.view(np.int32))   # bitwise, signs too
        assert not np.signbit(got[list(uids).index(2)]).any()
    dr.status_check()


def test_rows_backward_run_straddles_chunk_boundary(dr, orc):
    """Runs of 2..255 positions land across multiples of 256 of the sorted
    array (400 ids, ~50 k positions): none may be cut, all bit-exact."""
    rng = np.random.default_rng(43)
    lens = rng.integers(2, 256, 400)
    v = np.repeat(np.arange(400, dtype=np.int64) * 7 + 3, lens)
    rng.shuffle(v)
    B = v.size
    ev = dr.EmbeddingVariable("rstr", 8, 0.1)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 1)), combiner="sum")
    g = rng.standard_normal((B, 8)).astype(np.float32)
    out.backward(T(g))
    sl = ev.pending_grads.pop()
    U = int(sl.num_valid.item())
    uids, idx = orc.unique(v)
    assert H(sl.indices[:U]).tolist() == uids.tolist()
    ref = orc.sparse_segment_reduce_grad(g, idx, np.arange(B, dtype=np.int32), U, "sum")
    np.testing.assert_array_equal(H(sl.values[:U]), ref)


def _export(ev):
    k, vals = ev.export()[:2]
    k, vals = H(k), H(vals)
    o = np.argsort(k)
    return k[o], vals[o]


@pytest.mark.parametrize("opt_name", ["sgd", "adagrad", "adam", "ftrl"])
@pytest.mark.parametrize("onehot", [True, False])
def test_rows_train_step_equals_unique_path(dr, opt_name, onehot):
    """Three training steps (lookup -> backward -> apply) on the rows path
    (by-address apply) and on the Unique path (value-block apply): EV
    contents, slot contents and outputs bit-identical."""
    rng = np.random.default_rng(53 + int(onehot))
    B, D, F = 257, 16, 3

    def make_opt():
        return {"sgd": lambda: dr.GradientDescentOptimizer(0.05),
                "adagrad": lambda: dr.AdagradOptimizer(0.05),
                "adam": lambda: dr.AdamOptimizer(0.01),
                "ftrl": lambda: dr.FtrlOptimizer(0.05, l1_regularization_strength=0.01,
                                                 l2_regularization_strength=0.02)}[opt_name]()

    batches = []
    for _ in range(3):
        sps = []
        for f in range(F):
            if onehot:
                ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
                v = rng.integers(0, 70, B).astype(np.int64)
                sps.append((ind, v, (B, 1)))
            else:
                sps.append(_sparse(rng, B, 4, 70, allow_empty=True))
        batches.append((sps, rng.standard_normal((B, F * D)).astype(np.float32)))
    results = []
    for rows in (True, False):
        evs = [dr.EmbeddingVariable("rts_%s_%d_%d_%d" % (opt_name, int(onehot), int(rows), f), D,
                                    0.05) for f in range(F)]
        opt = make_opt()
        outs = []
        with _Path(rows):
            for step, (sps, g) in enumerate(batches):
                st = [dr.SparseTensor(T(i), T(v), s) for i, v, s in sps]
                out = dr.embedding_lookup_sparse_multi(evs, st, combiner="mean")
                out.backward(T(g))
                assert (evs[0].pending_grads[-1].grad_ptr is not None) == rows
                opt.apply_gradients(evs, global_step=step)
                outs.append(H(out))
        torch.cuda.synchronize()
        results.append((outs, [_export(e) for e in evs],
                        [[_export(s) for s in opt._slots(e) if s is not None] for e in evs]))
    (o1, e1, s1), (o2, e2, s2) = results
    for a, b in zip(o1, o2):
        np.testing.assert_array_equal(a, b)
    for (k1, v1), (k2, v2) in zip(e1, e2):
        np.testing.assert_array_equal(k1, k2)
        np.testing.assert_array_equal(v1, v2)
    for a, b in zip(s1, s2):
        for (k1, v1), (k2, v2) in zip(a, b):
            np.testing.assert_array_equal(k1, k2)
            np.testing.assert_array_equal(v1, v2)
    dr.status_check()


def test_sgd_known_rows_equals_probed_apply(dr):
    """SGD of a row-grouped backward applies through the forward's rows
    (dr_ev_apply_grouped_ptr_rows, no key-table probe).  Against the probing
    by-address apply on the same steps (new keys each step, steps_to_live
    versions, a shared key space): keys, values and versions identical."""
    from deeprec_amd import training
    rng = np.random.default_rng(91)
    B, D, F = 300, 16, 3
    batches = [([rng.integers(0, 120, B).astype(np.int64) for _ in range(F)],
                rng.standard_normal((B, F * D)).astype(np.float32)) for _ in range(4)]
    res = []
    for known in (True, False):
        old = training._KNOWN_ROWS
        training._KNOWN_ROWS = known
        try:
            evs = [dr.EmbeddingVariable("kr_%d_%d" % (int(known), f), D, 0.05, steps_to_live=7)
                   for f in range(F)]
            opt = dr.GradientDescentOptimizer(0.05)
            ind = T(np.stack([np.arange(B), np.zeros(B, np.int64)], 1))
            with _Path(True):
                for step, (vs, g) in enumerate(batches):
                    st = [dr.SparseTensor(ind, T(v), (B, 1)) for v in vs]
                    out = dr.embedding_lookup_sparse_multi(evs, st, combiner="sum")
                    out.backward(T(g))
                    assert evs[0].pending_grads[-1].rows is not None
                    opt.apply_gradients(evs, global_step=10 + step)
            torch.cuda.synchronize()
            ex = []
            for e in evs:
                k, v, ver = (H(a) for a in e.export()[:3])
                o = np.argsort(k)
                ex.append((k[o], v[o], ver[o]))
            res.append(ex)
        finally:
            training._KNOWN_ROWS = old
    for a, b in zip(*res):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    assert res[0][0][2].max() == 13          # versions stamped by the last step
    dr.status_check()


def test_rows_from_ptr_zero_sign(dr):
    """Bit 0 of a gradient address = 0.0f + g: -0.0 becomes +0.0 (the
    reference's unsorted segment sum starts from 0); without it the sign
    is kept."""
    from deeprec_amd._lib import lib, ptr, stream_handle
    src = torch.tensor([[-0.0, 1.0, -2.0, -0.0]], device=DEV)
    a = src.data_ptr()
    gp = torch.tensor([a | 1, a], dtype=torch.int64, device=DEV)
    out = torch.empty((2, 4), device=DEV)
    assert lib().dr_rows_from_ptr(ptr(gp), 2, None, 4, ptr(out), stream_handle(DEV)) == 0
    o = H(out)
    assert not np.signbit(o[0, 0]) and not np.signbit(o[0, 3])
    assert np.signbit(o[1, 0]) and np.signbit(o[1, 3])
    np.testing.assert_array_equal(o[:, 1:3], [[1.0, -2.0], [1.0, -2.0]])


def test_graph_captured_train_steps_equal_eager(dr):
    """Whole training steps (forward, autograd backward through the rows
    path, by-address SGD apply) captured as one hipGraph and replayed leave
    the EVs exactly where the same steps run eagerly leave them (the bench's
    train_step replays such a graph)."""
    rng = np.random.default_rng(61)
    B, D, F, S = 512, 32, 3, 4
    keys = [T(rng.integers(0, 3000, (F, B)).astype(np.int64)) for _ in range(S + 2)]
    ind = T(np.stack([np.arange(B), np.zeros(B, np.int64)], 1))
    ups = [T(rng.standard_normal((B, F * D)).astype(np.float32)) for _ in range(S + 2)]
    exports = []
    for graphed in (False, True):
        evs = [dr.EmbeddingVariable("gts_%d_%d" % (int(graphed), f), D, 0.05, capacity=8192)
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
    for (k1, v1), (k2, v2) in zip(*exports):
        np.testing.assert_array_equal(k1, k2)
        np.testing.assert_array_equal(v1, v2)


def test_ev_collected_during_capture_is_released_after(dr):
    """An EV whose last reference dies inside a hipGraph capture (cyclic
    garbage collected by an allocation in the captured step) does not free
    device memory there -- that would invalidate the capture -- but is
    released by the next uncaptured EV creation."""
    import gc
    from deeprec_amd import kv_variable_ops as kvo
    gc.collect()
    kvo._flush_deferred_releases()
    ev = dr.EmbeddingVariable("cap_gc", 8, 0.0, capacity=1024)
    ev._self_ref = ev                      # a cycle: only the collector frees it
    del ev
    x = torch.zeros(16, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x + 1
        gc.collect()
    assert len(kvo._DEFERRED) == 1
    g.replay()
    torch.cuda.synchronize()
    assert float(y.sum()) == 16.0
    keep = dr.EmbeddingVariable("cap_gc2", 8, 0.0, capacity=1024)
    assert len(kvo._DEFERRED) == 0
    # collected on ANOTHER thread (whose current stream is not capturing)
    # while this thread captures: still deferred, released after the capture
    import threading
    ev = dr.EmbeddingVariable("cap_gc3", 8, 0.0, capacity=1024)
    ev._self_ref = ev
    del ev
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        y2 = x + 2
        th = threading.Thread(target=gc.collect)
        th.start()
        th.join()
    assert len(kvo._DEFERRED) == 1
    g2.replay()
    torch.cuda.synchronize()
    assert float(y2.sum()) == 32.0
    dr.flush_releases()
    assert len(kvo._DEFERRED) == 0
    del keep


def test_kv_adam_device_powers_equal_host_powers(dr, monkeypatch):
    """KV Adam with its beta powers in HBM (dr_ev_apply_adam_grouped_dev:
    alpha formed by the kernel, powers advanced by an fp32 multiply on the
    device) leaves the EVs and both slots bit-identical to the host-powers
    apply (dr_ev_apply_grouped, alpha formed on the host) over three steps,
    by-address and value-block gradients both."""
    from deeprec_amd import training
    rng = np.random.default_rng(71)
    B, D = 3000, 16
    batches = []
    for _ in range(3):
        v = rng.integers(0, 500, B).astype(np.int64)
        batches.append((v, rng.standard_normal((B, D)).astype(np.float32)))
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    res = []
    for dev_powers in (True, False):
        monkeypatch.setattr(training, "_ADAM_DEVICE_POWERS", dev_powers)
        ev = dr.EmbeddingVariable("adam_pw_%d" % int(dev_powers), D, 0.1, capacity=2048)
        opt = dr.AdamOptimizer(0.01)
        for step, (v, g) in enumerate(batches):
            out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 1)),
                                             combiner="mean")
            out.backward(T(g))
            opt.apply_gradients([ev], global_step=step)
        torch.cuda.synchronize()
        m, s = opt._slots(ev)
        res.append([_export(ev), _export(m), _export(s)])
    for (k1, v1), (k2, v2) in zip(res[0], res[1]):
        np.testing.assert_array_equal(k1, k2)
        np.testing.assert_array_equal(v1.view(np.uint32), v2.view(np.uint32))


def test_din_item_gradient_order_matches_oracle(dr, orc):
    """Pins the order DIN's merged item lookup sums its gradient in: the
    reference looks up the target items and the history separately
    (model.py:61-98) and the optimizer sums the two IndexedSlices per id with
    unsorted_segment_sum over their concatenation (optimizer.py
    _deduplicate_indexed_slices; the CPU functor adds the rows in order) --
    one serial chain per id over [target positions, history positions].
    modelzoo.DIN's single lookup of [mids, mid_his] must give exactly that:
    for the mid and cat EVs, the unique ids in first-occurrence order and
    every per-id sum bit-equal to the oracle's serial segment sum of the same
    allv gradient rows (hooked), padding id 0 included."""
    from deeprec_amd import modelzoo as mz
    B, T_, D = 64, 20, 18
    R = (500, 300, 40)
    g = torch.Generator(device=DEV)
    g.manual_seed(77)
    evs = []
    for i, r in enumerate(R):
        ev = dr.EmbeddingVariable("dgo_%d" % i, D, 0.0, capacity=r + 4096, device=DEV)
        ev.insert_synthetic(0, r, seed=900 + i)
        evs.append(ev)
    model = mz.DIN(*evs).to(DEV)
    lens = torch.randint(1, T_ + 1, (B,), generator=g, device=DEV)
    mask = (torch.arange(T_, device=DEV)[None, :] < lens[:, None]).float()
    mh = torch.randint(1, R[1], (B, T_), generator=g, device=DEV) * mask.long()
    ch = torch.randint(1, R[2], (B, T_), generator=g, device=DEV) * mask.long()
    uids = torch.randint(0, R[0], (B,), generator=g, device=DEV)
    mids = torch.randint(0, R[1], (B,), generator=g, device=DEV)
    cats = torch.randint(0, R[2], (B,), generator=g, device=DEV)
    lab = (torch.rand(B, generator=g, device=DEV) > 0.5).long()
    target = torch.stack([lab, 1 - lab], 1).float()
    grads = []
    inner = model.item_lookup

    class Hooked(object):
        def __call__(self, ids):
            out = inner(ids)
            out.register_hook(lambda gr: grads.append(gr.detach().clone()))
            return out
    model.item_lookup = Hooked()
    y = model(uids, mids, cats, mh, ch, mask)
    (-(torch.log(y) * target).mean()).backward()
    torch.cuda.synchronize()
    assert len(grads) == 1
    gall = H(grads[0])                                      # [B + B T, 2D]
    for f, (tgt, his) in enumerate(((mids, mh), (cats, ch))):
        ids = np.concatenate([H(tgt), H(his).reshape(-1)]).astype(np.int64)
        uids_ref, idx = orc.unique(ids)
        sl = evs[1 + f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids_ref.tolist()
        gf = np.ascontiguousarray(gall[:, f * D:(f + 1) * D])
        ref = orc.sparse_segment_reduce_grad(gf, idx, np.arange(ids.size, dtype=np.int32), U,
                                             "sum")
        np.testing.assert_array_equal(H(sl.values[:U]).view(np.uint32), ref.view(np.uint32))
    dr.status_check()


@pytest.mark.parametrize("terms", ["din_pad_terms.npz", "din_pad_terms_s200.npz"])
def test_rows_backward_real_din_padding_chain(dr, orc, terms):
    """The padding id's chain with DIN's REAL gradient terms (tools/data:
    one step of configs[3] at the first step and after 200 Adam steps,
    dumped by tools/din_term_probe.py -- 4 050 segments, 203 800 positions,
    D = 18), beside 30 000 positions on other ids, through the default walk
    (64 positions read ahead, one counted LDS wait per 32): every per-id sum
    bit-equal to the oracle's serial sum."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "tools", "data", terms))
    tv, k = z["terms"].astype(np.float32), z["lens"].astype(np.int64)
    D = tv.shape[1]
    rng = np.random.default_rng(5)
    other = rng.integers(1, 5000, 30000).astype(np.int64)
    v = np.concatenate([np.zeros(int(k.sum()), np.int64), other])
    g = np.concatenate([np.repeat(tv, k, axis=0),
                        (rng.standard_normal((other.size, D)) * 1e-6).astype(np.float32)])
    B = v.size
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    ev = dr.EmbeddingVariable("rdinreal_%s" % terms[:-4], D, 0.1, capacity=8192)
    out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 1)), combiner="sum")
    out.backward(T(g))
    uids, idx = orc.unique(v)
    sl = ev.pending_grads.pop()
    U = int(sl.num_valid.item())
    assert H(sl.indices[:U]).tolist() == uids.tolist()
    ref = orc.sparse_segment_reduce_grad(g, idx, np.arange(B, dtype=np.int32), U, "sum")
    np.testing.assert_array_equal(H(sl.values[:U]).view(np.uint32), ref.view(np.uint32))
    dr.status_check()
