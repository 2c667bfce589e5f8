"""GPU: hot-id gradients of the row-grouped training default are the
reference's serial sums and do not depend on how the EV numbered its rows.

The reference's UnsortedSegmentSum / SparseSegmentSumGrad add a run's
positions serially in ascending order (segment_reduction_ops.cc:391-404,
math_grad.py:321-368).  The row-grouped backward sorts (row, position) pairs,
so where a hot id's run lands in the sorted array depends on the key -> row
map, which racing first-touch inserts assign.  Runs are summed from their own
first position: up to kSerialMax = 8192 positions exactly in the serial order
(bit-exact to the oracle), longer runs as ordered sums of 8192-position
pieces cut from the run start -- deterministic either way.

Two builds of the same 26-table EV set whose rows were inserted in different
orders (one stream, vs four racing streams in another order) must leave
bit-identical rows after a fused backward + SGD step on a Zipf(1.05) batch
whose hottest ids repeat > 5000 times per table.
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


def _zipf_keys(rng, n, vocab, a=1.05):
    p = 1.0 / np.arange(1, vocab + 1, dtype=np.float64) ** a
    p /= p.sum()
    ranks = rng.choice(vocab, size=n, p=p)
    # scatter the ranks over the key space (hot keys are not the small ones)
    return (ranks.astype(np.int64) * 7919 + 13) % (1 << 40)


def _init_rows(keys, D, f):
    # a per-(table, key) row, identical in both builds whatever row it lands in
    k = keys.astype(np.uint64)[:, None]
    c = np.arange(D, dtype=np.uint64)[None, :]
    h = (k * np.uint64(0x9E3779B97F4A7C15) + c * np.uint64(0xBF58476D1CE4E5B9)
         + np.uint64(f + 1)) >> np.uint64(40)
    return ((h.astype(np.float64) / float(1 << 24)) - 0.5).astype(np.float32)


def _build(dr, tag, tables, D, order_seed, streams):
    """EVs with every batch key pre-inserted: keys in a seeded order, split
    over `streams` side streams that run concurrently (racing row bumps)."""
    rng = np.random.default_rng(order_seed)
    evs = []
    for f, keys in enumerate(tables):
        ev = dr.EmbeddingVariable("%s_%d" % (tag, f), D, 0.0, capacity=1 << 16)
        uk = np.unique(keys)
        uk = uk[rng.permutation(uk.size)]
        vals = _init_rows(uk, D, f)
        parts = np.array_split(np.arange(uk.size), streams)
        ss = [torch.cuda.Stream() for _ in range(streams)]
        torch.cuda.synchronize()
        for s, idx in zip(ss, parts):
            with torch.cuda.stream(s):
                ev.insert(T(uk[idx]), T(vals[idx]))
        torch.cuda.synchronize()
        evs.append(ev)
    return evs


def _step(dr, evs, tables, g, lr):
    B = tables[0].size
    ind = T(np.stack([np.arange(B), np.zeros(B, np.int64)], 1))
    sps = [dr.SparseTensor(ind, T(k), (B, 1)) for k in tables]
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
    out.backward(T(g))
    dr.GradientDescentOptimizer(lr).apply_gradients(evs, global_step=1)
    torch.cuda.synchronize()
    dr.status_check()


def _export(ev):
    k, v = (H(a) for a in ev.export()[:2])
    o = np.argsort(k)
    return k[o], v[o]


@pytest.mark.parametrize("D", [16, 128])
def test_hot_id_sgd_bit_identical_across_insert_orders(dr, orc, D):
    rng = np.random.default_rng(2021 + D)
    F, B, lr = 26, 65536, 0.05
    vocab = 1000000
    tables = [_zipf_keys(rng, B, vocab) for _ in range(F)]
    # one constant feature (a Criteo column of cardinality 1): a 65536-position
    # run, one serial chain
    tables[25] = np.full(B, 123456789, np.int64)
    hot = [int(np.bincount(np.unique(t, return_inverse=True)[1]).max()) for t in tables[:25]]
    assert min(hot) > 5000, hot
    g = rng.standard_normal((B, F * D)).astype(np.float32)

    a = _build(dr, "det_a%d" % D, tables, D, order_seed=1, streams=1)
    b = _build(dr, "det_b%d" % D, tables, D, order_seed=2, streams=4)
    # the two builds number the hot keys' rows differently (so their runs sit
    # at different places of the row-sorted arrays)
    hk = [np.unique(t) for t in tables[:4]]
    ra = [H(a[f].resolve(T(hk[f]))) for f in range(4)]
    rb = [H(b[f].resolve(T(hk[f]))) for f in range(4)]
    assert all((x != y).mean() > 0.5 for x, y in zip(ra, rb))
    _step(dr, a, tables, g, lr)
    _step(dr, b, tables, g, lr)
    lr32 = np.float32(lr)
    for f in range(F):
        ka, va = _export(a[f])
        kb, vb = _export(b[f])
        np.testing.assert_array_equal(ka, kb)
        np.testing.assert_array_equal(va, vb)   # bit-identical whatever the row numbering
        # against the oracle's serial ascending-position sum
        uids, idx = orc.unique(tables[f])
        gs = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g[:, f * D:(f + 1) * D]), idx,
                                            np.arange(B, dtype=np.int32), uids.size, "sum")
        pos = np.searchsorted(ka, uids)
        assert np.array_equal(ka[pos], uids)
        want = _init_rows(uids, D, f) - lr32 * gs
        got = va[pos]
        # every run -- the constant feature's 65536 positions included -- is
        # one serial chain: exact
        np.testing.assert_array_equal(got, want)
