"""combiner="tile" of embedding_lookup_sparse (reference
python/ops/embedding_ops.py:468-476 _tile_combine_embedding, used at
:646-651 with weights and :665-671 without): each (row, column) of sp_ids
gets its own D-wide block of a [B, C * D] output, entries sharing a
(row, column) are summed in position order (UnsortedSegmentSum).  Checked
against numpy float32 transcriptions of the same steps: forward bit-exact;
gradients (the IndexedSlices an EV receives, the dense table's rows) within
1e-6 rel -- the unique-id gradient sums add the same terms in another order
than numpy's scatter."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd as dr
    dr.load()
    dr.set_validate(True)
    return dr


def _case(seed, B=48, C=5, vocab=40, dup=True):
    rng = np.random.default_rng(seed)
    ind = []
    for r in range(B):
        cols = np.sort(rng.choice(C, rng.integers(0, C + 1), replace=False))
        for c in cols:
            ind.append((r, c))
            if dup and rng.random() < 0.2:
                ind.append((r, c))            # a repeated (row, column): summed
    ind = np.array(ind, np.int64).reshape(-1, 2)
    vals = rng.integers(0, vocab, ind.shape[0]).astype(np.int64)
    w = rng.uniform(0.5, 2.0, ind.shape[0]).astype(np.float32)
    return ind, vals, w


def _tile_np(table, ind, vals, w, B, C, max_norm=None):
    D = table.shape[1]
    rows = table[vals].astype(np.float32)
    if max_norm is not None:
        l2 = np.sqrt((rows * rows).sum(1, keepdims=True, dtype=np.float32)).astype(np.float32)
        rows = (rows * np.float32(max_norm) / np.maximum(l2, np.float32(max_norm))).astype(
            np.float32)
    if w is not None:
        rows = (rows * w[:, None]).astype(np.float32)
    out = np.zeros((B * C, D), np.float32)
    for i, (r, c) in enumerate(ind):
        out[r * C + c] = out[r * C + c] + rows[i]
    return out.reshape(B, C * D)


@pytest.mark.parametrize("weighted", [False, True])
def test_tile_ev_forward_and_grads(dr, weighted):
    B, C, D = 48, 5, 8
    ind, vals, w = _case(3 + weighted, B, C)
    ev = dr.EmbeddingVariable("tile_%d" % weighted, D, lambda s: torch.randn(s) * 0.1)
    keys = np.arange(40, dtype=np.int64)
    table = ev.sparse_read(T(keys)).cpu().numpy()          # creates every row
    sp = dr.SparseTensor(T(ind), T(vals), (B, C))
    spw = dr.SparseTensor(T(ind), T(w), (B, C)) if weighted else None
    out = dr.embedding_lookup_sparse(ev, sp, spw, combiner="tile")
    want = _tile_np(table, ind, vals, w if weighted else None, B, C)
    assert tuple(out.shape) == (B, C * D)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), want)
    up = np.random.default_rng(9).standard_normal((B, C * D)).astype(np.float32)
    out.backward(T(up))
    from deeprec_amd.training import _dedup
    sl = _dedup(ev.pending_grads)
    n = sl.indices.numel() if sl.num_valid is None else int(sl.num_valid.item())
    got = dict(zip(sl.indices[:n].cpu().numpy().tolist(), sl.values[:n].cpu().numpy()))
    upr = up.reshape(B * C, D)
    ref = {}
    for i, (r, c) in enumerate(ind):
        g = upr[r * C + c] * (w[i] if weighted else np.float32(1))
        ref[int(vals[i])] = ref.get(int(vals[i]), np.zeros(D, np.float32)) + g
    assert set(got) == set(ref)
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-6, atol=1e-6)


def test_tile_dense_table_max_norm_matches_torch(dr):
    B, C, D, V = 32, 4, 16, 30
    ind, vals, w = _case(11, B, C, V)
    tab = (np.random.default_rng(2).standard_normal((V, D)) * 0.8).astype(np.float32)
    p = T(tab).requires_grad_(True)
    sp = dr.SparseTensor(T(ind), T(vals), (B, C))
    out = dr.embedding_lookup_sparse(p, sp, None, combiner="tile", max_norm=1.5)
    np.testing.assert_allclose(out.detach().cpu().numpy(),
                               _tile_np(tab, ind, vals, None, B, C, max_norm=1.5),
                               rtol=1e-6, atol=1e-7)
    up = T(np.random.default_rng(4).standard_normal((B, C * D)).astype(np.float32))
    out.backward(up)
    # torch fp32 reference of the same composition
    q = T(tab).requires_grad_(True)
    r = q[T(vals)]
    l2 = torch.sqrt((r * r).sum(1, keepdim=True))
    r = r * 1.5 / torch.maximum(l2, torch.tensor(1.5, device=DEV))
    seg = T(ind[:, 0] * C + ind[:, 1])
    ref = torch.zeros(B * C, D, device=DEV).index_add(0, seg, r).reshape(B, C * D)
    ref.backward(up)
    np.testing.assert_allclose(p.grad.cpu().numpy(), q.grad.cpu().numpy(), rtol=1e-5, atol=1e-6)


def test_tile_empty_batch_rows_are_zero(dr):
    ev = dr.EmbeddingVariable("tile_empty", 4, 1.0)
    ind = np.array([[0, 1], [2, 0]], np.int64)
    out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T([5, 6]), (3, 2)),
                                     combiner="tile").detach().cpu().numpy()
    want = np.zeros((3, 8), np.float32)
    want[0, 4:8] = 1.0
    want[2, 0:4] = 1.0
    np.testing.assert_array_equal(out, want)
