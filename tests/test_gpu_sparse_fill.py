"""dr_sparse_prune_fill (prune + SparseFillEmptyRows on the GPU) against the
oracle's serial restatement of sparse_fill_empty_rows_op_util.h:17-128 and
the prune steps of embedding_ops.py:1299-1306.  Integer/index work: exact."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(seed, B, nnz, rank=2, ordered=False):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, B, nnz)
    if ordered:
        rows = np.sort(rows)
    ind = np.stack([rows] + [rng.integers(0, 9, nnz) for _ in range(rank - 1)], 1).astype(np.int64)
    val = rng.integers(-3, 50, nnz).astype(np.int64)
    w = rng.uniform(-0.5, 1.0, nnz).astype(np.float32)
    return ind, val, w


@pytest.mark.parametrize("seed,B,nnz,rank,ordered", [(1, 50, 200, 2, False), (2, 1000, 300, 2, True),
                                                     (3, 7, 0, 2, False), (4, 64, 500, 3, False),
                                                     (5, 1, 10, 2, False)])
def test_fill_empty_rows_matches_oracle(seed, B, nnz, rank, ordered):
    import deeprec_amd as dr
    from deeprec_amd import embedding_ops as eo
    from oracle import oracle as orc
    ind, val, _ = _case(seed, B, nnz, rank, ordered)
    sp = dr.SparseTensor(torch.as_tensor(ind, device=DEV).reshape(nnz, rank),
                         torch.as_tensor(val, device=DEV), (B, 9))
    out, empty = eo.sparse_fill_empty_rows(sp, 77)
    ri, rv, re, rrev = orc.sparse_fill_empty_rows(ind, val, B, 77)
    np.testing.assert_array_equal(out.indices.cpu().numpy(), ri)
    np.testing.assert_array_equal(out.values.cpu().numpy(), rv)
    np.testing.assert_array_equal(empty.cpu().numpy(), re)
    _, _, _, rev = eo.sparse_prune_fill(sp, None, 77, 0)
    np.testing.assert_array_equal(rev.cpu().numpy(), rrev)


@pytest.mark.parametrize("combiner", ["sum", "mean"])
@pytest.mark.parametrize("with_w", [False, True])
def test_prune_and_fill_matches_oracle(combiner, with_w):
    import deeprec_amd as dr
    from deeprec_amd import embedding_ops as eo
    from oracle import oracle as orc
    B, nnz = 40, 150
    ind, val, w = _case(11, B, nnz)
    sp = dr.SparseTensor(torch.as_tensor(ind, device=DEV), torch.as_tensor(val, device=DEV), (B, 9))
    spw = dr.SparseTensor(sp.indices, torch.as_tensor(w, device=DEV), (B, 9)) if with_w else None
    gs, gw, ge = eo._prune_and_fill(sp, spw, combiner, 5, True)
    ri, rv, rw, re = orc.prune_and_fill(ind, val, (B, 9), w if with_w else None, combiner, 5, True)
    np.testing.assert_array_equal(gs.indices.cpu().numpy(), ri)
    np.testing.assert_array_equal(gs.values.cpu().numpy(), rv)
    np.testing.assert_array_equal(ge.cpu().numpy(), re)
    if with_w:
        np.testing.assert_array_equal(gw.values.cpu().numpy(), rw)


def test_safe_lookup_unordered_input_matches_oracle():
    import deeprec_amd as dr
    from oracle import oracle as orc
    B, nnz, D = 64, 300, 16
    ind, val, w = _case(21, B, nnz)
    ev = dr.EmbeddingVariable("spf_ev", D, 0.125)
    oev = orc.EV(D, 0.125)
    sp = dr.SparseTensor(torch.as_tensor(ind, device=DEV), torch.as_tensor(val, device=DEV), (B, 9))
    spw = dr.SparseTensor(sp.indices, torch.as_tensor(w, device=DEV), (B, 9))
    got = dr.safe_embedding_lookup_sparse(ev, sp, spw, combiner="mean")
    ref = orc.safe_embedding_lookup_sparse(oev, ind, val, (B, 9), w, combiner="mean")
    np.testing.assert_array_equal(got.detach().cpu().numpy(), ref)


def test_out_of_range_row_latches_invalid_argument():
    import deeprec_amd as dr
    from deeprec_amd import embedding_ops as eo
    ind = torch.as_tensor([[0, 0], [5, 0]], dtype=torch.int64, device=DEV)
    sp = dr.SparseTensor(ind, torch.as_tensor([1, 2], dtype=torch.int64, device=DEV), (3, 1))
    with pytest.raises(dr.InvalidArgumentError):   # at the op (validate mode) or the check
        eo.sparse_prune_fill(sp, None, 0, 0)
        dr.status_check()
