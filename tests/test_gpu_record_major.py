"""Fused one-hot lookup reading ids in place from a record-major [B, T]
matrix (dr_ev_lookup_onehot_strided; one Criteo record of T categorical ids
per row, the SOK/DLRM Criteo-TB input layout) against the oracle's
KvResourceGather (kv_variable_ops.cc:314-366: insert-on-miss with the EV
default row) and against the feature-major [T, B] path on twin EVs: outputs,
EV sizes and rows served bit-identical, with new keys (the miss kernel reads
the same strides) and duplicates inside the batch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd as dr
    dr.load()
    dr.set_validate(True)
    return dr


@pytest.mark.parametrize("D", [12, 32, 128])
def test_record_major_lookup_matches_oracle(dr, orc, D):
    from deeprec_amd import _lib
    from deeprec_amd.embedding_ops import SparseTensor, _Feature, _record_major
    rng = np.random.default_rng(D)
    T, B, R = 7, 3000, 2000
    evs, twins, oevs = [], [], []
    for t in range(T):
        keys = np.arange(R, dtype=np.int64) * 3 + t
        init = rng.standard_normal((R, D)).astype(np.float32)
        ev = dr.EmbeddingVariable("rm%d_%d" % (D, t), D, 0.5)
        tw = dr.EmbeddingVariable("rmt%d_%d" % (D, t), D, 0.5)
        oev = _orc_ev(orc, D)
        for e in (ev, tw):
            e.insert(torch.as_tensor(keys, device=DEV), torch.as_tensor(init, device=DEV))
        oev.insert(keys, init)
        evs.append(ev)
        twins.append(tw)
        oevs.append(oev)
    ids = rng.integers(0, 3 * R + 600, (B, T)).astype(np.int64)    # ~15 % new keys, repeats
    rec = torch.as_tensor(ids, device=DEV)                           # [B, T] record-major
    ind = torch.stack([torch.arange(B, device=DEV), torch.zeros(B, dtype=torch.int64,
                                                                 device=DEV)], 1)
    feats = [_Feature(evs[t], rec[:, t], ind, B, None, "sum", None, onehot=True)
             for t in range(T)]
    assert _record_major(feats) == rec.data_ptr()
    with torch.no_grad():
        out = dr.embedding_lookup_sparse_multi(
            evs, [SparseTensor(ind, rec[:, t], (B, 1)) for t in range(T)], combiner="sum")
        fm = torch.as_tensor(np.ascontiguousarray(ids.T), device=DEV)  # [T, B] feature-major
        out_t = dr.embedding_lookup_sparse_multi(
            twins, [SparseTensor(ind, fm[t], (B, 1)) for t in range(T)], combiner="sum")
    dr.status_check()
    got = out.cpu().numpy().reshape(B, T, D)
    for t in range(T):
        want = oevs[t].gather(ids[:, t])              # insert-on-miss in id order
        np.testing.assert_array_equal(got[:, t, :], want)
        assert int(evs[t].total_count()[0]) == int(twins[t].total_count()[0])
    assert torch.equal(out, out_t)
    # second pass: every key now exists (probe-only path), still equal
    with torch.no_grad():
        out2 = dr.embedding_lookup_sparse_multi(
            evs, [SparseTensor(ind, rec[:, t], (B, 1)) for t in range(T)], combiner="sum")
    assert torch.equal(out2, out)


def test_record_major_strided_rows_out(dr):
    """dr_ev_lookup_onehot_strided with rows_out: rows land at [t*B + b] for
    either id layout and match."""
    import ctypes as C
    from deeprec_amd._lib import check, lib, ptr, stream_handle, workspace
    T, B, D = 3, 500, 16
    rng = np.random.default_rng(9)
    evs = [dr.EmbeddingVariable("rmr%d" % t, D, 0.0) for t in range(T)]
    ids = rng.integers(0, 400, (B, T)).astype(np.int64)
    rec = torch.as_tensor(ids, device=DEV)
    fm = rec.t().contiguous()
    outs, rows = [], []
    for keys, sb, st in ((rec, T, 1), (fm, 1, B)):
        out = torch.empty((B, T * D), device=DEV)
        r = torch.full((T * B,), -7, dtype=torch.int64, device=DEV)
        h = (C.c_void_p * T)(*[e.handle.value for e in evs])
        wsb = lib().dr_ev_lookup_onehot_workspace_size(T, B)
        ws = workspace(wsb, DEV)
        check(lib().dr_ev_lookup_onehot_strided(h, T, ptr(keys), sb, st, B, ptr(out), T * D, 0,
                                                ptr(r), ptr(ws), wsb, stream_handle(DEV)))
        torch.cuda.synchronize()
        outs.append(out)
        rows.append(r)
    dr.status_check()
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(rows[0], rows[1])
    assert int(rows[0].min()) >= 0


def _orc_ev(orc, D):
    return orc.EV(D, 0.5)
