"""Parity at the headline configuration (BASELINE configs[2] per GPU): 26 EVs x
12.5 M rows x 128 fp32, B = 65 536, hotness 1 -- the table bench.py times.

The rows are regenerable (synth(seed, key, col), dr_common.h), so sampled
output rows are checked bit for bit against the host restatement
(oracle.synth_rows) at the real load factor and probe-chain lengths, for:
  * a uniform step through the fused one-hot kernel (dr_ev_lookup_onehot) and
    the resolve -> pool pipeline (whole outputs equal), and with the ids read
    in place from a record-major [B, T] matrix (dr_ev_lookup_onehot_strided,
    the bench's layout: whole output equal),
  * a step with ~10 % new keys (insert-on-miss: default rows, every EV grows
    by exactly its distinct new keys, existing rows unchanged),
  * a Zipf(1.05) step (hot keys, long duplicate runs),
with the device status word clean (KvResourceGather semantics,
kv_variable_ops.cc:314-366).
"""
import gc

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
T, R, D, B = 26, 12_500_000, 128, 65536
NCHECK = 8192


def _check(out, ids, seed, orc):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, B, NCHECK)
    t = rng.integers(0, T, NCHECK)
    got = out.view(B, T, D)[torch.as_tensor(b, device=DEV), torch.as_tensor(t, device=DEV)]
    got = got.cpu().numpy()
    keys = ids[torch.as_tensor(t, device=DEV), torch.as_tensor(b, device=DEV)].cpu().numpy()
    for tt in np.unique(t):
        sel = t == tt
        np.testing.assert_array_equal(got[sel], orc.synth_rows(1000 + int(tt), keys[sel], D))


def test_headline_shape_parity(orc):
    import deeprec_amd as dr
    from deeprec_amd import _lib
    from deeprec_amd.embedding_ops import SparseTensor, _Feature, _pool_all, _prepare_group
    dr.load()
    gc.collect()
    torch.cuda.empty_cache()
    evs = []
    try:
        for t in range(T):
            ev = dr.EmbeddingVariable("hl%d" % t, D, 0.0, capacity=R + (1 << 19), device=DEV)
            ev.insert_synthetic(0, R, seed=1000 + t)
            evs.append(ev)
        g = torch.Generator(device=DEV)
        g.manual_seed(2021)
        ind = torch.stack([torch.arange(B, device=DEV),
                           torch.zeros(B, dtype=torch.int64, device=DEV)], 1)
        seg = torch.arange(B, dtype=torch.int32, device=DEV)
        with torch.no_grad():
            ids = torch.randint(0, R, (T, B), generator=g, device=DEV, dtype=torch.int64)
            sps = [SparseTensor(ind, ids[t], (B, 1)) for t in range(T)]
            out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")   # fused one-hot
            dr.status_check()
            _check(out, ids, 1, orc)
            feats = [_Feature(evs[t], ids[t], seg, B, None, "sum", None, onehot=True)
                     for t in range(T)]
            _prepare_group(feats, need_grad=False)
            out2 = _pool_all(feats, _lib.ORDER_ALI)                         # resolve -> pool
            dr.status_check()
            assert torch.equal(out, out2)
            assert all(int(ev.total_count()[0]) == R for ev in evs)
            rec = ids.t().contiguous()                                       # [B, T] records
            out3 = dr.embedding_lookup_sparse_multi(
                evs, [SparseTensor(ind, rec[:, t], (B, 1)) for t in range(T)], combiner="sum")
            dr.status_check()
            assert torch.equal(out, out3)

            # ~10 % new keys: insert-on-miss
            newm = torch.rand((T, B), generator=g, device=DEV) < 0.1
            fresh = R + torch.randint(0, 1 << 40, (T, B), generator=g, device=DEV,
                                      dtype=torch.int64)
            ids_n = torch.where(newm, fresh, ids)
            rec_n = ids_n.t().contiguous()
            # the insert-on-miss step reads its ids record-major (strided miss path)
            outn = dr.embedding_lookup_sparse_multi(
                evs, [SparseTensor(ind, rec_n[:, t], (B, 1)) for t in range(T)], combiner="sum")
            sps = [SparseTensor(ind, ids_n[t], (B, 1)) for t in range(T)]
            dr.status_check()
            view = outn.view(B, T, D)
            assert not bool((view[newm.t()] != 0).any())
            for t in range(T):
                want = R + int(torch.unique(ids_n[t][newm[t]]).numel())
                assert int(evs[t].total_count()[0]) == want
            old = (~newm).t()
            bb, tt = torch.nonzero(old, as_tuple=True)
            sel = torch.randperm(bb.numel(), generator=torch.Generator().manual_seed(3))[:NCHECK]
            bb, tt = bb[sel.to(DEV)], tt[sel.to(DEV)]
            got = view[bb, tt].cpu().numpy()
            keys = ids_n[tt, bb].cpu().numpy()
            tn = tt.cpu().numpy()
            for t in np.unique(tn):
                np.testing.assert_array_equal(got[tn == t],
                                              orc.synth_rows(1000 + int(t), keys[tn == t], D))
            # the new keys now exist and read their default rows again
            outn2 = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
            assert torch.equal(outn, outn2)

            # Zipf(1.05): hot keys
            zk = (torch.as_tensor(np.random.default_rng(5).zipf(1.05, size=(T, B)), device=DEV)
                  - 1) % R
            sps = [SparseTensor(ind, zk[t], (B, 1)) for t in range(T)]
            outz = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
            dr.status_check()
            _check(outz, zk, 2, orc)
    finally:
        del evs
        gc.collect()
        dr.flush_releases()
