"""Parity at the BASELINE configs' own sizes (VERDICT r02 "next" #1), each on
the HIP path against the oracle / an fp64 reference:

* configs[1] DeepFM: 26 EVs x 1e7 rows x 64 fp32, B = 65 536, hotness 1 --
  the fused lookup (sampled rows bit-exact to the tables' synth rows) and one
  embedding training step with KV SGD: for three whole tables, every updated
  row equals synth - lr * g_u with g_u the oracle's SparseSegmentSumGrad
  (segment_reduction_ali_ops_util.h:331-458) over the oracle's first-
  occurrence Unique (unique_ali_op_util.h:192-222), i.e. the reference's
  KvResourceSparseApplyGradientDescent (training_ali_ops.cc:1653-1664).
* configs[3] DIN: uid / item / category EVs 5e5 / 4e5 / 2e3 x 18, B = 4 096,
  history lengths U[1, 100] -- the embedding lookups bit-exact, one training
  step (attention, masked softmax, Dice FCN, backward, KV SGD) against the
  same model in fp64 (rtol 1e-5 / atol 1e-6, north_star's 1e-5 rel).
* configs[4] DCN-v2 CrossNet layer at B = 65 536, d = 3 392 (13 + 26 x 128,
  padded to a multiple of 64): the bf16 MFMA kernel against fp64 on 512
  sampled rows (the cross layer is row-local), element tolerance
  2^-8 |want| (bf16 output rounding) + 1e-3 max |want| (fp32 accumulation of
  3 392 bf16 products).
"""
import gc

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _cleanup(dr):
    gc.collect()
    dr.flush_releases()
    torch.cuda.empty_cache()


def test_config1_deepfm_lookup_and_sgd_step(orc):
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import SparseTensor
    dr.load()
    _cleanup(dr)
    T, R, D, B, lr = 26, 10_000_000, 64, 65536, np.float32(0.01)
    evs = []
    try:
        for t in range(T):
            ev = dr.EmbeddingVariable("c1_%d" % t, D, 0.0, capacity=R + (1 << 20), device=DEV)
            ev.insert_synthetic(0, R, seed=5000 + t)
            evs.append(ev)
        g = torch.Generator(device=DEV)
        g.manual_seed(1)
        ids = torch.randint(0, R, (T, B), generator=g, device=DEV, dtype=torch.int64)
        ind = torch.stack([torch.arange(B, device=DEV),
                           torch.zeros(B, dtype=torch.int64, device=DEV)], 1)
        sps = [SparseTensor(ind, ids[t], (B, 1)) for t in range(T)]
        rec = ids.t().contiguous()
        with torch.no_grad():
            out = dr.embedding_lookup_sparse_multi(
                evs, [SparseTensor(ind, rec[:, t], (B, 1)) for t in range(T)], combiner="sum")
        dr.status_check()
        rng = np.random.default_rng(7)
        bs, ts = rng.integers(0, B, 4096), rng.integers(0, T, 4096)
        got = out.view(B, T, D)[torch.as_tensor(bs, device=DEV),
                                torch.as_tensor(ts, device=DEV)].cpu().numpy()
        keys = ids[torch.as_tensor(ts, device=DEV), torch.as_tensor(bs, device=DEV)].cpu().numpy()
        for t in np.unique(ts):
            np.testing.assert_array_equal(got[ts == t], orc.synth_rows(5000 + int(t),
                                                                        keys[ts == t], D))
        # one training step: fused lookup recording rows -> row-grouped
        # backward -> KV SGD by address
        up = torch.randn((B, T * D), generator=g, device=DEV)
        out_t = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
        assert torch.equal(out_t.detach(), out)
        out_t.backward(up)
        dr.GradientDescentOptimizer(float(lr)).apply_gradients(evs, global_step=1)
        dr.status_check()
        upn = up.cpu().numpy()
        seg = np.arange(B, dtype=np.int32)
        for t in (0, 13, 25):
            vals = ids[t].cpu().numpy()
            uids, idx = orc.unique(vals)
            gref = orc.sparse_segment_reduce_grad(upn[:, t * D:(t + 1) * D], idx, seg,
                                                  uids.shape[0], "sum")
            want = orc.synth_rows(5000 + t, uids, D) - lr * gref
            now = evs[t].sparse_read(torch.as_tensor(uids, device=DEV)).cpu().numpy()
            np.testing.assert_array_equal(now, want)
            # untouched keys keep their rows
            cold = np.setdiff1d(np.arange(0, R, 997, dtype=np.int64), uids)[:2048]
            np.testing.assert_array_equal(
                evs[t].sparse_read(torch.as_tensor(cold, device=DEV)).cpu().numpy(),
                orc.synth_rows(5000 + t, cold, D))
    finally:
        del evs
        _cleanup(dr)


def _din_ref(P, W, batch, dtype):
    uids, mids, cats, mid_his, cat_his, mask, target = batch
    B, T = mid_his.shape
    emb = torch.nn.functional.embedding
    PAD = -4294967296.0

    def lin(x, n):
        return x @ P[n + ".weight"].t() + P[n + ".bias"]

    def dice(x, n):
        mean = x.mean(0, keepdim=True)
        std = torch.sqrt(((x - mean) ** 2 + 1e-9).mean(0, keepdim=True))
        xp = torch.sigmoid((x - mean) / (std + 1e-9))
        return P[n + ".alpha"] * (1.0 - xp) * x + xp * x

    uid_e = emb(uids, W[0])
    item = torch.cat([emb(mids, W[1]), emb(cats, W[2])], 1)
    facts = torch.cat([emb(mid_his, W[1]), emb(cat_his, W[2])], 2)
    q = item.unsqueeze(1).expand(-1, T, -1)
    din_all = torch.cat([q, facts, q - facts, q * facts], -1)
    h = torch.sigmoid(lin(din_all, "f1_att"))
    h = torch.sigmoid(lin(h, "f2_att"))
    scores = lin(h, "f3_att").view(B, T)
    s = torch.where(mask.to(dtype) == 1, scores, torch.full_like(scores, PAD))
    a = torch.softmax(s, -1)
    att = torch.bmm(a.unsqueeze(1), facts).squeeze(1)
    his_sum = facts.sum(1)
    inp = torch.cat([uid_e, item, his_sum, item * his_sum, att], -1)
    bn = inp * (1.0 / (1.0 + 1e-3) ** 0.5) * P["bn1_gamma"] + P["bn1_beta"]
    x = dice(lin(bn, "dnn1"), "dice_1")
    x = dice(lin(x, "dnn2"), "dice_2")
    y = torch.softmax(lin(x, "dnn3"), -1) + 1e-8
    return -(torch.log(y) * target.to(dtype)).mean(), facts


def test_config3_din_full_size_step():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    _cleanup(dr)
    torch.manual_seed(3)
    D, B, T, lr = 18, 4096, 100, 0.05
    R = [500_000, 400_000, 2_000]
    gen = torch.Generator(device="cpu").manual_seed(8)
    tables = [torch.randn(r, D, generator=gen) * 0.1 for r in R]
    evs = []
    for t, w in enumerate(tables):
        ev = dr.EmbeddingVariable("c3_%d" % t, D, 0.0, device=DEV)
        ev.insert(torch.arange(w.shape[0], device=DEV), w.to(DEV))
        evs.append(ev)
    try:
        model = mz.DIN(*evs).to(DEV)
        uids = torch.randint(0, R[0], (B,), device=DEV)
        mids = torch.randint(0, R[1], (B,), device=DEV)
        cats = torch.randint(0, R[2], (B,), device=DEV)
        lens = torch.randint(1, T + 1, (B,), device=DEV)           # U[1, 100]
        mask = (torch.arange(T, device=DEV)[None, :] < lens[:, None]).float()
        mid_his = torch.randint(1, R[1], (B, T), device=DEV) * mask.long()   # zero padded
        cat_his = torch.randint(1, R[2], (B, T), device=DEV) * mask.long()
        lab = (torch.rand(B, device=DEV) > 0.5).long()
        target = torch.stack([lab, 1 - lab], 1).float()
        batch = (uids, mids, cats, mid_his, cat_his, mask, target)
        # the history lookup (B * T = 409 600 ids, ~half of them padding id 0)
        # is a pure row copy: bit-exact to the fp32 tables
        with torch.no_grad():
            his = torch.stack([mid_his.reshape(-1), cat_his.reshape(-1)])
            facts = model.item_lookup(his).view(B, T, -1)
        W32 = [t.to(DEV) for t in tables]
        want = torch.cat([torch.nn.functional.embedding(mid_his, W32[1]),
                          torch.nn.functional.embedding(cat_his, W32[2])], 2)
        assert torch.equal(facts, want)
        P = {k: v.detach().double().clone().requires_grad_(True)
             for k, v in model.state_dict().items()}
        W = [t.to(DEV).double().requires_grad_(True) for t in tables]
        ref_loss, _ = _din_ref(P, W, batch, torch.float64)
        ref_loss.backward()
        dopt = torch.optim.SGD(model.parameters(), lr=lr)
        loss = mz.din_train_step(model, batch, dopt, dr.GradientDescentOptimizer(lr))
        dr.status_check()
        torch.testing.assert_close(loss.double(), ref_loss.detach(), rtol=1e-5, atol=1e-6)
        for name, prm in model.named_parameters():
            wantp = (P[name] - lr * P[name].grad).detach()
            torch.testing.assert_close(prm.detach().double(), wantp, rtol=1e-5, atol=1e-6)
        for t in range(3):
            k, v = evs[t].export()[:2]
            rows = torch.zeros(R[t], D, device=DEV, dtype=torch.float64)
            rows[k] = v.double()
            wantw = (W[t] - lr * W[t].grad).detach()
            torch.testing.assert_close(rows, wantw, rtol=1e-5, atol=1e-6)
    finally:
        del evs
        _cleanup(dr)


def test_config4_crossnet_full_size_sampled_fp64():
    from deeprec_amd import ops
    B, d = 65536, 3392
    g = torch.Generator(device="cpu").manual_seed(2024)
    x0 = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    xl = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(d, d, generator=g) / d ** 0.5).to(DEV, torch.bfloat16)
    b = (torch.randn(d, generator=g) * 0.1).to(DEV)
    out, lin = ops.crossnet_forward(x0, xl, W, b)
    torch.cuda.synchronize()
    rows = torch.as_tensor(np.random.default_rng(4).choice(B, 512, replace=False), device=DEV)
    wlin = xl[rows].double() @ W.double().t() + b.double()
    want = x0[rows].double() * wlin + xl[rows].double()
    for got, ref in ((out[rows], want), (lin[rows], wlin)):
        err = (got.double() - ref).abs()
        bound = 2.0 ** -8 * ref.abs() + 1e-3 * ref.abs().max()
        assert bool((err <= bound).all()), float((err - bound).max())
    # the whole output is finite and repeatable launch to launch
    out2, lin2 = ops.crossnet_forward(x0, xl, W, b)
    assert torch.equal(out2, out) and torch.equal(lin2, lin)
    assert bool(torch.isfinite(out.float()).all())
