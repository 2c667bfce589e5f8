"""KV FTRL (KvResourceSparseApplyFtrl[V2], training_ali_ops.cc:167-331)
against the oracle's restatement, and one WDL training step
(modelzoo/WDL/train.py, BASELINE configs[0]) against a plain torch fp32 model.

FTRL tolerance: 1e-5 relative (north_star's fp32 bound) -- the row norm of
`linear` is an fp32 reduction whose order is not the oracle's (nor Eigen's),
everything else is the same scalar formula.  The WDL step compares at rtol
1e-5 / atol 1e-6 like the other model tests."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


@pytest.mark.parametrize("D", [1, 3, 16, 64])
@pytest.mark.parametrize("variant", ["ftrl", "ftrl_l1", "ftrl_v2_pow"])
def test_ev_ftrl_matches_oracle(orc, D, variant):
    import deeprec_amd as dr
    dr.load()
    dr.set_validate(True)
    lr, l1, l2, lr_power, shr = 0.2, 0.0, 0.0, -0.5, 0.0
    if variant == "ftrl_l1":
        l1, l2 = 0.05, 0.01                        # rows with |linear| <= l1 -> var = 0
    elif variant == "ftrl_v2_pow":
        l2, lr_power, shr = 0.01, -0.7, 0.02       # powf path, FtrlV2 shrinkage
    rng = np.random.default_rng(D * 31 + len(variant))
    ev = dr.EmbeddingVariable("ftrl_%s_%d" % (variant, D), D, 0.3)
    oev = orc.EV(D, 0.3)
    oacc, olin = oev.create_slot(1, 0.1), oev.create_slot(2, 0.0)
    opt = dr.FtrlOptimizer(lr, lr_power, 0.1, l1, l2, shr)
    for step in range(4):
        ids = rng.choice(200, 60, replace=False).astype(np.int64)
        g = (rng.standard_normal((60, D)) * 0.1).astype(np.float32)
        ev.pending_grads.append(dr.IndexedSlices(T(g), T(ids)))
        opt.apply_gradients([ev], global_step=step)
        oev.apply_ftrl(oacc, olin, lr, l1, l2, lr_power, shr, g, ids, step)
    keys = np.arange(200, dtype=np.int64)
    got = ev.sparse_read(T(keys)).cpu().numpy()
    want = oev.gather(keys)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)
    acc = ev.slot("Ftrl", 0.1).sparse_read(T(keys)).cpu().numpy()
    np.testing.assert_allclose(acc, oacc.gather(keys), rtol=1e-6)
    if variant == "ftrl_l1" and D <= 3:   # short rows: some |linear| stay <= l1
        assert (got == 0).any()


def test_ev_ftrl_rejects_bad_scalars():
    import deeprec_amd as dr
    from deeprec_amd._lib import DeepRecError
    ev = dr.EmbeddingVariable("ftrl_bad", 4, 0.0)
    ev.pending_grads.append(dr.IndexedSlices(torch.ones(2, 4, device=DEV),
                                             torch.arange(2, device=DEV)))
    with pytest.raises(DeepRecError):
        dr.FtrlOptimizer(0.1, learning_rate_power=0.5).apply_gradients([ev])


def _evs(dr, name, tables):
    evs = []
    for t, w in enumerate(tables):
        ev = dr.EmbeddingVariable("%s_%d" % (name, t), w.shape[1], 0.0, device=DEV)
        ev.insert(torch.arange(w.shape[0], device=DEV), w.to(DEV))
        evs.append(ev)
    return evs


def _rows(ev, R):
    k, v = ev.export()[:2]
    out = torch.zeros(R, ev.dim, device=DEV)
    out[k] = v
    return out


def test_wdl_train_step_matches_torch_reference():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    torch.manual_seed(21)
    cats = ["C1", "C2", "C10", "C11"]
    dims = [8, 8, 16, 8]                               # mixed dims, like EMBEDDING_DIMENSIONS
    nums = ["I1", "I2", "I10"]
    R, B, lr = 40, 128, 0.05
    g = torch.Generator(device="cpu").manual_seed(8)
    deep_t = [torch.randn(R, d, generator=g) * 0.1 for d in dims]
    wide_t = [torch.randn(R, 1, generator=g) * 0.1 for _ in dims]
    model = mz.WDL(cats, _evs(dr, "wdl_d", deep_t), _evs(dr, "wdl_w", wide_t), nums,
                   hidden=(32, 16)).to(DEV)
    with torch.no_grad():
        model.linear_num.copy_(torch.randn(3, 1) * 0.1)
        model.linear_bias.fill_(0.05)
    ids = torch.randint(0, R, (len(cats), B), device=DEV)
    ids[:, :8] = 3
    dense = torch.rand(B, len(nums), device=DEV)
    labels = (torch.rand(B, device=DEV) > 0.5).float()

    P = {k: v.detach().clone().requires_grad_(True) for k, v in model.named_parameters()}
    Wd = [t.to(DEV).clone().requires_grad_(True) for t in deep_t]
    Ww = [t.to(DEV).clone().requires_grad_(True) for t in wide_t]
    emb = {c: torch.nn.functional.embedding(ids[i], Wd[i]) for i, c in enumerate(cats)}
    cols = {c + "_embedding": emb[c] for c in cats}
    cols.update({n: dense[:, j:j + 1] for j, n in enumerate(nums)})
    x = torch.cat([cols[k] for k in sorted(cols)], 1)         # input_layer order
    for i in range(2):
        x = torch.relu(x @ P["dnn.%d.weight" % (2 * i)].t() + P["dnn.%d.bias" % (2 * i)])
    deep = x @ P["logits.weight"].t() + P["logits.bias"]
    wide = sum(torch.nn.functional.embedding(ids[i], Ww[i]) for i in range(len(cats)))
    logit = (deep + wide + dense @ P["linear_num"] + P["linear_bias"]).squeeze(1)
    ref_loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, labels)
    ref_loss.backward()

    deep_opt = torch.optim.SGD(model.deep_parameters(), lr=lr)
    wide_opt = torch.optim.SGD(model.wide_parameters(), lr=lr)
    sgd = dr.GradientDescentOptimizer(lr)
    loss = mz.wdl_train_step(model, dense, ids, labels, deep_opt, sgd, wide_opt, sgd)
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=1e-5, atol=1e-6)
    for name, prm in model.named_parameters():
        want = P[name] - lr * P[name].grad
        torch.testing.assert_close(prm.detach(), want.detach(), rtol=1e-5, atol=1e-6)
    for i in range(len(cats)):
        torch.testing.assert_close(_rows(model.deep_evs[i], R), (Wd[i] - lr * Wd[i].grad).detach(),
                                   rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(_rows(model.wide_evs[i], R), (Ww[i] - lr * Ww[i].grad).detach(),
                                   rtol=1e-5, atol=1e-6)


def test_wdl_reference_optimizers_step():
    """The reference's optimizer pairing (Adagrad deep, FTRL linear) runs and
    moves every variable kind."""
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    torch.manual_seed(22)
    cats, dims, nums, R, B = ["C1", "C2"], [8, 16], ["I1"], 30, 64
    g = torch.Generator(device="cpu").manual_seed(9)
    model = mz.WDL(cats, _evs(dr, "wdl2_d", [torch.randn(R, d, generator=g) for d in dims]),
                   _evs(dr, "wdl2_w", [torch.randn(R, 1, generator=g) for _ in dims]), nums,
                   hidden=(16,)).to(DEV)
    ids = torch.randint(0, R, (2, B), device=DEV)
    dense = torch.rand(B, 1, device=DEV)
    labels = (torch.rand(B, device=DEV) > 0.5).float()
    before = [_rows(ev, R).clone() for ev in model.evs]
    deep_opt = torch.optim.Adagrad(model.deep_parameters(), lr=0.01, initial_accumulator_value=0.1)
    ftrl = dr.FtrlOptimizer(0.2)
    for step in range(2):
        loss = mz.wdl_train_step(model, dense, ids, labels, deep_opt, dr.AdagradOptimizer(0.01),
                                 ftrl, ftrl, global_step=step)
    assert torch.isfinite(loss)
    for ev, b in zip(model.evs, before):
        assert not torch.equal(_rows(ev, R), b)
    assert float(model.linear_bias.detach().abs()) > 0


def test_ev_ftrl_empty_and_first_touch_slots(orc):
    """n = 0 is a no-op; a key first seen by the apply starts from the
    variable's and the slots' defaults (LookupOrCreateKey)."""
    import deeprec_amd as dr
    ev = dr.EmbeddingVariable("ftrl_edge", 4, 0.5)
    opt = dr.FtrlOptimizer(0.1, l1_regularization_strength=0.0)
    ev.pending_grads.append(dr.IndexedSlices(torch.zeros(0, 4, device=DEV),
                                             torch.zeros(0, dtype=torch.int64, device=DEV)))
    opt.apply_gradients([ev], global_step=0)
    assert int(ev.total_count()[0]) == 0
    g = np.full((1, 4), 0.25, np.float32)
    ev.pending_grads.append(dr.IndexedSlices(T(g), T([42])))
    opt.apply_gradients([ev], global_step=1)
    oev = orc.EV(4, 0.5)
    oacc, olin = oev.create_slot(1, 0.1), oev.create_slot(2, 0.0)
    oev.apply_ftrl(oacc, olin, 0.1, 0.0, 0.0, -0.5, 0.0, g, np.array([42]), 1)
    np.testing.assert_allclose(ev.sparse_read(T([42])).cpu().numpy(), oev.gather(np.array([42])),
                               rtol=1e-6)
