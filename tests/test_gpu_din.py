"""DIN user-behaviour attention (seq.hip) against plain PyTorch references of
modelzoo/DIN/script/utils.py:264-309 (din_attention, mode 'SUM') and
script/model.py:94-98,381-392, and one DIN training step (modelzoo.DIN)
against a torch fp32 model with dense tables.

Tolerances: the kernels vs an fp64 torch reference at rtol/atol 1e-5 (fp32
sums of <= 150 terms); the model step at fp32 rtol 1e-5 / atol 1e-6 like the
other model tests (north_star's 1e-5 rel)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PAD = -4294967296.0     # float32(-2**32 + 1), utils.py:291


def _ref_din_input(q, f):
    T = f.shape[1]
    qq = q.unsqueeze(1).expand(-1, T, -1)
    return torch.cat([qq, f, qq - f, qq * f], -1)


def _ref_pool(scores, mask, f):
    s = torch.where(mask == 1, scores, torch.full_like(scores, PAD))
    a = torch.softmax(s, -1)
    return torch.bmm(a.unsqueeze(1), f).squeeze(1), f.sum(1), a


def _case(B, T, H, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    q = torch.randn(B, H, generator=g, dtype=torch.float64)
    f = torch.randn(B, T, H, generator=g, dtype=torch.float64)
    lens = torch.randint(0, T + 1, (B,), generator=g)
    lens[0] = T
    if B > 1:
        lens[1] = 0                       # every position masked: uniform softmax
    mask = (torch.arange(T)[None, :] < lens[:, None]).double()
    scores = torch.randn(B, T, generator=g, dtype=torch.float64) * 3
    return [x.to(DEV) for x in (q, f, mask, scores)]


SHAPES = [(64, 100, 36), (33, 1, 36), (17, 150, 18), (9, 7, 5), (5, 65, 256), (3, 9, 64)]


@pytest.mark.parametrize("B,T,H", SHAPES)
def test_din_attention_input_fwd_bwd(B, T, H):
    from deeprec_amd import ops
    q, f, _, _ = _case(B, T, H, B + T + H)
    got = ops.din_attention_input(q.float(), f.float())
    want = _ref_din_input(q.float(), f.float())
    assert torch.equal(got, want)                       # pure copies / one op each: exact
    g = torch.randn(B, T, 4 * H, device=DEV, dtype=torch.float64)
    qr, fr = q.clone().requires_grad_(True), f.clone().requires_grad_(True)
    _ref_din_input(qr, fr).backward(g)
    gq, gf = ops.din_attention_input_grad(q.float(), f.float(), g.float())
    torch.testing.assert_close(gq.double(), qr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gf.double(), fr.grad, rtol=1e-5, atol=1e-5)
    # accumulate into an existing gradient
    base = torch.randn(B, T, H, device=DEV)
    acc = base.clone()
    ops.din_attention_input_grad(q.float(), f.float(), g.float(), grad_facts=acc)
    torch.testing.assert_close(acc.double(), base.double() + fr.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,T,H", SHAPES)
def test_din_attention_pool_fwd_bwd(B, T, H):
    from deeprec_amd import ops
    q, f, mask, scores = _case(B, T, H, 7 * B + T + H)
    att, hs, al = ops.din_attention_pool(scores.float(), mask.float(), f.float())
    w_att, w_hs, w_al = _ref_pool(scores, mask, f)
    torch.testing.assert_close(al.double(), w_al, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(att.double(), w_att, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(hs.double(), w_hs, rtol=1e-5, atol=1e-5)
    if B > 1:   # fully masked row -> 1/T each (softmax of equal paddings)
        torch.testing.assert_close(al[1], torch.full((T,), 1.0 / T, device=DEV))
    ga = torch.randn(B, H, device=DEV, dtype=torch.float64)
    gs = torch.randn(B, H, device=DEV, dtype=torch.float64)
    sr, fr = scores.clone().requires_grad_(True), f.clone().requires_grad_(True)
    a_, s_, _ = _ref_pool(sr, mask, fr)
    (a_ * ga).sum().add_((s_ * gs).sum()).backward()
    gsc, gf = ops.din_attention_pool_grad(al, mask.float(), f.float(), ga.float(), gs.float())
    torch.testing.assert_close(gsc.double(), sr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gf.double(), fr.grad, rtol=1e-5, atol=1e-5)
    assert torch.all(gsc[mask == 0] == 0)


def test_din_attention_rejects_bad_shapes():
    from deeprec_amd import ops
    from deeprec_amd._lib import DeepRecError
    f = torch.zeros(2, 3, 300, device=DEV)                   # H > 256
    with pytest.raises(DeepRecError):
        ops.din_attention_input(torch.zeros(2, 300, device=DEV), f)
    with pytest.raises(DeepRecError):                        # T == 0 has no softmax
        ops.din_attention_pool(torch.zeros(2, 0, device=DEV), torch.zeros(2, 0, device=DEV),
                               torch.zeros(2, 0, 8, device=DEV))


def _evs(dr, name, tables):
    evs = []
    for t, w in enumerate(tables):
        ev = dr.EmbeddingVariable("%s_%d" % (name, t), w.shape[1], 0.0, device=DEV)
        ev.insert(torch.arange(w.shape[0], device=DEV), w.to(DEV))
        evs.append(ev)
    return evs


def _ev_rows(ev, R):
    k, v = ev.export()[:2]
    out = torch.zeros(R, ev.dim, device=DEV)
    out[k] = v
    return out


def test_din_train_step_matches_torch_reference():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    torch.manual_seed(11)
    D, B, T, lr = 18, 96, 23, 0.05
    R = [40, 60, 12]                                    # uid, mid, cat vocab
    g = torch.Generator(device="cpu").manual_seed(4)
    tables = [torch.randn(r, D, generator=g) * 0.1 for r in R]
    evs = _evs(dr, "din", tables)
    model = mz.DIN(*evs).to(DEV)
    uids = torch.randint(0, R[0], (B,), device=DEV)
    mids = torch.randint(0, R[1], (B,), device=DEV)
    cats = torch.randint(0, R[2], (B,), device=DEV)
    lens = torch.randint(1, T + 1, (B,), device=DEV)
    mask = (torch.arange(T, device=DEV)[None, :] < lens[:, None]).float()
    mid_his = torch.randint(1, R[1], (B, T), device=DEV) * mask.long()     # zero padded
    cat_his = torch.randint(1, R[2], (B, T), device=DEV) * mask.long()
    lab = (torch.rand(B, device=DEV) > 0.5).long()
    target = torch.stack([lab, 1 - lab], 1).float()

    P = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    W = [t.to(DEV).clone().requires_grad_(True) for t in tables]

    def lin(x, n):
        return x @ P[n + ".weight"].t() + P[n + ".bias"]

    def dice(x, n):
        mean = x.mean(0, keepdim=True)
        std = torch.sqrt(((x - mean) ** 2 + 1e-9).mean(0, keepdim=True))
        xp = torch.sigmoid((x - mean) / (std + 1e-9))
        return P[n + ".alpha"] * (1.0 - xp) * x + xp * x

    emb = torch.nn.functional.embedding
    uid_e = emb(uids, W[0])
    item = torch.cat([emb(mids, W[1]), emb(cats, W[2])], 1)
    facts = torch.cat([emb(mid_his, W[1]), emb(cat_his, W[2])], 2)
    h = torch.sigmoid(lin(_ref_din_input(item, facts), "f1_att"))
    h = torch.sigmoid(lin(h, "f2_att"))
    scores = lin(h, "f3_att").view(B, T)
    att, his_sum, _ = _ref_pool(scores, mask, facts)
    inp = torch.cat([uid_e, item, his_sum, item * his_sum, att], -1)
    bn = inp * (1.0 / (1.0 + 1e-3) ** 0.5) * P["bn1_gamma"] + P["bn1_beta"]
    x = dice(lin(bn, "dnn1"), "dice_1")
    x = dice(lin(x, "dnn2"), "dice_2")
    y = torch.softmax(lin(x, "dnn3"), -1) + 1e-8
    ref_loss = -(torch.log(y) * target).mean()
    ref_loss.backward()

    dopt = torch.optim.SGD(model.parameters(), lr=lr)
    batch = (uids, mids, cats, mid_his, cat_his, mask, target)
    loss = mz.din_train_step(model, batch, dopt, dr.GradientDescentOptimizer(lr))
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=1e-5, atol=1e-6)
    for name, prm in model.named_parameters():
        want = P[name] - lr * P[name].grad
        torch.testing.assert_close(prm.detach(), want.detach(), rtol=1e-5, atol=1e-6)
    for t in range(3):
        want = W[t] - lr * W[t].grad
        torch.testing.assert_close(_ev_rows(evs[t], R[t]), want.detach(), rtol=1e-5, atol=1e-6)


def test_din_attention_empty_batch():
    from deeprec_amd import ops
    f = torch.zeros(0, 5, 36, device=DEV)
    q = torch.zeros(0, 36, device=DEV)
    assert ops.din_attention_input(q, f).shape == (0, 5, 144)
    gq, gf = ops.din_attention_input_grad(q, f, torch.zeros(0, 5, 144, device=DEV))
    assert gq.shape == (0, 36) and gf.shape == (0, 5, 36)
    att, hs, al = ops.din_attention_pool(torch.zeros(0, 5, device=DEV),
                                         torch.zeros(0, 5, device=DEV), f)
    assert att.shape == (0, 36) and al.shape == (0, 5)
    gs, gf = ops.din_attention_pool_grad(al, torch.zeros(0, 5, device=DEV), f,
                                         torch.zeros(0, 36, device=DEV))
    assert gs.shape == (0, 5)


@pytest.mark.parametrize("wgrad", ["lib", "mfma", "valu"])
@pytest.mark.parametrize("B,T,H,prefix", [(64, 100, 36, True), (40, 23, 36, False),
                                          (8, 1, 36, True), (16, 9, 16, False),
                                          (12, 30, 64, True), (20, 17, 32, False)])
def test_din_fused_attention_matches_fp64(B, T, H, prefix, wgrad, monkeypatch):
    """DinAttentionFused (dr_din_mlp_forward / _backward + the pool kernels):
    the attention MLP over the valid positions only, din_all never formed
    (W1 split into its per-sample and per-position parts) -- forward and
    every gradient (query, facts, the three layers' weights and biases)
    against torch fp64 autograd of the reference composition (utils.py:
    264-309), prefix masks (zero-padded histories, a fully masked row) and
    arbitrary 0/1 masks.  Weight gradients every way: the hand split-K pass
    (dr_din_mlp_wgrad, the default when cap % 4 == 0) on the matrix cores or,
    DR_DIN_WGRAD_VALU=1, the VALU, and library GEMMs (DR_DIN_WGRAD=lib).
    The hand passes run with every per-position buffer NaN-filled first
    (DinMlpBuffers.fill): their columns past the valid count stay unwritten
    and must never be read."""
    from deeprec_amd import modelzoo as mz
    from deeprec_amd import ops
    monkeypatch.setattr(ops, "_DIN_WGRAD_HAND", wgrad != "lib")
    if wgrad != "lib":
        monkeypatch.setattr(ops.DinMlpBuffers, "fill", float("nan"))
    monkeypatch.setenv("DR_DIN_WGRAD_VALU", "1" if wgrad == "valu" else "0")
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + T + H)
    q = torch.randn(B, H, generator=g, dtype=torch.float64) * 0.5
    f = torch.randn(B, T, H, generator=g, dtype=torch.float64) * 0.5
    if prefix:
        lens = torch.randint(0, T + 1, (B,), generator=g)
        lens[0] = T
        if B > 1:
            lens[1] = 0
        mask = (torch.arange(T)[None, :] < lens[:, None]).double()
    else:
        mask = (torch.rand(B, T, generator=g) < 0.6).double()
    w1 = torch.randn(80, 4 * H, generator=g, dtype=torch.float64) / (4 * H) ** 0.5
    b1 = torch.randn(80, generator=g, dtype=torch.float64) * 0.1
    w2 = torch.randn(40, 80, generator=g, dtype=torch.float64) / 80 ** 0.5
    b2 = torch.randn(40, generator=g, dtype=torch.float64) * 0.1
    w3 = torch.randn(1, 40, generator=g, dtype=torch.float64) / 40 ** 0.5
    b3 = torch.randn(1, generator=g, dtype=torch.float64) * 0.1
    ga = torch.randn(B, H, generator=g, dtype=torch.float64)
    gsum = torch.randn(B, H, generator=g, dtype=torch.float64)
    ins = [x.to(DEV) for x in (q, f, mask, w1, b1, w2, b2, w3, b3)]
    ref = [x.clone().requires_grad_(x.dim() > 0 and i != 2) for i, x in enumerate(ins)]
    rq, rf, rm, rw1, rb1, rw2, rb2, rw3, rb3 = ref
    h = torch.sigmoid(_ref_din_input(rq, rf) @ rw1.t() + rb1)
    h = torch.sigmoid(h @ rw2.t() + rb2)
    scores = (h @ rw3.t() + rb3).view(B, T)
    att, hsum, _ = _ref_pool(scores, rm, rf)
    (att * ga.to(DEV)).sum().add_((hsum * gsum.to(DEV)).sum()).backward()
    got = [x.float().clone().requires_grad_(i != 2) for i, x in enumerate(ins)]
    gatt, ghs = mz.DinAttentionFused.apply(*got)
    torch.testing.assert_close(gatt.double(), att.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ghs.double(), hsum.detach(), rtol=1e-5, atol=1e-5)
    (gatt * ga.to(DEV).float()).sum().add_((ghs * gsum.to(DEV).float()).sum()).backward()
    for name, a, b in zip(("query", "facts", "mask", "w1", "b1", "w2", "b2", "w3", "b3"), got, ref):
        if name == "mask":
            continue
        # weight gradients sum B*T position terms: fp32 vs fp64 at 2e-5 of the
        # gradient's scale
        scale = float(b.grad.abs().max()) + 1e-12
        err = float((a.grad.double() - b.grad).abs().max())
        assert err <= 2e-5 * scale + 1e-6, (name, err, scale)


@pytest.mark.parametrize("B,n", [(4096, 200), (4096, 80), (37, 19), (1, 5), (300, 1)])
def test_din_dice_fused_matches_fp64(B, n):
    """dr_din_dice_forward / _backward (one kernel each way) against torch
    fp64 autograd of dice() (modelzoo/DIN/script/utils.py:12-35: batch mean,
    std = sqrt(mean((x - mean)^2 + eps)), p = sigmoid((x - mean) / (std +
    eps)), alpha (1 - p) x + p x): output, grad_x and grad_alpha within fp32
    accumulation error; bit-identical across launches."""
    from deeprec_amd import modelzoo as mz
    g = torch.Generator(device="cpu").manual_seed(B * 7 + n)
    x = (torch.randn(B, n, generator=g, dtype=torch.float64) * 2.0 + 0.5)
    alpha = torch.randn(n, generator=g, dtype=torch.float64) * 0.3
    gy = torch.randn(B, n, generator=g, dtype=torch.float64)
    eps = 1e-9
    rx, ra = x.clone().requires_grad_(True), alpha.clone().requires_grad_(True)
    mean = rx.mean(0, keepdim=True)
    std = torch.sqrt(((rx - mean) ** 2 + eps).mean(0, keepdim=True))
    p = torch.sigmoid((rx - mean) / (std + eps))
    ry = ra * (1.0 - p) * rx + p * rx
    (ry * gy).sum().backward()
    dice = mz.Dice(n, epsilon=eps).to(DEV)
    with torch.no_grad():
        dice.alpha.copy_(alpha.float())
    gx_in = x.float().to(DEV).requires_grad_(True)
    y = dice(gx_in)
    y.backward(gy.float().to(DEV))
    torch.testing.assert_close(y.double().cpu(), ry.detach(), rtol=1e-5, atol=1e-5)
    scale = float(rx.grad.abs().max()) + 1e-12
    assert float((gx_in.grad.double().cpu() - rx.grad).abs().max()) <= 1e-4 * scale + 1e-6
    scale = float(ra.grad.abs().max()) + 1e-12
    assert float((dice.alpha.grad.double().cpu() - ra.grad).abs().max()) <= 1e-4 * scale + 1e-5
    y2 = dice(gx_in.detach())
    assert torch.equal(y2, y.detach())


@pytest.mark.parametrize("B,Du,H", [(4096, 18, 36), (7, 5, 16), (1, 0, 4)])
def test_din_fcn_input_fused_matches_torch(B, Du, H):
    """dr_din_fcn_input_forward / _backward (model.py:118-124: inp = [uid,
    item, his_sum, item * his_sum, att], bn = inp * c * gamma + beta) against
    the torch composition in fp64: output and all six gradients."""
    from deeprec_amd import modelzoo as mz
    g = torch.Generator(device="cpu").manual_seed(B + Du + H)
    ts = [torch.randn(B, k, generator=g, dtype=torch.float64) for k in (Du, H, H, H)]
    gamma = torch.randn(Du + 4 * H, generator=g, dtype=torch.float64)
    beta = torch.randn(Du + 4 * H, generator=g, dtype=torch.float64)
    gout = torch.randn(B, Du + 4 * H, generator=g, dtype=torch.float64)
    c = 1.0 / (1.0 + 1e-3) ** 0.5
    ref = [t.clone().requires_grad_(True) for t in ts + [gamma, beta]]
    u, i, h, a, gm, bt = ref
    (torch.cat([u, i, h, i * h, a], -1) * c * gm + bt).mul(gout).sum().backward()
    got = [t.float().to(DEV).requires_grad_(True) for t in ts + [gamma, beta]]
    out = mz._DinFcnInputFn.apply(*got, c)
    want = torch.cat([u, i, h, i * h, a], -1) * c * gm + bt
    torch.testing.assert_close(out.double().cpu(), want.detach(), rtol=1e-5, atol=1e-5)
    out.backward(gout.float().to(DEV))
    for name, x, r in zip(("uid", "item", "his_sum", "att", "gamma", "beta"), got, ref):
        scale = float(r.grad.abs().max()) + 1e-12 if r.grad.numel() else 1.0
        err = float((x.grad.double().cpu() - r.grad).abs().max()) if r.grad.numel() else 0.0
        assert err <= 1e-5 * scale * max(1.0, B ** 0.5) + 1e-6, (name, err, scale)
