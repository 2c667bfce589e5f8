"""DCN-v2 cross layer (BASELINE configs[4]) on the bf16 MFMA kernel against a
plain PyTorch fp32 reference of x0 * (xl W^T + b) + xl computed from the same
bf16 operands, its backward against torch autograd, and one DCNv2 training
step against an fp32 torch model with dense tables.

Tolerances are bf16 ones, stated per assertion: the kernel rounds its
outputs to bf16 (relative step 2^-8) after an fp32-accumulated K sum, so
outputs are compared at 1/64 of the reference's max magnitude."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref(x0, xl, W, b):
    lin = xl.float() @ W.float().t() + b
    return x0.float() * lin + xl.float(), lin


def _close(got, want, frac=1.0 / 64):
    err = (got.float() - want.float()).abs().max().item()
    assert err <= frac * want.float().abs().max().item() + 1e-2, err


@pytest.mark.parametrize("B,d", [(300, 192), (129, 3392), (64, 64)])
def test_crossnet_forward_matches_torch(B, d):
    from deeprec_amd import ops
    g = torch.Generator(device="cpu").manual_seed(B + d)
    x0 = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    xl = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(d, d, generator=g) / d ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(d, generator=g).to(DEV)
    out, lin = ops.crossnet_forward(x0, xl, W, b)
    want, wlin = _ref(x0, xl, W, b)
    _close(out, want)
    _close(lin, wlin)
    out2, none = ops.crossnet_forward(x0, xl, W, None, with_lin=False)
    assert none is None
    _close(out2, _ref(x0, xl, W, torch.zeros(d, device=DEV))[0])


def test_crossnet_layer_unpadded_d_matches_torch():
    from deeprec_amd import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    B, d = 70, 13 + 26 * 16                       # 429: zero-padded to 448 inside
    x0 = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    xl = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(d, d, generator=g) / d ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(d, generator=g).to(DEV)
    _close(ops.crossnet_layer(x0, xl, W, b), _ref(x0, xl, W, b)[0])


def test_cross_layer_backward_matches_autograd():
    from deeprec_amd.modelzoo import CrossLayer
    g = torch.Generator(device="cpu").manual_seed(9)
    B, d = 256, 128
    x0 = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    xl = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(d, d, generator=g) / d ** 0.5).to(DEV)
    b = torch.randn(d, generator=g).to(DEV)
    G = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    a0, al = x0.clone().requires_grad_(True), xl.clone().requires_grad_(True)
    w, bb = W.clone().requires_grad_(True), b.clone().requires_grad_(True)
    CrossLayer.apply(a0, al, w, bb).backward(G)
    r0, rl = x0.float().requires_grad_(True), xl.float().requires_grad_(True)
    rw, rb = W.to(torch.bfloat16).float().requires_grad_(True), b.clone().requires_grad_(True)
    (r0 * (rl @ rw.t() + rb) + rl).backward(G.float())
    for got, want in ((a0.grad, r0.grad), (al.grad, rl.grad), (w.grad, rw.grad), (bb.grad, rb.grad)):
        _close(got, want, frac=1.0 / 32)


@pytest.mark.parametrize("B,d", [(300, 192), (1000, 3392), (64, 64)])
def test_crossnet_backward_elem_matches_torch(B, d):
    """dr_crossnet_backward_elem_bf16: u = bf16(g * x0) bit-exact to torch's
    bf16 multiply, acc + g * lin in fp32 and db = column sums of u against
    fp64 references (fp32 rounding tolerance); repeated launches are
    bit-identical (fixed-order column sums)."""
    from deeprec_amd import ops
    gen = torch.Generator(device="cpu").manual_seed(B * 7 + d)
    g, x0, lin = (torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16) for _ in range(3))
    acc0 = torch.randn(B, d, generator=gen).to(DEV)
    u, acc, db = ops.crossnet_backward_elem(g, x0, lin, acc0.clone())
    assert torch.equal(u, g * x0)
    want = acc0.double() + g.double() * lin.double()
    assert (acc.double() - want).abs().max().item() <= 1e-6 * want.abs().max().item()
    wdb = u.double().sum(0)
    assert (db.double() - wdb).abs().max().item() <= 1e-5 * (u.double().abs().sum(0).max().item())
    u2, acc2, db2 = ops.crossnet_backward_elem(g, x0, lin, None)
    assert torch.equal(u2, u) and torch.equal(db2, db)
    assert torch.equal(acc2, (g.float() * lin.float()))


@pytest.mark.parametrize("B,d", [(300, 192), (1000, 3392), (64, 64), (513, 448), (9472, 3392)])
def test_crossnet_dx_matches_torch(B, d):
    """dr_crossnet_dx_bf16 (dx = u W + g on the 256^2 MFMA schedule, W^T as
    the B operand) against the fp32 torch product from the same bf16
    operands (bf16 output tolerance) and the library's bf16 addmm; repeated
    launches bit-identical."""
    from deeprec_amd import ops
    gen = torch.Generator(device="cpu").manual_seed(B * 3 + d)
    u = torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16)
    g = torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16)
    W = (torch.randn(d, d, generator=gen) / d ** 0.5).to(DEV, torch.bfloat16)
    dx = ops.crossnet_dx(u, W.t().contiguous(), g)
    want = u.float() @ W.float() + g.float()
    _close(dx, want)
    _close(dx, torch.addmm(g, u, W))
    for _ in range(3):
        assert torch.equal(ops.crossnet_dx(u, W.t().contiguous(), g), dx)


@pytest.mark.parametrize("kernel,order", [("w4", "4"), ("w4", "0"), ("w4", "14"), ("w4", "xcd"),
                                          ("8ph", "4")])
@pytest.mark.parametrize("B,d", [(1024, 192), (4096, 3392), (64, 64), (2048, 448),
                                 (65536, 3392)])
def test_crossnet_dw_matches_fp64(B, d, kernel, order, monkeypatch):
    """dr_crossnet_dw_bf16 (dW = u^T x in TN form, batch slices summed in
    order) on each kernel (w4 = one wave per SIMD, the default, in tile-major
    and slice-major work orders; 8ph = the 256^2 eight-phase A/B): against the
    fp64 product of the same bf16 operands, within fp32 accumulation error
    (each entry a sum of B products: |err| <= 2^-22 sqrt(B) max|row
    norms|-scale bound, checked as 1e-5 of the entry scale), and
    bit-identical across launches."""
    from deeprec_amd import ops
    monkeypatch.setenv("DR_CROSSNET_DW_KERNEL", kernel)
    monkeypatch.setenv("DR_CROSSNET_DW_ORDER", order)
    gen = torch.Generator(device="cpu").manual_seed(B + 7 * d)
    u = torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16)
    x = torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16)
    dw = ops.crossnet_dw(u, x)
    assert dw is not None and dw.dtype == torch.float32 and dw.shape == (d, d)
    if B * d * d <= 4096 * 3392 * 3392:
        want = u.double().t() @ x.double()
    else:   # sampled rows / columns of the full-size product
        idx = torch.arange(0, d, 53, device=DEV)
        want = u.double()[:, idx].t() @ x.double()
        dw = dw[idx]
    scale = float(B) ** 0.5
    err = float((dw.double() - want).abs().max())
    assert err <= 1e-5 * scale * 4, (err, scale)
    full = ops.crossnet_dw(u, x)
    for _ in range(2):
        assert torch.equal(ops.crossnet_dw(u, x), full)


def test_cross_stack_backward_matches_autograd():
    """CrossStack (3 layers, one fused elementwise pass per layer in the
    backward) against torch autograd of the fp32 composition from the same
    bf16 operands: bf16 tolerances as the single layer."""
    from deeprec_amd.modelzoo import CrossStack
    gen = torch.Generator(device="cpu").manual_seed(11)
    B, d, L = 384, 192, 3
    x0 = torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16)
    Ws = [(torch.randn(d, d, generator=gen) / d ** 0.5).to(DEV) for _ in range(L)]
    bs = [(torch.randn(d, generator=gen) * 0.1).to(DEV) for _ in range(L)]
    G = torch.randn(B, d, generator=gen).to(DEV, torch.bfloat16)
    a0 = x0.clone().requires_grad_(True)
    ws = [w.clone().requires_grad_(True) for w in Ws]
    bb = [b.clone().requires_grad_(True) for b in bs]
    out = CrossStack.apply(a0, *ws, *bb)
    out.backward(G)
    r0 = x0.float().requires_grad_(True)
    rw = [w.to(torch.bfloat16).float().requires_grad_(True) for w in Ws]
    rb = [b.clone().requires_grad_(True) for b in bs]
    x = r0
    for w, b in zip(rw, rb):
        x = r0 * (x @ w.t() + b) + x
    _close(out, x.detach(), frac=1.0 / 32)
    x.backward(G.float())
    _close(a0.grad, r0.grad, frac=1.0 / 16)
    for got, want in zip(ws + bb, rw + rb):
        _close(got.grad, want.grad, frac=1.0 / 16)


@pytest.mark.parametrize("bf16", [False, True])
def test_dcn_train_step_matches_torch_reference(bf16):
    """bf16=False: deep MLP under autocast; True: the deep MLP and the output
    layer on the hand MFMA tower node (needs B % 512 == 0 and widths that are
    multiples of 64), x0 cast straight into its bf16 buffer."""
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    torch.manual_seed(13)
    T, R, D, lr = 4, 50, 16, 0.05
    B, deep = (512, (128, 64)) if bf16 else (256, (64, 32))
    gen = torch.Generator(device="cpu").manual_seed(6)
    tables = [torch.randn(R, D, generator=gen) * 0.1 for _ in range(T)]
    evs = []
    for t, w in enumerate(tables):
        ev = dr.EmbeddingVariable("dcn_%d" % t, D, 0.0, device=DEV)
        ev.insert(torch.arange(R, device=DEV), w.to(DEV))
        evs.append(ev)
    model = mz.DCNv2(evs, 13, layers=2, deep=deep, bf16=bf16).to(DEV)
    ids = torch.randint(0, R, (T, B), device=DEV)
    dense = torch.randn(B, 13, device=DEV)
    labels = (torch.rand(B, device=DEV) > 0.5).float()
    P = {k.replace("deep.net.", "deep."): v.detach().clone()
         for k, v in model.state_dict().items()}
    # fp32 torch reference of the same model (bf16 rounding of x0 and of the
    # cross weights as in the kernel path; everything else fp32)
    W = [t.to(DEV).clone().requires_grad_(True) for t in tables]
    emb = torch.cat([torch.nn.functional.embedding(ids[t], W[t]) for t in range(T)], 1)
    x0 = torch.cat([dense, emb, torch.zeros(B, model.dp - model.d, device=DEV)], 1)
    x = x0
    for i in range(2):
        wi = P["cross_w.%d" % i].to(torch.bfloat16).float()
        x = x0 * (x @ wi.t() + P["cross_b.%d" % i]) + x
    h = x
    for i in range(2):
        h = torch.relu(h @ P["deep.%d.weight" % (2 * i)].t() + P["deep.%d.bias" % (2 * i)])
    pred = torch.sigmoid(h @ P["last.weight"].t() + P["last.bias"]).squeeze(1)
    p = pred.clamp(1e-7, 1 - 1e-7)
    ref_loss = -(labels * torch.log(p) + (1 - labels) * torch.log(1 - p)).mean()
    ref_loss.backward()
    before = [_rows(ev, R) for ev in evs]
    dopt = torch.optim.SGD(model.parameters(), lr=lr)
    loss = mz.train_step(model, dense, ids, labels, dopt, dr.GradientDescentOptimizer(lr))
    assert abs(loss.item() - ref_loss.item()) <= 2e-2 * abs(ref_loss.item())   # bf16 path
    for t in range(T):
        got = (before[t] - _rows(evs[t], R)) / lr                 # the applied EV gradient
        _close(got, W[t].grad, frac=1.0 / 16)


def _rows(ev, R):
    k, v = ev.export()[:2]
    out = torch.zeros(R, ev.dim, device=DEV)
    out[k] = v
    return out


@pytest.mark.parametrize("B,d", [(4096, 3392), (1000, 512), (9472, 3392)])
def test_crossnet_large_tile_repeatable(B, d):
    """The 256 x 256 glds kernel at the DCN width over many full and partial
    tiles: within bf16 tolerance of torch, and bit-identical over repeated
    launches (an LDS staging race would show as launch-to-launch drift)."""
    from deeprec_amd import ops
    g = torch.Generator(device="cpu").manual_seed(B ^ d)
    x0 = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    xl = torch.randn(B, d, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(d, d, generator=g) / d ** 0.5).to(DEV, torch.bfloat16)
    b = torch.randn(d, generator=g).to(DEV)
    out, lin = ops.crossnet_forward(x0, xl, W, b)
    want, wlin = _ref(x0, xl, W, b)
    _close(out, want)
    _close(lin, wlin)
    for _ in range(6):
        o2, l2 = ops.crossnet_forward(x0, xl, W, b)
        assert torch.equal(o2, out) and torch.equal(l2, lin)
