"""Model glue (modelzoo.py) against a plain PyTorch fp32 reference of the
same model: the interactions' backward kernels against torch autograd, and
one DLRM / DeepFM training step (loss, dense grads, EV rows after the KV
SGD step) against dense torch tables with the same weights.  fp32 tolerance
1e-5 relative (north_star), stated per assertion."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
RTOL, ATOL = 1e-5, 1e-6


def _tril_dot(X):
    F = X.shape[1]
    Z = torch.bmm(X, X.transpose(1, 2))
    i, j = torch.tril_indices(F, F, -1, device=X.device)
    return Z[:, i, j]


def test_dot_interaction_grad_matches_torch_autograd():
    from deeprec_amd import ops
    torch.manual_seed(0)
    for B, F, D in ((300, 27, 128), (77, 5, 16), (64, 32, 64)):
        X = torch.randn(B, F, D, device=DEV, dtype=torch.float64)
        G = torch.randn(B, F * (F - 1) // 2, device=DEV, dtype=torch.float64)
        Xr = X.clone().requires_grad_(True)
        _tril_dot(Xr).backward(G)
        got = ops.dot_interaction_grad(X.float(), G.float())
        torch.testing.assert_close(got.double(), Xr.grad, rtol=1e-4, atol=1e-4)


def test_fm2_grad_matches_torch_autograd():
    from deeprec_amd import ops
    torch.manual_seed(1)
    E = torch.randn(200, 26, 64, device=DEV, dtype=torch.float64)
    G = torch.randn(200, 64, device=DEV, dtype=torch.float64)
    Er = E.clone().requires_grad_(True)
    (0.5 * (Er.sum(1) ** 2 - (Er ** 2).sum(1))).backward(G)
    got = ops.fm_second_order_grad(E.float(), G.float())
    torch.testing.assert_close(got.double(), Er.grad, rtol=1e-4, atol=1e-4)


def _tables(T, R, D, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [torch.randn(R, D, generator=g) * 0.1 for _ in range(T)]


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


@pytest.mark.parametrize("model_name", ["dlrm", "deepfm"])
def test_model_train_step_matches_torch_reference(model_name):
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    torch.manual_seed(5)
    T, R, D, B, lr = 4, 50, 16, 256, 0.05
    tables = _tables(T, R, D, 3)
    evs = _evs(dr, "mz_" + model_name, tables)
    ids = torch.randint(0, R, (T, B), device=DEV)
    ids[:, :10] = 7                                     # duplicates -> summed grads
    dense = torch.randn(B, 13, device=DEV)
    labels = (torch.rand(B, device=DEV) > 0.5).float()
    if model_name == "dlrm":
        model = mz.DLRM(evs, 13, (32,), (32, 16)).to(DEV)
        wide_tables = []
    else:
        wide_tables = _tables(T, R, 1, 4)
        model = mz.DeepFM(evs, _evs(dr, "mzw", wide_tables), (32, 16), (16,)).to(DEV)
    # torch reference: identical dense weights, dense tables as leaves
    ref_model = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    W = [t.to(DEV).clone().requires_grad_(True) for t in tables]
    Ww = [t.to(DEV).clone().requires_grad_(True) for t in wide_tables]

    def lin(x, name):
        return x @ ref_model[name + ".weight"].t() + ref_model[name + ".bias"]

    def mlp(x, prefix, n, last_act=True):
        for i in range(n):
            x = lin(x, "%s.%d" % (prefix, 2 * i))
            if last_act or i < n - 1:
                x = torch.relu(x)
        return x

    emb = torch.cat([torch.nn.functional.embedding(ids[t], W[t]) for t in range(T)], 1)
    if model_name == "dlrm":
        x0 = mlp(dense, "bottom", 2)
        X = torch.cat([x0.unsqueeze(1), emb.view(B, T, D)], 1)
        net = mlp(torch.cat([x0, _tril_dot(X)], 1), "top", 2)
    else:
        wide = torch.cat([torch.nn.functional.embedding(ids[t], Ww[t]) for t in range(T)], 1)
        e3 = emb.view(B, T, D)
        fm = 0.5 * (e3.sum(1) ** 2 - (e3 ** 2).sum(1))
        net = mlp(torch.cat([mlp(emb, "dnn", 2), wide.sum(1, keepdim=True), fm], 1), "final", 1)
    pred = torch.sigmoid(lin(net, "last")).squeeze(1)
    p = pred.clamp(1e-7, 1 - 1e-7)
    ref_loss = -(labels * torch.log(p) + (1 - labels) * torch.log(1 - p)).mean()
    ref_loss.backward()

    dopt = torch.optim.SGD(model.parameters(), lr=lr)
    loss = mz.train_step(model, dense, ids, labels, dopt, dr.GradientDescentOptimizer(lr))
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=RTOL, atol=ATOL)
    for name, prm in model.named_parameters():
        want = ref_model[name] - lr * ref_model[name].grad
        torch.testing.assert_close(prm.detach(), want.detach(), rtol=RTOL, atol=ATOL)
    for t in range(T):
        want = W[t] - lr * W[t].grad
        torch.testing.assert_close(_ev_rows(evs[t], R), want.detach(), rtol=RTOL, atol=ATOL)
    for t in range(len(Ww)):
        want = Ww[t] - lr * Ww[t].grad
        torch.testing.assert_close(_ev_rows(model.wide_evs[t], R), want.detach(), rtol=RTOL,
                                   atol=ATOL)
