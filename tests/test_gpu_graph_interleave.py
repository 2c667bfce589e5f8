"""hipGraph replays interleaved with another model's eager steps, in ONE
process -- round 5's failure (profiles/r05_din_graph_probe.log: a twin
model's eager steps between the replays made them diverge or go NaN).

The cause is the ROCm runtime's graph packet capture, not engine state: a
graph of two plain torch sums, replayed after other allocations and kernels
ran in the process, changes value from its second replay on unless
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 is in the environment when HIP initialises
(tools/torch_graph_churn_probe.py, profiles/r06_graph_replay_bisect.log).
deeprec_amd sets it on import (and tests/conftest.py before any test touches
the GPU); these tests hold the workaround and the models to it:

* the plain-torch reproducer stays constant over replays with churn between;
* DIN at BASELINE configs[3]'s shape (B = 4096, histories U[1, 100], dim 18,
  Adam dense + KV): model A eager, model B as four captured steps, each
  replay preceded by A's eager step of the same batch, two rounds -- losses,
  parameters and every EV row bit-equal;
* DLRM (bf16 MFMA towers, dot interaction, SGD dense + KV) the same way.
Reference callers: modelzoo/DIN/script/model.py:61-150, modelzoo/DLRM/train.py."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _bits_equal(a, b):
    return torch.equal(a.view(torch.int32), b.view(torch.int32))


def _state(model, evs):
    ps = [p.detach().clone() for p in model.parameters()]
    es = []
    for ev in evs:
        k, v = ev.export()[:2]
        o = torch.argsort(k)
        es.append((k[o], v[o]))
    return ps, es


def _assert_same_state(a, b):
    (pa, ea), (pb, eb) = a, b
    for n, (x, y) in enumerate(zip(pa, pb)):
        assert _bits_equal(x, y), "parameter %d differs" % n
    for t, ((ka, va), (kb, vb)) in enumerate(zip(ea, eb)):
        assert torch.equal(ka, kb), "EV %d key sets differ" % t
        assert _bits_equal(va, vb), "EV %d rows differ" % t


def _churn(dev, seed):
    g = torch.Generator().manual_seed(seed)
    junk = [torch.full((int(s),), float("nan"), device=dev)
            for s in torch.randint(1, 1 << 18, (3000,), generator=g).tolist()]
    del junk


def test_runtime_flag_set_before_hip_init():
    from deeprec_amd import _lib
    assert os.environ.get(_lib.GRAPH_PACKET_CAPTURE_ENV) == "0"


def test_plain_torch_graph_stable_under_churn():
    dev = DEV
    g0 = torch.Generator(device=dev).manual_seed(3)
    a = torch.randn(4096, 36, generator=g0, device=dev)
    b = torch.randn(4096, 100, 36, generator=g0, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            a.sum() + b.sum()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = a.sum() + b.sum()
    vals = []
    for r in range(4):
        _churn(dev, r)
        g.replay()
        torch.cuda.synchronize()
        vals.append(float(out))
    assert len(set(vals)) == 1, vals
    assert vals[0] == pytest.approx(float(a.sum() + b.sum()), rel=1e-5)


def _din_models(dr, mz, B, T, D, R):
    out = []
    for tag in "ab":
        evs = []
        for i, r in enumerate(R):
            ev = dr.EmbeddingVariable("gi_%s%d" % (tag, i), D, 0.0, capacity=r + (1 << 16),
                                      device=DEV)
            ev.insert_synthetic(0, r, seed=700 + i)
            evs.append(ev)
        torch.manual_seed(11)
        model = mz.DIN(*evs).to(DEV)
        out.append((evs, model, torch.optim.Adam(model.parameters(), lr=0.001, capturable=True),
                    dr.AdamOptimizer(0.001)))
    return out


def _din_batches(B, T, R):
    g = torch.Generator(device=DEV)
    g.manual_seed(2021)
    out = []
    for _ in range(4):
        lens = torch.randint(1, T + 1, (B,), generator=g, device=DEV)
        Tb = int(lens.max())
        mask = (torch.arange(Tb, device=DEV)[None, :] < lens[:, None]).float()
        mh = torch.randint(1, R[1], (B, Tb), generator=g, device=DEV) * mask.long()
        ch = torch.randint(1, R[2], (B, Tb), generator=g, device=DEV) * mask.long()
        lab = (torch.rand(B, generator=g, device=DEV) > 0.5).long()
        out.append((torch.randint(0, R[0], (B,), generator=g, device=DEV),
                    torch.randint(0, R[1], (B,), generator=g, device=DEV),
                    torch.randint(0, R[2], (B,), generator=g, device=DEV), mh, ch, mask,
                    torch.stack([lab, 1 - lab], 1).float()))
    return out


def test_din_graph_replays_interleaved_with_eager_model():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    B, T, D = 4096, 100, 18
    R = (500_000, 400_000, 2_000)
    bat = _din_batches(B, T, R)
    A, Bm = _din_models(dr, mz, B, T, D, R)
    for i in range(4):
        for m in (A, Bm):
            mz.din_train_step(m[1], bat[i], m[2], m[3], i)
    torch.cuda.synchronize()
    _assert_same_state(_state(A[1], A[0]), _state(Bm[1], Bm[0]))
    for m in (A, Bm):
        for ev in m[0]:
            ev.reserve(8 * B * (T + 1))
    torch.cuda.synchronize()
    graphs, losses = [], []
    for j in range(4):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            losses.append(mz.din_train_step(Bm[1], bat[j], Bm[2], Bm[3], 4 + j))
        graphs.append(g)
    for r in range(2):
        for j in range(4):
            la = mz.din_train_step(A[1], bat[j], A[2], A[3], 4 + j).detach()
            graphs[j].replay()
            torch.cuda.synchronize()
            assert _bits_equal(la, losses[j].detach()), (r, j, float(la), float(losses[j]))
    _assert_same_state(_state(A[1], A[0]), _state(Bm[1], Bm[0]))
    dr.status_check(DEV)


def test_dlrm_graph_replays_interleaved_with_eager_model():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    T, D, B, R, NB = 26, 128, 8192, 60_000, 2
    models = []
    for tag in "ab":
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("gid_%s%d" % (tag, t), D, 0.0, capacity=R + 4 * B,
                                      device=DEV)
            ev.insert_synthetic(0, R, seed=1000 + t)
            evs.append(ev)
        torch.manual_seed(0)
        model = mz.DLRM(evs, 13, bf16=True).to(DEV)
        models.append((evs, model, torch.optim.SGD(model.parameters(), lr=0.01),
                       dr.GradientDescentOptimizer(0.01)))
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    ids = [torch.randint(0, R + 1000, (T, B), generator=g, device=DEV) for _ in range(NB)]
    dense = [torch.randn((B, 13), generator=g, device=DEV) for _ in range(NB)]
    lab = [(torch.rand(B, generator=g, device=DEV) > 0.5).float() for _ in range(NB)]

    def step(m, k):
        return mz.train_step(m[1], dense[k], ids[k], lab[k], m[2], m[3])
    for i in range(2):
        for m in models:
            step(m, i % NB)
    torch.cuda.synchronize()
    A, Bm = models
    _assert_same_state(_state(A[1], A[0]), _state(Bm[1], Bm[0]))
    for ev in Bm[0] + A[0]:
        ev.reserve(4 * NB * B)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gl = [step(Bm, k) for k in range(NB)]
    for r in range(2):
        la = [step(A, k).detach() for k in range(NB)]
        graph.replay()
        torch.cuda.synchronize()
        for k in range(NB):
            assert _bits_equal(la[k], gl[k].detach()), (r, k, float(la[k]), float(gl[k]))
    _assert_same_state(_state(A[1], A[0]), _state(Bm[1], Bm[0]))
    dr.status_check(DEV)


def test_adam_device_powers_prepare_and_sync():
    """KV Adam's beta powers: prepare() creates the device copy eagerly (a
    capture may then hold the first EV apply), _finish advances host and
    device copies with the same fp32 roundings, and sync_host_powers() --
    what a caller runs after graph replays, which advance only the device
    copy -- reads them back unchanged."""
    import deeprec_amd as dr
    opt = dr.AdamOptimizer(0.001, beta1=0.9, beta2=0.999)
    opt.prepare(DEV)
    assert str(DEV) in opt._pw
    for _ in range(3):
        opt._finish()
    h1, h2 = opt.b1p, opt.b2p
    dev_pw = opt._pw[str(DEV)][0].tolist()
    assert dev_pw == [h1, h2]
    opt._pw[str(DEV)][0].mul_(opt._pw[str(DEV)][1])   # a replay's device-only advance
    opt.sync_host_powers()
    f32 = lambda x: torch.tensor(x, dtype=torch.float32)  # noqa: E731
    assert opt.b1p == (f32(h1) * f32(0.9)).item() and opt.b2p == (f32(h2) * f32(0.999)).item()
