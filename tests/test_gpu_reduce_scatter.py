"""SOK-style owner-side pooling + reduce-scatter (ReduceScatterShardedLookup)
for multi-hot bags, with the HIP engine on one GPU.  World sizes 1-3 are
emulated in one process (a thread per rank, in-memory all-gather /
reduce-scatter in rank order); every rank holds only the EV rows of the keys
it owns (key % world).  Forward outputs and the EV gradients are compared
with a plain torch fp32 computation on the full tables.

Tolerance: fp32, rtol 1e-5 / atol 1e-6 -- the bag sum is associated per
owner and then across owners, not in the single-GPU order."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
T, D, B, K = 3, 16, 96, 1500


class _Comm(object):
    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.box = [None] * world

    def gather(self, rank, t):
        self.box[rank] = t
        self.bar.wait()
        out = torch.cat([self.box[r] for r in range(self.world)])
        self.bar.wait()
        return out

    def reduce_scatter(self, rank, t):
        self.box[rank] = t
        self.bar.wait()
        n = t.shape[0] // self.world
        out = self.box[0][rank * n:(rank + 1) * n].clone()
        for r in range(1, self.world):
            out += self.box[r][rank * n:(rank + 1) * n]
        self.bar.wait()
        return out


def _table(t):
    k = np.arange(K, dtype=np.float64)[:, None]
    return np.sin(0.011 * k + 0.9 * t + 0.07 * np.arange(D)[None, :]).astype(np.float32)


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("combiner", ["sum", "mean"])
def test_reduce_scatter_lookup_matches_torch(world, combiner):
    import deeprec_amd as dr
    from deeprec_amd.sharded import ReduceScatterShardedLookup
    dr.load()
    comm = _Comm(world)
    rng = np.random.default_rng(11 * world + len(combiner))
    engines, inputs = [], []
    for r in range(world):
        evs = []
        own = np.arange(r, K, world, dtype=np.int64)
        for t in range(T):
            ev = dr.EmbeddingVariable("rs%d_%s_%d_%d" % (world, combiner, r, t), D, 0.0,
                                      device=DEV)
            ev.insert(torch.as_tensor(own, device=DEV), torch.as_tensor(_table(t)[own], device=DEV))
            evs.append(ev)
        eng = ReduceScatterShardedLookup(evs, world, r, B, torch.device(DEV))
        eng._all_gather_fixed = (lambda rr: lambda x: comm.gather(rr, x))(r)
        eng._all_gather_var = (lambda rr: lambda x, sizes: comm.gather(rr, x))(r)
        eng._reduce_scatter = (lambda rr: lambda x: comm.reduce_scatter(rr, x))(r)
        engines.append(eng)
        ids, offs = [], []
        for t in range(T):
            lens = rng.integers(0, 7, B)
            lens[5] = 0
            v = rng.integers(0, K, int(lens.sum())).astype(np.int64)
            v[:3] = 7                                        # repeated ids
            ids.append(v)
            offs.append(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32))
        grad = rng.standard_normal((B, T * D)).astype(np.float32)
        inputs.append((ids, offs, grad))

    outs = [None] * world
    errs = []

    def run(r):
        try:
            ids, offs, _ = inputs[r]
            outs[r] = engines[r].forward([torch.as_tensor(x, device=DEV) for x in ids],
                                         [torch.as_tensor(o, device=DEV) for o in offs], combiner)
        except Exception as e:  # surface thread failures
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    if errs:
        raise errs[0]
    # backward: autograd runs on one device thread, so the ranks' backward
    # passes go one after another with the all-gathered gradient (rank
    # order) handed to each -- what the collective returns on every rank
    gathered = torch.cat([torch.as_tensor(inputs[r][2], device=DEV) for r in range(world)])
    for r in range(world):
        engines[r]._all_gather_fixed = lambda x: gathered
        outs[r].backward(torch.as_tensor(inputs[r][2], device=DEV))
        outs[r] = outs[r].detach()
    torch.cuda.synchronize()

    W = [torch.as_tensor(_table(t), device=DEV).requires_grad_(True) for t in range(T)]
    loss = 0
    for r in range(world):
        ids, offs, grad = inputs[r]
        cols = []
        for t in range(T):
            lens = torch.as_tensor(np.diff(offs[t]), device=DEV)
            seg = torch.repeat_interleave(torch.arange(B, device=DEV), lens)
            rows = W[t][torch.as_tensor(ids[t], device=DEV)]
            pooled = torch.zeros(B, D, device=DEV).index_add(0, seg, rows)
            if combiner == "mean":
                pooled = pooled / torch.clamp(lens, min=1)[:, None].float()
            cols.append(pooled)
        ref = torch.cat(cols, 1)
        torch.testing.assert_close(outs[r], ref.detach(), rtol=1e-5, atol=1e-6)
        loss = loss + (ref * torch.as_tensor(grad, device=DEV)).sum()
    loss.backward()
    for r in range(world):
        for t in range(T):
            dense = torch.zeros(K, D, device=DEV)
            for sl in engines[r].evs[t].pending_grads:
                n = sl.indices.numel() if sl.num_valid is None else int(sl.num_valid.item())
                dense.index_add_(0, sl.indices[:n].to(torch.int64), sl.values[:n])
            own = torch.arange(r, K, world, device=DEV)
            torch.testing.assert_close(dense[own], W[t].grad[own], rtol=1e-5, atol=1e-6)
            assert float(dense[torch.arange(K, device=DEV) % world != r].abs().sum()) == 0.0
