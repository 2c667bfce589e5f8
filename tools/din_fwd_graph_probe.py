"""Bisecting tools/din_graph_probe.py's divergence: pieces of the DIN
forward captured twice as hipGraphs over the same batch, each replay
compared with the eager result (no parameter changes in between)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    from din_graph_probe import batches_for, build
    dr.load()
    dev = torch.device("cuda:0")
    B, T, D = 4096, 100, 18
    R = (500_000, 400_000, 2_000)
    bat = batches_for(dev, B, T, R)
    evs, model, dopt, eopt = build(dr, mz, dev, "f", B, T, D, R)
    for ev in evs:
        ev.reserve(8 * B * (T + 1))
    uids, mids, cats, mid_his, cat_his, mask, target = bat[0]
    Tb = mid_his.shape[1]

    def lookups():
        ids = torch.stack([torch.cat([mids, mid_his.reshape(-1)]),
                           torch.cat([cats, cat_his.reshape(-1)])])
        allv = model.item_lookup(ids)
        return allv[:B], allv[B:].view(B, Tb, -1)

    def attention():
        item_eb, facts = lookups()
        return mz.DinAttentionFused.apply(item_eb, facts, mask, model.f1_att.weight,
                                          model.f1_att.bias, model.f2_att.weight,
                                          model.f2_att.bias, model.f3_att.weight,
                                          model.f3_att.bias)

    def full():
        return (model(uids, mids, cats, mid_his, cat_his, mask),)

    def loss_bwd():
        y = model(uids, mids, cats, mid_his, cat_his, mask)
        loss = -(torch.log(y) * target).mean()
        dopt.zero_grad(set_to_none=True)
        loss.backward()
        for ev in evs:
            ev.pending_grads = []
        return (loss,) + tuple(p.grad for p in model.parameters())

    sgd = torch.optim.SGD(model.parameters(), lr=0.01)

    def with_opt(opt):
        def f():
            out = loss_bwd()
            opt.step()
            return out
        return f

    pieces = (("lookups", lookups), ("attention", attention), ("forward", full),
              ("forward+backward", loss_bwd), ("+ dense SGD", with_opt(sgd)),
              ("+ dense Adam", with_opt(dopt)))
    only = os.environ.get("DFP_ONLY")
    for name, fn in pieces:
        if only and name not in only.split(","):
            continue
        for _ in range(2):
            fn()
        for ev in evs:
            ev.pending_grads = []
        torch.cuda.synchronize()
        want = [t.detach().clone() for t in fn()]
        for ev in evs:
            ev.pending_grads = []
        graphs, outs = [], []
        for k in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                o = fn()
            for ev in evs:
                ev.pending_grads = []
            graphs.append(g)
            outs.append(o)
        res = []
        for k in range(2):
            graphs[k].replay()
            torch.cuda.synchronize()
            res.append(all(torch.equal(a.detach(), b) for a, b in zip(outs[k], want)))
        # then the state moves (in place, eagerly) and the graphs replay again
        with torch.no_grad():
            for prm in model.parameters():
                prm.mul_(1.01)
            for ev in evs:
                k_, v_ = ev.export()[:2]
                ev.insert(k_, v_ * 1.01)
        for ev in evs:   # (insert counts as adds: headroom again for the next capture)
            ev.reserve(8 * B * (T + 1))
        torch.cuda.synchronize()
        want2 = [t.detach().clone() for t in fn()]
        for ev in evs:
            ev.pending_grads = []
        for k in range(2):
            graphs[k].replay()
            torch.cuda.synchronize()
            res.append(all(torch.equal(a.detach(), b) for a, b in zip(outs[k], want2)))
            if name == "forward+backward" and not res[-1]:
                names = ["loss"] + [n for n, _ in model.named_parameters()]
                bad = [names[i] for i, (a, b) in enumerate(zip(outs[k], want2))
                       if not torch.equal(a.detach(), b)]
                print("  replay %d after the change: differs in %s" % (k, bad[:8]), flush=True)
        print("%-18s graph replays equal eager (before / after a state change): %s"
              % (name, res), flush=True)
    dr.status_check(dev)


if __name__ == "__main__":
    main()
