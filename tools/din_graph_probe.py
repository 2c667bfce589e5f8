"""The DIN training step (BASELINE configs[3] shape, tools/model_step.py din)
captured as hipGraphs, one per batch (the history length differs per batch):
two identical models from the same seeds, A stepped eagerly, B by graph
replays after the same warmup; losses, dense parameters and EV contents
compared bit for bit after every step, then both timed.

usage: python tools/din_graph_probe.py [--steps 20]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def build(dr, mz, dev, tag, B, T, D, R):
    if os.environ.get("GMP_BLAS"):   # graph_mem_probe bisection: rocblas / hipblaslt
        torch.backends.cuda.preferred_blas_library(os.environ["GMP_BLAS"])
    evs = []
    for i, r in enumerate(R):
        ev = dr.EmbeddingVariable("dgp_%s%d" % (tag, i), D, 0.0, capacity=r + (1 << 16), device=dev)
        ev.insert_synthetic(0, r, seed=700 + i)
        evs.append(ev)
    torch.manual_seed(11)
    model = mz.DIN(*evs).to(dev)
    # DGP_FOREACH=0: the per-parameter Adam (no multi-tensor address lists)
    fe = {"0": False, "1": True}.get(os.environ.get("DGP_FOREACH", ""), None)
    dopt = torch.optim.Adam(model.parameters(), lr=0.001, capturable=True, foreach=fe)
    eopt = dr.AdamOptimizer(0.001)
    skip = os.environ.get("DGP_SKIP", "")   # bisection: "ev" / "dense" updates left out
    if skip == "ev":
        def drop(var_list, global_step=None):
            for v in var_list:
                for sl in v.pending_grads:
                    getattr(sl, "indices", None)   # formed, then dropped
                v.pending_grads = []
        eopt.apply_gradients = drop
    elif skip == "dense":
        dopt.step = lambda *a, **k: None
    return evs, model, dopt, eopt


def batches_for(dev, B, T, R):
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    out = []
    for _ in range(4):
        lens = torch.randint(1, T + 1, (B,), generator=g, device=dev)
        Tb = int(lens.max())
        mask = (torch.arange(Tb, device=dev)[None, :] < lens[:, None]).float()
        mh = torch.randint(1, R[1], (B, Tb), generator=g, device=dev) * mask.long()
        ch = torch.randint(1, R[2], (B, Tb), generator=g, device=dev) * mask.long()
        lab = (torch.rand(B, generator=g, device=dev) > 0.5).long()
        out.append((torch.randint(0, R[0], (B,), generator=g, device=dev),
                    torch.randint(0, R[1], (B,), generator=g, device=dev),
                    torch.randint(0, R[2], (B,), generator=g, device=dev), mh, ch, mask,
                    torch.stack([lab, 1 - lab], 1).float()))
    return out


def snapshot(model, evs):
    ps = [p.detach().clone() for p in model.parameters()]
    es = []
    for ev in evs:
        k, v = ev.export()[:2]
        o = torch.argsort(k)
        es.append((k[o].clone(), v[o].clone()))
    return ps, es


def same(a, b, names=None, report=False):
    (pa, ea), (pb, eb) = a, b
    ok = True
    for n, (x, y) in enumerate(zip(pa, pb)):
        if not torch.equal(x.view(torch.int32), y.view(torch.int32)):
            ok = False
            if report:
                d = (x - y).abs()
                print("  param %s differs: %d elements, max |diff| %.3g (max |x| %.3g)"
                      % (names[n] if names else n, int((d > 0).sum()), float(d.max()),
                         float(x.abs().max())), flush=True)
    for t, ((ka, va), (kb, vb)) in enumerate(zip(ea, eb)):
        if not (torch.equal(ka, kb) and torch.equal(va.view(torch.int32), vb.view(torch.int32))):
            ok = False
            if report:
                if torch.equal(ka, kb):
                    d = (va - vb).abs()
                    print("  EV %d differs: %d rows, max |diff| %.3g" % (
                        t, int((d.amax(1) > 0).sum()), float(d.max())), flush=True)
                else:
                    print("  EV %d key sets differ (%d vs %d)" % (t, ka.numel(), kb.numel()),
                          flush=True)
    return ok


def one_model(dr, mz, dev, bat, B, T, D, R, steps, mode):
    """One model in this process: DGP_MODE=eager saves every step's loss and
    the final state to gpurun_out/dgp_eager.pt; DGP_MODE=graph replays the
    captured steps and compares with that file -- no second model's eager
    calls between the replays."""
    path = os.environ.get("DGP_FILE", os.path.join("/tmp", "dgp_eager_%d.pt" % B))
    evs, model, dopt, eopt = build(dr, mz, dev, "m", B, T, D, R)
    warm = 4
    for i in range(warm):
        mz.din_train_step(model, bat[i % 4], dopt, eopt, i)
    for ev in evs:
        ev.reserve(8 * B * (T + 1))
    torch.cuda.synchronize()
    losses = []
    if mode == "eager":
        for i in range(warm, warm + steps):
            losses.append(mz.din_train_step(model, bat[i % 4], dopt, eopt, i).detach().clone())
        torch.cuda.synchronize()
        ps, es = snapshot(model, evs)
        torch.save({"losses": [l.cpu() for l in losses], "ps": [p.cpu() for p in ps],
                    "es": [(k.cpu(), v.cpu()) for k, v in es]}, path)
        print("eager run saved (%d steps)" % steps, flush=True)
        return
    ref = torch.load(path, weights_only=True)
    graphs = []
    for j in range(4):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = mz.din_train_step(model, bat[(warm + j) % 4], dopt, eopt, warm + j)
        graphs.append((g, loss))
    ok = True
    for n, i in enumerate(range(warm, warm + steps)):
        g, lb = graphs[(i - warm) % 4]
        g.replay()
        torch.cuda.synchronize()
        same_l = torch.equal(ref["losses"][n].view(torch.int32), lb.detach().cpu().view(torch.int32))
        if not same_l:
            print("step %d loss differs: %r vs %r" % (i, float(ref["losses"][n]),
                                                       float(lb.detach())), flush=True)
            ok = False
            break
    if ok:
        ps, es = snapshot(model, evs)
        ok = all(torch.equal(a.view(torch.int32), b.cpu().view(torch.int32))
                 for a, b in zip(ref["ps"], ps))
        for (ka, va), (kb, vb) in zip(ref["es"], es):
            ok = ok and torch.equal(ka, kb.cpu()) and torch.equal(va.view(torch.int32),
                                                                    vb.cpu().view(torch.int32))
    print("graph replays (alone in their process) == eager run: %s over %d steps" % (ok, steps),
          flush=True)
    if not ok:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    dev = torch.device("cuda:0")
    B, T, D = args.batch, 100, 18
    R = (500_000, 400_000, 2_000)
    bat = batches_for(dev, B, T, R)
    mode = os.environ.get("DGP_MODE", "")   # "eager" / "graph": one model per process
    if mode:
        return one_model(dr, mz, dev, bat, B, T, D, R, args.steps, mode)
    A = build(dr, mz, dev, "a", B, T, D, R)
    Bm = build(dr, mz, dev, "b", B, T, D, R)
    warm = 4   # every batch once: per-shape caches, slots, device beta powers
    for m in (A, Bm):
        evs, model, dopt, eopt = m
        for i in range(warm):
            mz.din_train_step(model, bat[i % 4], dopt, eopt, i)
    torch.cuda.synchronize()
    assert same(snapshot(A[1], A[0]), snapshot(Bm[1], Bm[0])), "warmup diverged"
    for ev in A[0]:   # the eager twin grows its tables the same way
        ev.reserve(8 * B * (T + 1))
    evs, model, dopt, eopt = Bm
    for ev in evs:   # a captured resolve must not be able to outgrow the table
        ev.reserve(8 * B * (T + 1))   # 4 graphs x (lookup + apply) adds, counted conservatively
    torch.cuda.synchronize()
    graphs = []
    shared = os.environ.get("DGP_SHARED_POOL", "0") == "1"
    pool = torch.cuda.graph_pool_handle() if shared else None
    # capture order (DGP_ORDER, e.g. "1,0,3,2"): graph k replays batch order[k]
    order = [int(x) for x in os.environ.get("DGP_ORDER", "0,1,2,3").split(",")]
    # DGP_ZERO_OUTSIDE=1: zero_grad(set_to_none) before each capture and a
    # no-op inside it (torch's documented whole-network pattern)
    zero_out = os.environ.get("DGP_ZERO_OUTSIDE", "0") == "1"
    real_zero = dopt.zero_grad
    if os.environ.get("DGP_CAPTURE_ONLY") == "1":
        # kernels that run while a capture is open ran eagerly, not into the
        # graph: a kernel trace of this window shows them (gaps mark it)
        torch.cuda.synchronize()
        time.sleep(0.3)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            mz.din_train_step(model, bat[order[0]], dopt, eopt, warm)
        torch.cuda.synchronize()
        time.sleep(0.3)
        print("captured one graph (capture-only mode)", flush=True)
        return
    for j in order:
        g = torch.cuda.CUDAGraph()
        if zero_out:
            real_zero(set_to_none=True)
            dopt.zero_grad = lambda *a, **k: None
        with torch.cuda.graph(g, pool=pool):
            loss = mz.din_train_step(model, bat[j], dopt, eopt, warm + j)
        dopt.zero_grad = real_zero
        graphs.append((g, loss))
    torch.cuda.synchronize()
    print("captured %d graphs, batch order %s, skip %r, powers %s" % (
        len(order), order, os.environ.get("DGP_SKIP", ""), list(eopt._pw.keys())), flush=True)
    equal = True
    def ptrs():
        out = [p.data_ptr() for p in model.parameters()]
        for st in dopt.state.values():
            out += [v.data_ptr() for v in st.values() if torch.is_tensor(v)]
        return out
    ptrs0 = ptrs()
    # replay sequence (DGP_REPLAY, indices into the captured graphs)
    rep = [int(x) for x in os.environ.get("DGP_REPLAY", ",".join(
        str(k) for k in range(len(order)))).split(",")]
    # DGP_SEQUENTIAL=1: the eager twin runs all its steps first (snapshots
    # kept), then the graphs replay -- no eager allocation between replays
    seq = os.environ.get("DGP_SEQUENTIAL", "0") == "1"
    pre = {}
    if os.environ.get("DGP_CHURN") == "1":
        # no eager step at all: only allocations filled with NaN, then freed
        for _ in range(8):
            junk = [torch.full((1 << 22,), float("nan"), device=dev) for _ in range(64)]
            del junk
        torch.cuda.synchronize()
        print("churned the default pool with NaN-filled blocks", flush=True)
    twin = os.environ.get("DGP_TWIN_OP", "")
    if twin:
        if twin == "none":
            twin = "-"
        # bisecting the interference: only part of a step on the twin model
        # A between capture and replay, then B's replays are checked for NaN
        for i in range(8):
            bt = bat[i % 4]
            if twin == "fwd":
                with torch.no_grad():
                    A[1](*bt[:6])
            elif twin == "fwdbwd":
                y = A[1](*bt[:6])
                (-(torch.log(y) * bt[6]).mean()).backward()
                for ev in A[0]:
                    ev.pending_grads = []
            elif twin == "lookup":
                with torch.no_grad():
                    A[1].item_lookup(torch.stack([bt[1], bt[2]]))
            elif twin == "apply":
                y = A[1](*bt[:6])
                (-(torch.log(y) * bt[6]).mean()).backward()
                A[3].apply_gradients(A[0], global_step=i)
            elif twin == "dense":
                y = A[1](*bt[:6])
                A[2].zero_grad(set_to_none=True)
                (-(torch.log(y) * bt[6]).mean()).backward()
                A[2].step()
                for ev in A[0]:
                    ev.pending_grads = []
        torch.cuda.synchronize()
        for k, (g, lb) in enumerate(graphs[:2]):
            g.replay()
            torch.cuda.synchronize()
            print("twin op %r then graph %d replay: loss %r" % (twin, k, float(lb.detach())),
                  flush=True)
        return
    if seq:
        for i in range(warm, warm + args.steps):
            k = rep[(i - warm) % len(rep)]
            la = mz.din_train_step(A[1], bat[order[k]], A[2], A[3], warm + order[k])
            pre[i] = (la.detach().clone(), snapshot(A[1], A[0]))
        torch.cuda.synchronize()
    for i in range(warm, warm + args.steps):
        k = rep[(i - warm) % len(rep)]
        if not seq:
            la = mz.din_train_step(A[1], bat[order[k]], A[2], A[3], warm + order[k])
        g, lb = graphs[k]
        print("step %d: graph %d (batch %d)" % (i, k, order[k]), flush=True)
        g.replay()
        torch.cuda.synchronize()
        if seq:
            la, snapA = pre[i]
            okl = torch.equal(la.view(torch.int32), lb.detach().view(torch.int32))
            names = [n for n, _ in model.named_parameters()]
            ok = same(snapA, snapshot(model, evs), names, report=True) and okl
            equal = equal and ok
            if not ok:
                print("step %d differs: loss %r vs %r" % (i, float(la), float(lb.detach())),
                      flush=True)
                break
            continue
        okl = torch.equal(la.view(torch.int32), lb.view(torch.int32))
        names = [n for n, _ in model.named_parameters()]
        ok = same(snapshot(A[1], A[0]), snapshot(model, evs), names, report=True) and okl
        equal = equal and ok
        if not ok:
            print("step %d differs: loss %r vs %r" % (i, float(la.detach()), float(lb.detach())),
                  flush=True)
            break
    print("eager == graph over %d steps: %s" % (args.steps, equal), flush=True)
    print("parameter / optimizer-state storage unchanged since capture: %s" % (ptrs() == ptrs0),
          flush=True)
    n = args.steps
    for name, fn in (("eager", lambda i: mz.din_train_step(A[1], bat[order[i % len(order)]],
                                                           A[2], A[3], i)),
                     ("graph", lambda i: graphs[i % len(order)][0].replay())):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        print(json.dumps({"din_step": name, "ms_per_step": round(ms, 3), "batch": B,
                          "samples_per_s": round(B / ms * 1e3, 1)}), flush=True)
    dr.status_check(dev)


if __name__ == "__main__":
    main()
