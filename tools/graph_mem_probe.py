"""Round 6: which memory does a captured DIN step read that the caching
allocator already counts as free?  (The round-5 symptom: a second model's
eager steps between the captures and the replays change the replays'
losses -- profiles/r05_din_graph_probe.log.)

One model per process (B = --batch), the eager reference from
tools/din_graph_probe.py DGP_MODE=eager (same DGP_FILE).  Here:
  * the allocator's history is recorded over the four captures; every
    block of the default pool (not a graph pool) that is freed INSIDE a
    capture window but was allocated before it is listed with the Python
    frames of its allocation and its free -- a tensor a captured kernel may
    still read after its memory went back to the pool;
  * GMP_POISON=default: before every replay, every inactive block of the
    default pool is zero-filled (hipMemsetAsync on the raw address, memory
    the allocator still holds); =graph: the graph pools' inactive blocks
    too; =none: nothing.
  * GMP_CHURN=small: before every replay, 3000 NaN-filled tensors of
    1 B - 1 MB are allocated and freed (what a second model's dense Adam
    does to the small pool); small0: the same zero-filled; large: 64
    NaN-filled tensors of 2 - 64 MB.  GMP_REPORT=1 lists the parameters,
    gradients, optimizer states and EV rows that are not finite after the
    first replays; GMP_BLAS picks torch's BLAS library (in the eager run
    too).
Each replay's loss is compared bit for bit with the eager run's.

usage: GMP_POISON=default python tools/graph_mem_probe.py --batch 4096 --steps 4"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import din_graph_probe as dgp  # noqa: E402


def _frames(fr, n=6):
    out = []
    for f in fr or []:
        fn = f.get("filename", "")
        if "deeprec" in fn or "tools/" in fn or "torch/optim" in fn or "autograd" in fn:
            out.append("%s:%s %s" % (os.path.basename(fn), f.get("line"), f.get("name")))
        if len(out) >= n:
            break
    return " <- ".join(out)


def _traces():
    snap = torch.cuda.memory._snapshot()
    return snap, snap["device_traces"][0]


def _poison(mode, dev):
    if mode == "none":
        return 0
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    st = torch.cuda.current_stream(dev).cuda_stream
    snap = torch.cuda.memory._snapshot()
    n = 0
    for seg in snap["segments"]:
        pool = tuple(seg.get("segment_pool_id", (0, 0)))
        if mode == "default" and pool != (0, 0):
            continue
        for b in seg["blocks"]:
            if b["state"] == "inactive":
                assert hip.hipMemsetAsync(C.c_void_p(b["address"]), 0, b["size"],
                                          C.c_void_p(st)) == 0
                n += b["size"]
    torch.cuda.synchronize()
    return n


def _churn(dev, seed, kind):
    g = torch.Generator().manual_seed(seed)
    if kind == "large":   # 2 - 64 MB blocks (the large pool)
        sizes = torch.randint(1 << 19, 1 << 24, (64,), generator=g).tolist()
    else:
        sizes = torch.randint(1, 1 << 18, (3000,), generator=g).tolist()
    val = 0.0 if kind == "small0" else float("nan")
    junk = [torch.full((s,), val, device=dev) for s in sizes]
    del junk
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    dev = torch.device("cuda:0")
    B, T, D = args.batch, 100, 18
    R = (500_000, 400_000, 2_000)
    bat = dgp.batches_for(dev, B, T, R)
    path = os.environ.get("DGP_FILE", os.path.join("/tmp", "dgp_eager_%d.pt" % B))
    ref = torch.load(path, weights_only=True)
    evs, model, dopt, eopt = dgp.build(dr, mz, dev, "m", B, T, D, R)
    warm = 4
    for i in range(warm):
        mz.din_train_step(model, bat[i % 4], dopt, eopt, i)
    for ev in evs:
        ev.reserve(8 * B * (T + 1))
    torch.cuda.synchronize()
    torch.cuda.memory._record_memory_history(max_entries=400000, stacks="python")
    if os.environ.get("GMP_NO_EMPTY_CACHE") == "1":
        # torch.cuda.graph's __enter__ empties the allocator cache (and the
        # BLAS workspaces) before every capture: not here
        torch.cuda.empty_cache = lambda: None
    graphs, windows = [], []
    for j in range(4):
        _, tr = _traces()
        w0 = len(tr)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = mz.din_train_step(model, bat[(warm + j) % 4], dopt, eopt, warm + j)
        _, tr = _traces()
        windows.append((w0, len(tr)))
        graphs.append((g, loss))
    snap, tr = _traces()
    torch.cuda.memory._record_memory_history(enabled=None)
    graph_segs = []
    for seg in snap["segments"]:
        if tuple(seg.get("segment_pool_id", (0, 0))) != (0, 0):
            graph_segs.append((seg["address"], seg["address"] + seg["total_size"]))

    def in_graph_pool(a):
        return any(lo <= a < hi for lo, hi in graph_segs)
    last_alloc = {}
    cands = []
    for k, e in enumerate(tr):
        act, a = e.get("action"), e.get("addr")
        if act == "alloc":
            last_alloc[a] = (k, e)
        elif act == "free_requested":
            for gi, (w0, w1) in enumerate(windows):
                if w0 <= k < w1:
                    al = last_alloc.get(a)
                    if al is not None and al[0] < w0 and not in_graph_pool(a):
                        cands.append((gi, a, e.get("size"), _frames(al[1].get("frames")),
                                      _frames(e.get("frames"))))
    print("default-pool blocks allocated before a capture and freed inside it: %d" % len(cands),
          flush=True)
    seen = set()
    for gi, a, sz, fa, ff in cands:
        key = (fa, ff)
        if key in seen:
            continue
        seen.add(key)
        print("  capture %d: %d B at %#x\n    alloc: %s\n    free:  %s" % (gi, sz, a, fa, ff),
              flush=True)
    mode = os.environ.get("GMP_POISON", "none")
    churn = os.environ.get("GMP_CHURN", "")
    ok = True
    # GMP_REPLAY: the graph replayed at each step (default 0,1,2,3,...); the
    # eager reference is only comparable while it is the capture order
    seq = [int(x) for x in os.environ.get("GMP_REPLAY", "").split(",") if x]
    for n in range(args.steps):
        gi = seq[n % len(seq)] if seq else n % 4
        gph, lb = graphs[gi]
        nb = _poison(mode, dev)
        if churn:
            _churn(dev, n, churn)
        gph.replay()
        torch.cuda.synchronize()
        same = torch.equal(ref["losses"][n].view(torch.int32), lb.detach().cpu().view(torch.int32))
        print("replay %d (graph %d, poison %s %d B, churn %r): loss %r eager %r -> %s" % (
            n, gi, mode, nb, churn, float(lb.detach()), float(ref["losses"][n]),
            "equal" if same else "DIFFERS"), flush=True)
        ok = ok and same
        if os.environ.get("GMP_REPORT") == "1" and n < 2:
            bad = []
            for name, p in model.named_parameters():
                for tag, t in (("param", p), ("grad", p.grad)) + tuple(
                        (k, v) for k, v in dopt.state[p].items() if torch.is_tensor(v)):
                    if t is not None and t.is_floating_point() and not bool(torch.isfinite(t).all()):
                        bad.append("%s.%s" % (name, tag))
            for t_, ev in enumerate(evs):
                k, v = ev.export()[:2]
                nb = int((~torch.isfinite(v)).any(1).sum())
                if nb:
                    bad.append("ev%d: %d rows" % (t_, nb))
                for sn in ("Adam", "Adam_1"):
                    sk, sv = ev.slot(sn, 0.0).export()[:2]
                    nb = int((~torch.isfinite(sv)).any(1).sum())
                    if nb:
                        bad.append("ev%d.%s: %d rows" % (t_, sn, nb))
            print("  non-finite after replay %d: %s" % (n, bad or "none"), flush=True)
    print("graph_mem_probe: all replays equal eager: %s" % ok, flush=True)


if __name__ == "__main__":
    main()
