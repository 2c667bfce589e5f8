"""Training-step probe (N = 1): forward (grouped Unique -> EV resolve -> pool),
backward (pooled grad -> per-unique-key grads, dr_pool_grad) and the KV SGD /
Adagrad apply, on the bench's table shape.  Prints one JSON line.

  python tools/train_probe.py [--rows 12500000] [--opt sgd|adagrad] [--steps 10]

A measurement aid (profiles/ and DESIGN.md); bench.py's headline metric is
the forward lookup.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=26)
    ap.add_argument("--rows", type=int, default=12_500_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--opt", default="sgd", choices=["sgd", "adagrad", "adam", "ftrl"])
    ap.add_argument("--graph", action="store_true",
                    help="replay the steps as one captured hipGraph (no host launch gaps)")
    ap.add_argument("--bf16", action="store_true", help="bf16 EV value rows (fp32 slots)")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="Zipf(a) keys (numpy's zipf, mod rows); 0 = uniform")
    args = ap.parse_args()
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import SparseTensor
    dr.load()
    dev = torch.device("cuda", 0)
    T, D, B, R = args.tables, args.dim, args.batch, args.rows
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("tr%d" % t, D, 0.0, capacity=R + (1 << 20), device=dev,
                                  value_dtype=torch.bfloat16 if args.bf16 else torch.float32)
        ev.insert_synthetic(0, R, seed=1000 + t)
        evs.append(ev)
    opt = {"sgd": lambda: dr.GradientDescentOptimizer(0.01),
           "adagrad": lambda: dr.AdagradOptimizer(0.01),
           "adam": lambda: dr.AdamOptimizer(0.001),
           "ftrl": lambda: dr.FtrlOptimizer(0.01)}[args.opt]()
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    if args.zipf > 0:
        import numpy as np
        batches = [torch.as_tensor((np.random.default_rng(77 + i).zipf(args.zipf, size=(T, B)) - 1)
                                   % R, device=dev) for i in range(4)]
    else:
        batches = [torch.randint(0, R, (T, B), generator=g, device=dev) for _ in range(4)]
    hottest = int(max(torch.unique(b[0], return_counts=True)[1].max() for b in batches))
    ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev)], 1)
    upstream = torch.randn((B, T * D), generator=g, device=dev)

    def step(i):
        ids = batches[i % len(batches)]
        sps = [SparseTensor(ind, ids[t], (B, 1)) for t in range(T)]
        out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
        out.backward(upstream)
        opt.apply_gradients(evs)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    graph = None
    if args.graph:
        # the 4 batches' steps in a row, one graph (every kernel of every
        # step is in it; only the host's launch work disappears)
        for ev in evs:   # worst-case adds of the captured steps (resolve + apply)
            ev.reserve(2 * len(batches) * B)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for i in range(len(batches)):
                step(i)
        graph.replay()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        for i in range(0, args.steps, len(batches)):
            graph.replay()
        args.steps = (args.steps + len(batches) - 1) // len(batches) * len(batches)
    else:
        for i in range(args.steps):
            step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dr.status_check(dev)
    ms = el / args.steps * 1e3
    print(json.dumps({"probe": "train_step", "opt": args.opt, "graph": bool(args.graph),
                      "bf16": bool(args.bf16), "tables": T, "rows": R, "dim": D,
                      "zipf": args.zipf, "hottest_run_table0": hottest,
                      "batch": B, "ms_per_step": round(ms, 3),
                      "lookups_per_s": round(T * B / (ms * 1e-3), 1),
                      "samples_per_s": round(B / (ms * 1e-3), 1)}), flush=True)


if __name__ == "__main__":
    main()
