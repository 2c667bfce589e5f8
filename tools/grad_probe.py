"""Grouped pooled-lookup backward (dr_pool_grad_grouped) under id skew:
all-distinct ids vs one hot id repeated over half the positions (a padded
DIN history), D = 18 and 128.  Prints one JSON line per case (HIP events
around the backward only).  A measurement aid for DESIGN.md §6.

  python tools/grad_probe.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def main():
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import SparseTensor
    dr.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for D in (18, 128):
        for hot in (0.0, 0.5):
            n = 409600
            evs = [dr.EmbeddingVariable("gp_%d_%d_%d" % (D, int(hot * 10), t), D, 0.1, device=dev,
                                        capacity=1 << 20) for t in range(2)]
            ids = torch.randint(1, 400000, (2, n), generator=g, device=dev)
            if hot > 0:
                ids[:, :int(n * hot)] = 0
                ids = ids[:, torch.randperm(n, generator=g, device=dev)]
            ind = torch.stack([torch.arange(n, device=dev), torch.zeros(n, dtype=torch.int64,
                                                                          device=dev)], 1)
            sps = [SparseTensor(ind, ids[t].contiguous(), (n, 1)) for t in range(2)]
            G = torch.randn(n, 2 * D, generator=g, device=dev)
            times = []
            for it in range(6):
                out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                out.backward(G)
                b.record()
                b.synchronize()
                times.append(a.elapsed_time(b))
                for e in evs:
                    e.pending_grads = []
            ms = sorted(times[1:])[len(times[1:]) // 2]
            print(json.dumps({"dim": D, "positions": 2 * n, "hot_fraction": hot,
                              "backward_ms": round(ms, 3)}), flush=True)


if __name__ == "__main__":
    main()
