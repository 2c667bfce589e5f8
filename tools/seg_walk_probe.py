"""Time the row-grouped backward of DIN's padding-id run alone, per walk
mode: the real padding terms of one DIN step at configs[3] (tools/data/
din_pad_terms.npz, written by tools/din_term_probe.py DTP_SAVE: 4 050
segments, 1..99 identical rows each, D = 18, 203 800 positions) as one id's
run, 30 000 other positions on 5 000 ids beside it, the mid / cat pair as one
grouped lookup; each mode's result checked bit-equal to the plain walk.

usage: python tools/seg_walk_probe.py [--iters 20]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))

import torch  # noqa: E402

MODES = {"rounds": {"DR_GRAD_SEG_ROUNDS": "1", "DR_GRAD_SEG_SCAN": "4096"},
         "seg-rep_add": {"DR_GRAD_SEG_ROUNDS": "0", "DR_GRAD_SEG_SCAN": "4096"},
         "plain": {"DR_GRAD_SEG_ROUNDS": "0", "DR_GRAD_SEG_SCAN": "0"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--terms", default="din_pad_terms.npz",
                    help="tools/data file: din_pad_terms.npz (first step) or "
                         "din_pad_terms_s200.npz (after 200 Adam steps)")
    args = ap.parse_args()
    import deeprec_amd as dr
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(ROOT, "tools", "data", args.terms))
    terms, k = z["terms"].astype(np.float32), z["lens"].astype(np.int64)
    D = terms.shape[1]
    rng = np.random.default_rng(5)
    other = rng.integers(1, 5000, 30000).astype(np.int64)
    v = np.concatenate([np.zeros(int(k.sum()), np.int64), other])
    g = np.concatenate([np.repeat(terms, k, axis=0),
                        (rng.standard_normal((other.size, D)) * 1e-6).astype(np.float32)])
    B = v.size
    ind = torch.as_tensor(np.stack([np.arange(B), np.zeros(B, np.int64)], 1), device=dev)
    vt = torch.as_tensor(v, device=dev)
    gg = torch.as_tensor(np.concatenate([g, -g], 1), device=dev)   # both tables DIN-like
    ref = None
    for mode in args.modes.split(","):
        os.environ.update(MODES[mode])
        evs = [dr.EmbeddingVariable("swp_%s_%d" % (mode, f), D, 0.1, capacity=8192, device=dev)
               for f in range(2)]
        sts = [dr.SparseTensor(ind, vt, (B, 1)) for _ in range(2)]

        def once():
            out = dr.embedding_lookup_sparse_multi(evs, sts, combiner="sum")
            out.backward(gg)
            return [e.pending_grads.pop() for e in evs]
        sl = once()
        torch.cuda.synchronize()
        got = [s.values[:int(s.num_valid.item())].clone() for s in sl]
        if ref is None:
            ref = got
        same = all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(ref, got))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            once()
        e1.record()
        torch.cuda.synchronize()
        print("%-12s lookup+backward %.3f ms  bit-equal to first mode: %s"
              % (mode, e0.elapsed_time(e1) / args.iters, same), flush=True)
    dr.status_check(dev)


if __name__ == "__main__":
    main()
