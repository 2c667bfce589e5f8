"""Full training step of a modelzoo model on the bench's table shape (N = 1):
DLRM (modelzoo/DLRM/train.py), DeepFM (modelzoo/DeepFM/train.py) or DCN-v2
(configs[4], 3 bf16 cross layers + deep MLP) forward,
BCE loss, backward, dense SGD, KV SGD / Adagrad on every EV; or DIN
(modelzoo/DIN, BASELINE configs[3]: uid / item / category EVs of dim 18,
history lengths U[1, maxlen], Adam as in the reference).  Prints one JSON
line with samples/s and the per-phase split.  A measurement aid for
SURVEY 8f #4; bench.py's headline metric is the forward lookup.

  python tools/model_step.py [--model dlrm|deepfm|din|dcn|wdl] [--rows 12500000] [--dim 128]
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
    ap.add_argument("--model", default="dlrm", choices=["dlrm", "deepfm", "din", "dcn", "wdl"])
    ap.add_argument("--maxlen", type=int, default=100, help="DIN history length bound")
    ap.add_argument("--tables", type=int, default=26)
    ap.add_argument("--rows", type=int, default=12_500_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--batch", type=int, default=None, help="65536 (DIN: 4096)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--opt", default="sgd", choices=["sgd", "adagrad"])
    ap.add_argument("--bf16", action="store_true", help="MLPs in bf16 (the reference's --bf16)")
    args = ap.parse_args()
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    dev = torch.device("cuda", 0)
    if args.model == "din":
        args.batch = args.batch or 4096
        return din(args, dr, mz, dev)
    if args.model == "wdl":
        args.batch = args.batch or 65536
        return wdl(args, dr, mz, dev)
    args.batch = args.batch or 65536
    T, D, B, R = args.tables, args.dim, args.batch, args.rows
    t0 = time.perf_counter()
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("ms%d" % t, D, 0.0, capacity=R + (1 << 19), device=dev)
        ev.insert_synthetic(0, R, seed=1000 + t)
        evs.append(ev)
    if args.model == "dlrm":
        model = mz.DLRM(evs, 13, (512, 256), (512, 256), bf16=args.bf16).to(dev)
    elif args.model == "dcn":     # BASELINE configs[4]: bf16 CrossNet on MFMA, 3 layers
        model = mz.DCNv2(evs, 13, layers=3, deep=(1024, 512), bf16=args.bf16).to(dev)
    else:
        wide = []
        for t in range(T):
            ev = dr.EmbeddingVariable("msw%d" % t, 1, 0.0, capacity=R + (1 << 19), device=dev)
            ev.insert_synthetic(0, R, seed=5000 + t)
            wide.append(ev)
        model = mz.DeepFM(evs, wide, bf16=args.bf16).to(dev)
    torch.cuda.synchronize()
    print("[model_step] tables ready in %.1fs" % (time.perf_counter() - t0), file=sys.stderr,
          flush=True)
    dopt = torch.optim.SGD(model.parameters(), lr=0.01)
    eopt = dr.GradientDescentOptimizer(0.01) if args.opt == "sgd" else dr.AdagradOptimizer(0.01)
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    batches = [(torch.randn(B, 13, generator=g, device=dev),
                torch.randint(0, R, (T, B), generator=g, device=dev),
                (torch.rand(B, generator=g, device=dev) > 0.5).float()) for _ in range(4)]
    for i in range(args.warmup):
        mz.train_step(model, *batches[i % 4][:2], batches[i % 4][2], dopt, eopt, i)
    torch.cuda.synchronize()
    print("[model_step] warmup ok", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = mz.train_step(model, *batches[i % 4][:2], batches[i % 4][2], dopt, eopt, i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dr.status_check(dev)
    print(json.dumps({"model": args.model, "samples_per_s": round(B * args.steps / el, 1),
                      "lookups_per_s": round(T * B * args.steps / el, 1),
                      "ms_per_step": round(el / args.steps * 1e3, 3), "batch": B, "tables": T,
                      "rows": R, "dim": D, "opt": args.opt, "bf16_mlp": args.bf16, "loss": float(loss)}), flush=True)


# modelzoo/WDL/train.py:23-81: per-column hash buckets and embedding dims
WDL_BUCKETS = [2500, 2000, 300000, 250000, 1000, 100, 20000, 4000, 20, 100000, 10000, 250000,
               40000, 100, 100, 200000, 50, 10000, 4000, 20, 250000, 100, 100, 250000, 400, 100000]
WDL_DIMS = [64, 64, 128, 128, 64, 64, 64, 64, 64, 128, 64, 128, 64, 64, 64, 128, 64, 64, 64, 64,
            128, 64, 64, 128, 64, 128]


def wdl(args, dr, mz, dev):
    """WDL step (configs[0]'s model, here on the GPU): 26 categorical columns
    with the reference's bucket sizes and dims, 13 numeric columns, dnn
    [1024, 512, 256]; Adagrad 0.01 (deep) and FTRL 0.2 (linear) as
    modelzoo/WDL/train.py:302-335."""
    B = args.batch
    cats = ["C%d" % (i + 1) for i in range(26)]
    nums = ["I%d" % (i + 1) for i in range(13)]
    deep, wide = [], []
    for i, (r, d) in enumerate(zip(WDL_BUCKETS, WDL_DIMS)):
        ev = dr.EmbeddingVariable("wdl_d%d" % i, d, 0.0, capacity=r + (1 << 16), device=dev)
        ev.insert_synthetic(0, r, seed=900 + i)
        deep.append(ev)
        ew = dr.EmbeddingVariable("wdl_w%d" % i, 1, 0.0, capacity=r + (1 << 16), device=dev)
        ew.insert_synthetic(0, r, seed=950 + i)
        wide.append(ew)
    model = mz.WDL(cats, deep, wide, nums, bf16=args.bf16).to(dev)
    deep_opt = torch.optim.Adagrad(model.deep_parameters(), lr=0.01,
                                   initial_accumulator_value=0.1)
    ftrl = dr.FtrlOptimizer(0.2)
    adagrad = dr.AdagradOptimizer(0.01)
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    bk = torch.tensor(WDL_BUCKETS, device=dev)[:, None]
    batches = [(torch.rand(B, 13, generator=g, device=dev),
                (torch.rand(26, B, generator=g, device=dev) * bk).to(torch.int64),
                (torch.rand(B, generator=g, device=dev) > 0.5).float()) for _ in range(4)]
    for i in range(args.warmup):
        mz.wdl_train_step(model, *batches[i % 4], deep_opt, adagrad, ftrl, ftrl, i)
    torch.cuda.synchronize()
    print("[model_step] warmup ok", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = mz.wdl_train_step(model, *batches[i % 4], deep_opt, adagrad, ftrl, ftrl, i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dr.status_check(dev)
    print(json.dumps({"model": "wdl", "samples_per_s": round(B * args.steps / el, 1),
                      "lookups_per_s": round(52 * B * args.steps / el, 1),
                      "ms_per_step": round(el / args.steps * 1e3, 3), "batch": B,
                      "opt": "adagrad+ftrl", "bf16_mlp": args.bf16,
                      "loss": float(loss.detach())}), flush=True)


def din(args, dr, mz, dev):
    """DIN step: B samples, history lengths U[1, maxlen] padded to the batch
    max (prepare_data, modelzoo/DIN/train.py:24-88), vocab 5e5 users / 4e5
    items / 2e3 categories, dim 18, Adam."""
    B, T, D = args.batch, args.maxlen, 18
    R = (500_000, 400_000, 2_000)
    evs = []
    for i, r in enumerate(R):
        ev = dr.EmbeddingVariable("din%d" % i, D, 0.0, capacity=r + (1 << 16), device=dev)
        ev.insert_synthetic(0, r, seed=700 + i)
        evs.append(ev)
    model = mz.DIN(*evs).to(dev)
    dopt = torch.optim.Adam(model.parameters(), lr=0.001)
    eopt = dr.AdamOptimizer(0.001)
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    batches = []
    for _ in range(4):
        lens = torch.randint(1, T + 1, (B,), generator=g, device=dev)
        Tb = int(lens.max())
        mask = (torch.arange(Tb, device=dev)[None, :] < lens[:, None]).float()
        mh = torch.randint(1, R[1], (B, Tb), generator=g, device=dev) * mask.long()
        ch = torch.randint(1, R[2], (B, Tb), generator=g, device=dev) * mask.long()
        lab = (torch.rand(B, generator=g, device=dev) > 0.5).long()
        batches.append((torch.randint(0, R[0], (B,), generator=g, device=dev),
                        torch.randint(0, R[1], (B,), generator=g, device=dev),
                        torch.randint(0, R[2], (B,), generator=g, device=dev), mh, ch, mask,
                        torch.stack([lab, 1 - lab], 1).float()))
    for i in range(args.warmup):
        mz.din_train_step(model, batches[i % 4], dopt, eopt, i)
    torch.cuda.synchronize()
    print("[model_step] warmup ok", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = mz.din_train_step(model, batches[i % 4], dopt, eopt, i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dr.status_check(dev)
    nnz = sum(int(b[5].numel()) * 2 + 3 * B for b in batches) / 4
    print(json.dumps({"model": "din", "samples_per_s": round(B * args.steps / el, 1),
                      "lookups_per_s": round(nnz * args.steps / el, 1),
                      "ms_per_step": round(el / args.steps * 1e3, 3), "batch": B, "maxlen": T,
                      "dim": D, "vocab": R, "opt": "adam", "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
