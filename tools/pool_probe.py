"""Pool-kernel probe: achieved GB/s of the one-hot grouped gather vs the
address span the rows are drawn from (TLB / locality sensitivity).

  python tools/pool_probe.py [--gb 128] [--iters 20]

Not part of the product or the tests; a measurement aid for DESIGN.md.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--tables", type=int, default=26)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--fill", action="store_true", help="write the pool before reading it")
    ap.add_argument("--split", type=int, default=1, help="separate allocations (table t -> t %% split)")
    ap.add_argument("--spans", default="12,16,18,20,22,24,26")
    args = ap.parse_args()
    from deeprec_amd import _lib, ops
    _lib.load()
    dev = torch.device("cuda", 0)
    D, B, T = args.dim, args.batch, args.tables
    rows = int(args.gb * 2**30) // (4 * D) // args.split
    pools = [torch.empty((rows, D), dtype=torch.float32, device=dev) for _ in range(args.split)]
    if args.fill:
        for p in pools:
            p.fill_(0.5)
    pool = pools[0]
    out = torch.empty((B, T * D), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    res = []
    spans = [1 << int(s) for s in args.spans.split(",") if s] + [rows]
    for span in spans:
        span = min(span, rows)
        for mode in ("random", "sequential", "slot-sequential", "random-runs8"):
            if mode != "random" and span != rows:
                continue
            sel = []
            for t in range(T):
                if mode == "random":
                    sel.append(torch.randint(0, span, (B,), generator=g, device=dev))
                elif mode == "sequential":      # table-major rows
                    sel.append(torch.arange(t * B, (t + 1) * B, device=dev) % rows)
                elif mode == "slot-sequential":  # row = output slot: a plain copy
                    sel.append((torch.arange(B, device=dev) * T + t) % rows)
                else:                            # random 4 KiB runs of 8 rows
                    base = torch.randint(0, span // 8, (B // 8 + 1,), generator=g, device=dev)
                    r = (base[:, None] * 8 + torch.arange(8, device=dev)[None, :]).reshape(-1)
                    sel.append(r[:B] % rows)
            descs = []
            for t in range(T):
                d = _lib.DrPoolDesc()
                d.pool, d.pool_rows, d.ids = pools[t % args.split].data_ptr(), rows, sel[t].data_ptr()
                d.out, d.out_stride, d.combiner, d.max_norm = out.data_ptr() + 4 * t * D, T * D, 0, -1.0
                descs.append(d)
            ops.pool_grouped(descs, B, D, onehot=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                ops.pool_grouped(descs, B, D, onehot=True)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            byts = T * B * (8 + 2 * 4 * D)
            r = {"span_rows": span, "span_gb": round(span * 4 * D / 2**30, 3), "mode": mode,
                 "us": round(ms * 1e3, 1), "GBps": round(byts / ms / 1e6, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    # stream references on the same box: copy (R+W), fill (W), sum (R)
    def timed(fn, nbytes, name):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / args.iters
        print(json.dumps({"ref": name, "us": round(ms * 1e3, 1),
                          "GBps": round(nbytes / ms / 1e6, 1)}), flush=True)
    src = pool[: out.shape[0] * T].view(out.shape)
    timed(lambda: out.copy_(src), 2 * out.numel() * 4, "torch copy_ (read+write)")
    timed(lambda: out.fill_(1.0), out.numel() * 4, "torch fill_ (write)")
    timed(lambda: torch.sum(src), out.numel() * 4, "torch sum (read)")
    # torch's own gather for comparison (index_select on the full span)
    sel = torch.randint(0, rows, (T * B,), generator=g, device=dev)
    torch.index_select(pool, 0, sel)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        torch.index_select(pool, 0, sel)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps({"torch_index_select_full_span_us": round(ms * 1e3, 1),
                      "GBps": round(T * B * (8 + 8 * D) / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
