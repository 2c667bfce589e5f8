"""Per-op roofline table for every SURVEY §8(d) kernel kind (N = 1).

Each op of the C ABI is timed on torch's current stream (the stream the
library launches on) with HIP events over `--iters` calls after a warm-up,
and its ALGORITHMIC bytes (SURVEY §8(d) formulas, restated per line below) or
flops are divided by the average call time.  One JSON line per op.  Shapes
are BASELINE.json's configs: Cfg2 (26 x 1e7 x 64), Cfg3 per GPU
(12.5 M x 128, 26 x 65 536 lookups), DIN-like multi-hot bags, DCN-v2 d=3341.

  python tools/kernel_roofline.py [--iters 20] [--only name,name]

A measurement aid for DESIGN.md / profiles/, not part of the product.
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md
BF16_DENSE_TFLOPS = 2500.0  # dense (no 2:1 sparsity)


def timed(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def report(name, ms, nbytes=None, flops=None, shape=""):
    line = {"op": name, "shape": shape, "us": round(ms * 1e3, 1)}
    if nbytes is not None:
        gbs = nbytes / ms / 1e6
        line.update({"bytes": int(nbytes), "GBps": round(gbs, 1),
                     "frac_hbm": round(gbs / HBM_PEAK_GBS, 3)})
    if flops is not None:
        tf = flops / ms / 1e9
        line.update({"flops": int(flops), "TFLOPs": round(tf, 1),
                     "frac_mfma_bf16": round(tf / BF16_DENSE_TFLOPS, 3)})
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    only = set(s for s in args.only.split(",") if s)
    import deeprec_amd as dr
    from deeprec_amd import ops
    from deeprec_amd._lib import check, lib, ptr, stream_handle
    dr.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    it = args.iters
    N = 26 * 65536  # lookups per step per GPU (Cfg3)

    def want(name):
        return not only or name in only

    # -- dense ResourceGather: 8 (id) + D*4 read + D*4 write per lookup --------
    for R, D in ((12_500_000, 128), (10_000_000, 64)):
        if not want("gather"):
            break
        table = torch.empty((R, D), device=dev)
        ops.fill_synthetic(table, 7)
        idx = torch.randint(0, R, (N,), generator=g, device=dev)
        ms = timed(lambda: ops.gather(table, idx), it)
        report("gather", ms, N * (8 + 2 * D * 4), shape="table %dx%d, %d ids" % (R, D, N))
        del table

    # -- KvResourceGather: + 16 B slot read per lookup (all keys present) ------
    for R, D in ((12_500_000, 128), (10_000_000, 64)):
        if not want("ev_gather"):
            break
        ev = dr.EmbeddingVariable("rl_ev%d" % D, D, 0.0, capacity=R + (1 << 19), device=dev)
        ev.insert_synthetic(0, R, seed=11)
        keys = torch.randint(0, R, (N,), generator=g, device=dev)
        ms = timed(lambda: ev.sparse_read(keys), it)
        report("ev_gather", ms, N * (8 + 16 + 2 * D * 4),
               shape="EV %d keys x %d, %d ids (resolve + copy)" % (R, D, N))
        # resolve alone: 8 (key) + 16 (slot) + 8 (row out)
        ms = timed(lambda: ev.resolve(keys), it)
        report("ev_resolve", ms, N * (8 + 16 + 8), shape="EV %d keys, %d ids" % (R, N))
        del ev

    # -- SparseSegmentSum over multi-hot bags (DIN-like, len ~ U[1,40]) --------
    if want("segment_sum") or want("segment_grad"):
        B, R = 65536, 10_000_000
        for D in (64, 128):
            lens = torch.randint(1, 41, (B,), generator=g, device=dev)
            seg = torch.repeat_interleave(torch.arange(B, device=dev), lens).to(torch.int32)
            nnz = seg.numel()
            data = torch.empty((R, D), device=dev)
            ops.fill_synthetic(data, 3)
            idx = torch.randint(0, R, (nnz,), generator=g, device=dev).to(torch.int32)
            if want("segment_sum"):
                ms = timed(lambda: ops.sparse_segment_sum(data, idx, seg, B), it)
                report("sparse_segment_sum", ms, nnz * (4 + 4 + D * 4) + B * D * 4,
                       shape="B %d, nnz %d, D %d" % (B, nnz, D))
                ms = timed(lambda: ops.sparse_segment_mean(data, idx, seg, B), it)
                report("sparse_segment_mean", ms, nnz * (4 + 4 + D * 4) + B * D * 4,
                       shape="B %d, nnz %d, D %d" % (B, nnz, D))
            if want("segment_grad"):
                # grad w.r.t. U = nnz distinct-ish rows: idx in [0, U)
                U = nnz
                gidx = torch.randperm(U, generator=g, device=dev).to(torch.int32)
                top = torch.randn((B, D), generator=g, device=dev)
                ms = timed(lambda: ops.sparse_segment_sum_grad(top, gidx, seg, U), it)
                report("sparse_segment_sum_grad", ms, nnz * (4 + 4 + D * 4) + U * D * 4,
                       shape="B %d, nnz %d, U %d, D %d" % (B, nnz, U, D))
            del data

    # -- UnsortedSegmentSum: nnz*(4 + D*4) + U*D*4 ------------------------------
    if want("unsorted_segment_sum"):
        D, n, U = 128, N, 1 << 20
        data = torch.randn((n, D), generator=g, device=dev)
        seg = torch.randint(0, U, (n,), generator=g, device=dev).to(torch.int32)
        ms = timed(lambda: ops.unsorted_segment_sum(data, seg, U), it)
        report("unsorted_segment_sum", ms, n * (4 + D * 4) + U * D * 4,
               shape="nnz %d, U %d, D %d" % (n, U, D))

    # -- radix sort pairs: per 8-bit pass 8n (hist read) + 12n read + 12n write --
    if want("sort"):
        n = N
        vals = torch.arange(n, device=dev, dtype=torch.int32)
        for bits in (20, 32):
            keys = torch.randint(0, 1 << bits, (n,), generator=g, device=dev)
            ms = timed(lambda: ops.sort_pairs(keys, vals, bits), it)
            passes = (bits + 7) // 8
            report("sort_pairs", ms, passes * n * 32,
                   shape="%d (u64 key, i32 val), %d bits, %d passes" % (n, bits, passes))

    # -- Unique (grouped, 26 features): nnz*(8+4) + U*8 ------------------------
    if want("unique"):
        keys = torch.randint(0, 12_500_000, (N,), generator=g, device=dev)
        koff = [t * 65536 for t in range(27)]
        ms = timed(lambda: ops.unique_grouped(keys, koff), it)
        report("unique_grouped", ms, N * (8 + 4) + N * 8, shape="26 x 65536 keys")

    # -- FM 2nd order: B*F*D*4 + B*D*4; grad 2*B*F*D*4 + B*D*4 ----------------
    if want("fm2"):
        B, F, D = 65536, 26, 64
        e = torch.randn((B, F, D), generator=g, device=dev)
        ms = timed(lambda: ops.fm_second_order(e), it)
        report("fm2", ms, B * F * D * 4 + B * D * 4, shape="[%d,%d,%d]" % (B, F, D))
        top = torch.randn((B, D), generator=g, device=dev)
        ms = timed(lambda: ops.fm_second_order_grad(e, top), it)
        report("fm2_grad", ms, 2 * B * F * D * 4 + B * D * 4, shape="[%d,%d,%d]" % (B, F, D))

    # -- DLRM dot interaction: read B*F*D*4, write B*F(F-1)/2*4 ---------------
    if want("dot"):
        B, F, D = 65536, 27, 128
        x = torch.randn((B, F, D), generator=g, device=dev)
        ms = timed(lambda: ops.dot_interaction(x), it)
        report("dot_interaction", ms, B * F * D * 4 + B * F * (F - 1) // 2 * 4,
               flops=B * F * (F - 1) // 2 * 2 * D, shape="[%d,%d,%d]" % (B, F, D))

    # -- DCN-v2 CrossNet layer, bf16 MFMA: 2*B*d^2 flop ------------------------
    if want("crossnet"):
        for B in (16384, 65536):
            d = 13 + 26 * 128
            dp = (d + 63) // 64 * 64
            x0 = torch.randn((B, dp), generator=g, device=dev).to(torch.bfloat16)
            xl = torch.randn((B, dp), generator=g, device=dev).to(torch.bfloat16)
            w = (torch.randn((dp, dp), generator=g, device=dev) / dp ** 0.5).to(torch.bfloat16)
            bias = torch.zeros(dp, device=dev)
            out = torch.empty((B, dp), dtype=torch.bfloat16, device=dev)
            lin = torch.empty((B, dp), dtype=torch.bfloat16, device=dev)

            def cross(lin_out=None):
                check(lib().dr_crossnet_forward_bf16(ptr(x0), ptr(xl), ptr(w), ptr(bias), B, dp,
                                                     ptr(out), lin_out, stream_handle(dev)))
            ms = timed(cross, it)
            report("crossnet_layer_bf16", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (glds pipelined, fused epilogue)" % (B, dp))
            ms = timed(lambda: cross(ptr(lin)), it)
            report("crossnet_forward_bf16_with_lin", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (+ lin output)" % (B, dp))
            ms = timed(lambda: torch.matmul(xl, w.t()), it)
            report("torch_matmul_bf16_same_shape", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (hipBLASLt GEMM alone, no epilogue)" % (B, dp))
            ms = timed(lambda: torch.addcmul(xl, x0, torch.addmm(bias.to(torch.bfloat16), xl,
                                                                  w.t())), it)
            report("torch_crossnet_composed", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (hipBLASLt addmm + addcmul)" % (B, dp))
            # the backward's input gradient dx = u W + g: hand kernel on W^T
            # vs the library's addmm (the composed CrossStack step used it)
            wt = w.t().contiguous()
            dxo = torch.empty((B, dp), dtype=torch.bfloat16, device=dev)

            def dx():
                check(lib().dr_crossnet_dx_bf16(ptr(xl), ptr(wt), ptr(x0), B, dp, ptr(dxo),
                                                stream_handle(dev)))
            ms = timed(dx, it)
            report("crossnet_dx_bf16", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (dx = u W + g, 256^2 kernel on W^T)" % (B, dp))
            ms = timed(lambda: torch.addmm(x0, xl, w), it)
            report("torch_addmm_dx_same_shape", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (hipBLASLt addmm(g, u, W))" % (B, dp))
            ms = timed(lambda: torch.matmul(xl.t(), x0).float(), it)
            report("torch_dw_same_shape", ms, flops=2 * B * dp * dp,
                   shape="B %d, d %d (hipBLASLt u^T x + fp32 cast: the dW GEMM)" % (B, dp))

    # -- KV sparse apply: U*(24 + (1+2k)*D*4), k = columns touched -------------
    if want("apply"):
        R, D, U = 12_500_000, 128, 65536 * 26 // 2
        ev = dr.EmbeddingVariable("rl_ap", D, 0.0, capacity=R + (1 << 19), device=dev)
        ev.insert_synthetic(0, R, seed=5)
        acc = ev.slot("Adagrad", 0.1)
        m = ev.slot("Adam", 0.0)
        v = ev.slot("Adam_1", 0.0)
        keys = torch.randperm(R, generator=g, device=dev)[:U].contiguous()
        grad = torch.randn((U, D), generator=g, device=dev) * 1e-3
        # first touch of the slot columns outside the timed region
        check(lib().dr_ev_apply_adagrad(ev.handle, acc.handle, 0.0, ptr(grad), ptr(keys), U, None,
                                        1, stream_handle(dev)))
        check(lib().dr_ev_apply_adam(ev.handle, m.handle, v.handle, 0.9, 0.999, 0.0, 0.9, 0.999,
                                     1e-8, ptr(grad), ptr(keys), U, None, 1, stream_handle(dev)))
        torch.cuda.synchronize()

        def sgd():
            check(lib().dr_ev_apply_sgd(ev.handle, 1e-3, ptr(grad), ptr(keys), U, None, 1,
                                        stream_handle(dev)))

        def adagrad():
            check(lib().dr_ev_apply_adagrad(ev.handle, acc.handle, 1e-3, ptr(grad), ptr(keys), U,
                                            None, 1, stream_handle(dev)))

        def adam():
            check(lib().dr_ev_apply_adam(ev.handle, m.handle, v.handle, 0.9, 0.999, 1e-3, 0.9,
                                         0.999, 1e-8, ptr(grad), ptr(keys), U, None, 1,
                                         stream_handle(dev)))
        for name, fn, k in (("sgd", sgd, 1), ("adagrad", adagrad, 2), ("adam", adam, 3)):
            ms = timed(fn, it)
            report("ev_apply_" + name, ms, U * (24 + (1 + 2 * k) * D * 4),
                   shape="EV %d keys x %d, %d unique keys" % (R, D, U))
        del ev, acc, m, v


if __name__ == "__main__":
    main()
