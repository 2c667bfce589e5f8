"""CrossNet backward weight gradient at the DCN shape (B = 65 536,
d = 3 392): dW = u^T x as torch.matmul (hipBLASLt) vs the hand TN MFMA GEMM
(dr_gemm_tn_bf16) over split-K choices; times with HIP events on the current
stream and the max relative difference between the two."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    import deeprec_amd as dr
    from deeprec_amd import ops
    from deeprec_amd.modelzoo import _dw_split
    dr.load()
    B, d = 65536, 3392
    g = torch.Generator(device="cuda").manual_seed(1)
    u = torch.randn(B, d, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(B, d, device="cuda", generator=g).to(torch.bfloat16)
    flop = 2.0 * B * d * d
    if "--hand-only" in sys.argv:   # counter passes: the hand kernel alone, 5 calls
        for _ in range(5):
            ops.crossnet_dw(u, x)
        torch.cuda.synchronize()
        print("hand dW x5 done", flush=True)
        return
    ref = torch.matmul(u.t(), x).float()
    t = timed(lambda: torch.matmul(u.t(), x).float())
    print("matmul(u.t(), x).float(): %.3f ms  %.0f TF/s" % (t, flop / t / 1e9), flush=True)
    got = ops.crossnet_dw(u, x)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    t = timed(lambda: ops.crossnet_dw(u, x))
    print("crossnet_dw (256^2 four-phase TN, split %d): %.3f ms  %.0f TF/s  max rel diff %.2e"
          % (dr._lib.lib().dr_crossnet_dw_workspace_size(B, d) // (4 * d * d), t, flop / t / 1e9,
             err), flush=True)
    if os.environ.get("DR_CROSSNET_DW_KERNEL", "w4") == "w4":   # work orders (read per call)
        for o in ("0", "2", "4", "8", "14", "xcd"):
            os.environ["DR_CROSSNET_DW_ORDER"] = o
            got = ops.crossnet_dw(u, x)
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            t = timed(lambda: ops.crossnet_dw(u, x))
            print("crossnet_dw w4 order %s: %.3f ms  %.0f TF/s  max rel diff %.2e"
                  % (o, t, flop / t / 1e9, err), flush=True)
        del os.environ["DR_CROSSNET_DW_ORDER"]
    t = timed(lambda: torch.matmul(u.t(), x).float())
    print("matmul(u.t(), x).float() again: %.3f ms" % t, flush=True)
    try:   # the library GEMM writing fp32 directly (aten::mm.dtype)
        got = torch.mm(u.t(), x, out_dtype=torch.float32)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        t = timed(lambda: torch.mm(u.t(), x, out_dtype=torch.float32))
        print("mm(u.t(), x, out_dtype=fp32): %.3f ms  %.0f TF/s  max rel diff %.2e"
              % (t, flop / t / 1e9, err), flush=True)
    except Exception as e:  # not in this torch build
        print("mm out_dtype unavailable: %s" % str(e)[:120], flush=True)
    tiles = ((d + 127) // 128) ** 2
    for s in sorted({1, 2, 4, _dw_split(tiles, B)}):
        got = ops.gemm_tn(u, x, split_k=s)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        t = timed(lambda: ops.gemm_tn(u, x, split_k=s))
        print("gemm_tn split %d: %.3f ms  %.0f TF/s  max rel diff %.2e" % (s, t, flop / t / 1e9, err),
              flush=True)


if __name__ == "__main__":
    main()
