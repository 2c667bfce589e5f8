"""DLRM tower GEMMs: the hand MFMA path (modelzoo._MfmaMLP, dr_gemm_nt_bf16)
against torch autocast bf16 (hipBLASLt) on the same Linear stack, forward +
backward, B = 65 536.  Prints one JSON line per tower.  A measurement aid for
DESIGN.md (profiles/r03_mlp_probe.log).

  python tools/mlp_probe.py [--batch 65536] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dr.load()
    dev = torch.device("cuda", 0)
    B = args.batch
    for name, sizes in (("dlrm_top", [479, 512, 256]), ("dlrm_bottom", [13, 512, 256, 128])):
        torch.manual_seed(0)
        hand = mz._MfmaMLP(sizes).to(dev)
        lib = mz._mlp(sizes).to(dev)
        lib.load_state_dict({k.split("net.", 1)[1]: v for k, v in hand.state_dict().items()})
        x = torch.randn((B, sizes[0]), device=dev, requires_grad=True)
        go = torch.randn((B, sizes[-1]), device=dev)

        def run_hand():
            hand(x).backward(go)

        def run_lib():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = lib(x).float()
            y.backward(go)

        th = timed(run_hand, args.iters)
        tl = timed(run_lib, args.iters)
        fl = sum(2 * B * sizes[i] * sizes[i + 1] for i in range(len(sizes) - 1)) * 3
        print(json.dumps({"tower": name, "sizes": sizes, "batch": B,
                          "hand_mfma_ms": round(th, 4), "torch_autocast_ms": round(tl, 4),
                          "gemm_tflops_hand": round(fl / th / 1e9, 1),
                          "gemm_tflops_torch": round(fl / tl / 1e9, 1),
                          "step": "forward + backward (dx, dW, db) of the tower"}), flush=True)


if __name__ == "__main__":
    main()
