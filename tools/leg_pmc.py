"""Launch only the fused one-hot EV lookup of one bench leg, for rocprofv3
--pmc passes (FETCH_SIZE / WRITE_SIZE each in its own run): the leg's
tables (bench.py deepfm_leg: 26 x 10 M x 64 fp32; dcn_bf16_leg: 26 x 12.5 M
x 128 bf16, bf16 output), its 4 rotating batches, --iters launches timed with
HIP events (bench._onehot_kernel_ms).  The tables' bulk-insert kernels run
first under other names; tools/pmc_summary.py keeps the lookup kernel's
dispatches only.

usage: python tools/leg_pmc.py --leg deepfm|dcn [--iters 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", choices=("deepfm", "dcn"), required=True)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536)
    args = ap.parse_args()
    import bench
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import _Feature
    dr.load()
    dev = torch.device("cuda:0")
    if args.leg == "deepfm":
        T, D, R, dt, seed0, out = 26, 64, 10_000_000, torch.float32, 5000, None
    else:
        T, D, R, dt, seed0, out = 26, 128, 12_500_000, torch.bfloat16, 6000, torch.bfloat16
    B = args.batch
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("%s%d" % (args.leg, t), D, 0.0, device=dev,
                                  capacity=R + (1 << 20), value_dtype=dt)
        ev.insert_synthetic(0, R, seed=seed0 + t)
        evs.append(ev)
    batches = bench.make_batches(4, T, B, R, 0.0, 91, dev)
    recs = [ids.t().contiguous() for ids in batches]
    seg = torch.arange(B, dtype=torch.int32, device=dev)
    fsets = [[_Feature(evs[t], r[:, t], seg, B, None, "sum", None, onehot=True) for t in range(T)]
             for r in recs]
    torch.cuda.synchronize()
    k_ms = bench._onehot_kernel_ms(fsets, args.iters, out_dtype=out)
    row = D * (2 if dt == torch.bfloat16 else 4)
    per = 8 + 16 + 2 * row
    print(json.dumps({"leg": args.leg, "kernel_ms": round(k_ms, 4), "bytes_per_lookup": per,
                      "bytes_per_launch": T * B * per,
                      "frac": round(T * B * per / (k_ms * 1e-3) / 1e9 / bench.PEAK_HBM_GBS, 4)}),
          flush=True)
    dr.status_check(dev)


if __name__ == "__main__":
    main()
