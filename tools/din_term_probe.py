"""How repetitive are the terms of DIN's padding-id run?  One DIN step at
the bench shape (tools/model_step.py din): the gradient reaching the history
lookup, read at the padding positions (mask 0, id 0) in ascending position
order -- the order of the run's serial sum -- and split into segments of
bitwise-identical rows.  Prints the run length, the number of segments
(whole rows and per column) and the longest segment."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))


def main():
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dev = torch.device("cuda:0")
    B, T, D = 4096, 100, 18
    R = (500_000, 400_000, 2_000)
    evs = []
    for i, r in enumerate(R):
        ev = dr.EmbeddingVariable("dtp%d" % i, D, 0.0, capacity=r + (1 << 16), device=dev)
        ev.insert_synthetic(0, r, seed=700 + i)
        evs.append(ev)
    model = mz.DIN(*evs).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(2021)
    lens = torch.randint(1, T + 1, (B,), generator=g, device=dev)
    Tb = int(lens.max())
    mask = (torch.arange(Tb, device=dev)[None, :] < lens[:, None]).float()
    mh = torch.randint(1, R[1], (B, Tb), generator=g, device=dev) * mask.long()
    ch = torch.randint(1, R[2], (B, Tb), generator=g, device=dev) * mask.long()
    lab = (torch.rand(B, generator=g, device=dev) > 0.5).long()
    batch = (torch.randint(0, R[0], (B,), generator=g, device=dev),
             torch.randint(0, R[1], (B,), generator=g, device=dev),
             torch.randint(0, R[2], (B,), generator=g, device=dev), mh, ch, mask,
             torch.stack([lab, 1 - lab], 1).float())
    # DTP_STEPS: train this many steps first (Adam, the bench's optimizers),
    # so the terms are a trained model's rather than the first step's
    nsteps = int(os.environ.get("DTP_STEPS", "0"))
    if nsteps:
        dopt = torch.optim.Adam(model.parameters(), lr=0.001)
        eopt = dr.AdamOptimizer(0.001)
        for i in range(nsteps):
            mz.din_train_step(model, batch, dopt, eopt, i)
        torch.cuda.synchronize()
    grads = []
    inner = model.item_lookup

    class Hooked(object):
        def __call__(self, ids):
            out = inner(ids)
            if ids.shape[1] in (B * Tb, B + B * Tb):   # history-only or one item lookup
                out.register_hook(lambda gr: grads.append(gr.detach().clone()))
            return out
    model.item_lookup = Hooked()
    y = model(*batch[:6])
    loss = -(torch.log(y) * batch[6]).mean()
    loss.backward()
    torch.cuda.synchronize()
    gh = grads[0][-B * Tb:].reshape(B * Tb, 2, D)     # [positions, table, D]
    pad = (mask.reshape(-1) == 0).nonzero().squeeze(1)  # ascending positions of id 0
    segs = {}
    for t, name in ((0, "mid"), (1, "cat")):
        rows = gh[pad, t].contiguous().view(torch.int32)
        n = rows.shape[0]
        diff_row = (rows[1:] != rows[:-1]).any(1)
        seg = 1 + int(diff_row.sum())
        diff_col = (rows[1:] != rows[:-1])
        seg_col = 1 + diff_col.sum(0)
        bounds = torch.cat([torch.zeros(1, dtype=torch.long, device=dev),
                            diff_row.nonzero().squeeze(1) + 1,
                            torch.tensor([n], device=dev)])
        longest = int((bounds[1:] - bounds[:-1]).max())
        if os.environ.get("DTP_SAVE"):   # segment terms + lengths, for host replays
            import numpy as np
            segs[name] = (rows[bounds[:-1]].view(torch.float32).cpu().numpy(),
                          (bounds[1:] - bounds[:-1]).cpu().numpy())
        print("%s: padding run %d positions, %d row segments (mean %.1f, longest %d), "
              "per-column segments %d..%d; samples with padding %d"
              % (name, n, seg, n / seg, longest, int(seg_col.min()), int(seg_col.max()),
                 int((lens < Tb).sum())), flush=True)
    if segs:
        import numpy as np
        np.savez(os.environ["DTP_SAVE"], **{"%s_terms" % k: v[0] for k, v in segs.items()},
                 **{"%s_len" % k: v[1] for k, v in segs.items()})


if __name__ == "__main__":
    main()
