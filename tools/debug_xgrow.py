"""Debug aid: the xgmi serve growth path on one GPU (world 1), repeated in one
process so that freed memory is reused; prints which rows come out wrong."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))

T, D, B, DEFAULT = 4, 64, 512, 0.5


def once(rep, cap):
    import deeprec_amd as dr
    from deeprec_amd.sharded import XgmiShardedLookup
    dev = torch.device("cuda", 0)
    evs = [dr.EmbeddingVariable("dbg%d_%d" % (rep, t), D, DEFAULT, device=dev, capacity=cap)
           for t in range(T)]
    eng = XgmiShardedLookup(evs, 1, 0, B, dev)
    for step in range(3):
        ids = (np.arange(T * B, dtype=np.int64).reshape(T, B) + step * T * B)
        with torch.no_grad():
            out = eng.forward(torch.as_tensor(ids, device=dev)).cpu().numpy().reshape(B, T, D)
        dr.status_check()
        bad = np.argwhere(~(out == np.float32(DEFAULT)).all(2))
        if bad.shape[0]:
            t = int(bad[0][1])
            keys = ids[t][bad[bad[:, 1] == t][:, 0]]
            rows = evs[t].resolve(torch.as_tensor(keys, device=dev)).cpu().numpy()
            print("rep %d step %d: %d bad (bag, table); tables %s; table %d rows %s ... "
                  "values %s" % (rep, step, bad.shape[0], np.unique(bad[:, 1]).tolist(), t,
                                 np.sort(rows)[:8].tolist(), out[bad[0][0], t, :4].tolist()),
                  flush=True)
    # junk traffic so that the next repetition reuses dirty memory
    x = torch.full((1 << 24,), 7.0, device=dev)
    del x, eng, evs


def main():
    import deeprec_amd as dr
    dr.load()
    for rep in range(6):
        once(rep, 256)
    print("done", flush=True)


if __name__ == "__main__":
    main()
