"""Two-process check of the peer-write engine through real HIP IPC mappings.

  python tools/xgmi_ipc_check.py [--world 2]

The parent never touches the GPU; it spawns `world` processes that all use
cuda:0 (a 1-GPU box cannot host two RCCL ranks, so the cross-rank barrier is
torch.cuda.synchronize() + a gloo barrier).  Each rank exports its inbox and
output through dr_ipc_export, maps the others with dr_ipc_import, runs three
XgmiShardedLookup steps and compares its output with the CPU oracle bit for
bit, and each step's backward (gradient rows pulled from the peers' mapped
gradient buffers) with the rows the requesters hold.  Prints one JSON line per rank; exit code != 0 on any mismatch.
"""
import argparse
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T, D, B, KEYSPACE, DEFAULT = 5, 128, 2048, 40000, 0.25


def _vals(t, keys):
    k = np.asarray(keys, np.float64)[:, None]
    return np.sin(0.011 * k + 0.9 * t + 0.07 * np.arange(D)[None, :]).astype(np.float32)


def _step_ids(step, rank):
    ids = np.random.default_rng(99 + 1000 * step + rank).integers(0, KEYSPACE, (T, B))
    ids = ids.astype(np.int64)
    ids[:, :7] = 5 + step
    return ids


def _step_grad(step, rank):
    rng = np.random.default_rng(7 + 1000 * step + rank)
    return rng.standard_normal((B, T * D)).astype(np.float32)


def worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import deeprec_amd as dr
    from deeprec_amd.sharded import XgmiShardedLookup
    from oracle import oracle as orc
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dr.load()
    own = np.arange(rank, KEYSPACE // 2, world, dtype=np.int64)
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("ipc%d_%d" % (rank, t), D, DEFAULT, capacity=KEYSPACE,
                                  device=dev)
        ev.insert(torch.as_tensor(own, device=dev), torch.as_tensor(_vals(t, own), device=dev))
        evs.append(ev)

    def barrier():
        torch.cuda.synchronize()
        dist.barrier()

    eng = XgmiShardedLookup(evs, world, rank, B, dev, barrier=barrier)
    allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    ok = bwd_ok = True
    for step in range(3):
        ids = _step_ids(step, rank)
        out = eng.forward(torch.as_tensor(ids, device=dev)).cpu().numpy()
        barrier()   # everyone copied its output before the next step rewrites it
        for t in range(T):
            ref_ev = orc.EV(D, DEFAULT)
            ref_ev.insert(allk, _vals(t, allk))
            ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[t], B, combiner="sum")
            if not np.array_equal(out[:, t * D:(t + 1) * D], ref):
                ok = False
        # backward: pull the gradient rows of the keys this rank owns from
        # every requester's mapped gradient buffer; each rank regenerates
        # the others' ids / grads from their seeds to build the expectation
        got = eng.backward(torch.as_tensor(_step_grad(step, rank), device=dev))
        for t in range(T):
            wk, wg = [], []
            for s in range(world):
                ids_s, g_s = _step_ids(step, s), _step_grad(step, s)
                sel = np.nonzero(ids_s[t] % world == rank)[0]
                wk.append(ids_s[t][sel])
                wg.append(g_s[sel, t * D:(t + 1) * D])
            k, v, n = got[t]
            m = int(n.item())
            bwd_ok = bwd_ok and np.array_equal(k[:m].cpu().numpy(), np.concatenate(wk)) and \
                np.array_equal(v[:m].cpu().numpy(), np.concatenate(wg).reshape(-1, D))
            evs[t].pending_grads.clear()
    dr.status_check(dev)
    for ev in evs:
        k = ev.export()[0].cpu().numpy()
        ok = ok and bool(np.all(k % world == rank))
    eng.close()
    # the parent prints the lines (one whole line per rank, never interleaved)
    q.put(json.dumps({"rank": rank, "world": world, "ipc_peer_write_ok": ok,
                      "ipc_grad_pull_ok": bool(bwd_ok)}))
    dist.destroy_process_group()
    if not (ok and bwd_ok):
        raise SystemExit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    q = mp.get_context("spawn").SimpleQueue()
    try:
        mp.spawn(worker, args=(args.world, port, q), nprocs=args.world, join=True)
    finally:
        while not q.empty():
            print(q.get(), flush=True)


if __name__ == "__main__":
    main()
