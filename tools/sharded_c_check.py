"""Multi-process check of the sharded C entries (dr_comm_init with a callback
table, dr_sharded_forward / dr_sharded_backward).

  python tools/sharded_c_check.py [--world 2]

The parent never touches the GPU; it spawns `world` processes that all use
cuda:0 and a gloo process group.  Each rank holds the EV shards of the keys
it owns (key % world == rank, rows f(t, key) pre-inserted for half the key
space, the rest first-touch defaults) and drives the exchange through the
library with Comm.host_staged (the gloo all-to-all behind the dr_comm
callback).  Checks, bit for bit:
  * forward (one-hot forward-only, one-hot with gradient, multi-hot mean,
    bf16 EVs) == this rank's batch looked up on one GPU in a full local copy
    of every table (embedding_lookup_sparse_multi);
  * backward (incl. hot keys over 257 / 5000 / 21846 / 65536 positions of
    a 70000-id batch): the owner's IndexedSlices == the concatenation over source
    ranks (ascending) of each source's first-occurrence unique keys that
    this rank owns with their SparseSegment*Grad rows (the oracle's Unique +
    sparse_segment_reduce_grad over every rank's batch and gradient).
  * the host-read-free kinds (dr_sharded_create_ex, round 6): XGMI (peer
    writes into IPC-mapped buffers; backward: every position's gradient row,
    source-rank-major, source-slot order) and the fixed-capacity all-to-all
    (the same slices as the variable engine) -- one-hot forward / backward,
    fixed-kind multi-hot mean bags, bf16 EVs -- through the comm's
    all_gather / barrier callbacks.
The parent prints one JSON line per rank (sent through a queue, so lines
never interleave); exit code != 0 on any mismatch.
"""
import argparse
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T, D, B, KEYSPACE, DEFAULT = 4, 32, 512, 6000, 0.125


def _vals(t, keys, dim=D):
    k = np.asarray(keys, np.float64)[:, None]
    return np.cos(0.013 * k + 0.7 * t + 0.05 * np.arange(dim)[None, :]).astype(np.float32)


def _onehot_ids(step, rank):
    ids = np.random.default_rng(31 + 1000 * step + rank).integers(0, KEYSPACE, (T, B))
    ids[:, :9] = 17 + step          # a repeated id in every table
    return ids.astype(np.int64)


LONG_RUNS = (257, 5000, 21846, 65536)   # per table (T = 4)


def _long_ids(rank, n):
    """[T, n] one-hot ids; table t's key 4321 + t fills LONG_RUNS[t] shuffled
    positions (a run of that length in the row-sorted backward)."""
    rng = np.random.default_rng(913 + rank)
    ids = rng.integers(0, KEYSPACE, (T, n)).astype(np.int64)
    for t in range(T):
        ids[t][ids[t] == 4321 + t] = 0
        ids[t, rng.permutation(n)[:LONG_RUNS[t]]] = 4321 + t
    return ids


def _bags(step, rank):
    """T tables of B bags of 0..4 ids (bag 0 holds 3): per table its ids and
    CSR offsets."""
    rng = np.random.default_rng(77 + 1000 * step + rank)
    lens = rng.integers(0, 5, (T, B))
    lens[:, 0] = 3
    ids, offs = [], []
    for t in range(T):
        o = np.concatenate([[0], np.cumsum(lens[t])]).astype(np.int32)
        v = rng.integers(0, KEYSPACE, int(o[-1])).astype(np.int64)
        v[: min(v.size, 5)] = 3                  # a hot key
        ids.append(v)
        offs.append(o)
    return ids, offs, lens


def _grad(step, rank, rows):
    return np.random.default_rng(5 + 1000 * step + rank).standard_normal(
        (rows, T * D)).astype(np.float32)


def worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import SparseTensor, embedding_lookup_sparse_multi
    from deeprec_amd.sharded import Comm, NativeShardedLookup
    from oracle import oracle as orc
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dr.load()
    dr.set_validate(True)
    half = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    res = {"rank": rank, "world": world, "checks": []}

    def evset(tag, value_dtype=torch.float32, full=False):
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("%s%d_%d" % (tag, rank, t), D, DEFAULT, capacity=KEYSPACE,
                                      device=dev, value_dtype=value_dtype)
            k = half if full else half[half % world == rank]
            v = _vals(t, k)
            ev.insert(torch.as_tensor(k, device=dev),
                      torch.as_tensor(v, device=dev).to(value_dtype))
            evs.append(ev)
        return evs

    comm = Comm.host_staged()
    shard = evset("sh")
    full = evset("fu", full=True)
    eng = NativeShardedLookup(comm, shard, dev)
    ok = True

    def check(name, a, b):
        nonlocal ok
        same = bool(np.array_equal(a, b))
        res["checks"].append([name, same])
        ok = ok and same

    ind1 = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64,
                                                                 device=dev)], 1)
    for step in range(2):
        # -- one-hot: forward-only (raw ids routed), then with gradient --
        ids = _onehot_ids(step, rank)
        it = torch.as_tensor(ids, device=dev)
        ref = embedding_lookup_sparse_multi(full, [SparseTensor(ind1, it[t], (B, 1))
                                                   for t in range(T)], combiner="sum")
        out = eng.forward(it, combiner="sum", need_grad=False)
        torch.cuda.synchronize()
        check("onehot_fwd_%d" % step, out.cpu().numpy(), ref.detach().cpu().numpy())
        out = eng.forward(it, combiner="sum", need_grad=True)
        check("onehot_fwd_grad_%d" % step, out.cpu().numpy(), ref.detach().cpu().numpy())
        g = _grad(step, rank, B)
        slices = eng.backward(torch.as_tensor(g, device=dev))
        for t in range(T):
            k, v = slices[t]
            kk, vv = [], []
            for p in range(world):
                idp = _onehot_ids(step, p)[t]
                gp = _grad(step, p, B)[:, t * D:(t + 1) * D]
                u, idx = orc.unique(idp)
                gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(gp), idx,
                                                    np.arange(B, dtype=np.int32), u.size, "sum")
                own = u % world == rank
                kk.append(u[own])
                vv.append(gu[own])
            check("onehot_bwd_keys_%d_%d" % (step, t), k.cpu().numpy(), np.concatenate(kk))
            check("onehot_bwd_grads_%d_%d" % (step, t), v.cpu().numpy(), np.concatenate(vv))
        for e in shard:
            e.pending_grads.clear()
        # -- multi-hot mean bags --
        ids, offs, lens = _bags(step, rank)
        it = [torch.as_tensor(x, device=dev) for x in ids]
        ot = [torch.as_tensor(o, device=dev) for o in offs]
        sps = []
        for t in range(T):
            rows = np.repeat(np.arange(B), lens[t])
            ind = np.stack([rows, np.zeros_like(rows)], 1).astype(np.int64)
            sps.append(SparseTensor(torch.as_tensor(ind, device=dev), it[t], (B, 5)))
        ref = embedding_lookup_sparse_multi(full, sps, combiner="mean")
        out = eng.forward(it, bag_offs=ot, combiner="mean", need_grad=True)
        torch.cuda.synchronize()
        check("bags_fwd_%d" % step, out.cpu().numpy(), ref.detach().cpu().numpy())
        g = _grad(100 + step, rank, B)
        slices = eng.backward(torch.as_tensor(g, device=dev))
        for t in range(T):
            k, v = slices[t]
            kk, vv = [], []
            for p in range(world):
                idp, offp, lenp = _bags(step, p)
                u, idx = orc.unique(idp[t])
                seg = np.repeat(np.arange(B), lenp[t]).astype(np.int32)
                gp = _grad(100 + step, p, B)[:, t * D:(t + 1) * D]
                gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(gp), idx, seg, u.size,
                                                    "mean")
                own = u % world == rank
                kk.append(u[own])
                vv.append(gu[own])
            check("bags_bwd_keys_%d_%d" % (step, t), k.cpu().numpy(), np.concatenate(kk))
            check("bags_bwd_grads_%d_%d" % (step, t), v.cpu().numpy(), np.concatenate(vv))
        for e in shard:
            e.pending_grads.clear()
    # -- long runs: table t's hot key over LONG_RUNS[t] of BL positions on every
    # rank (257 .. 65536): each source's SparseSegment*Grad row of it is one
    # serial chain on the Unique path of the sharded backward --
    BL = 70000
    indl = torch.stack([torch.arange(BL, device=dev),
                        torch.zeros(BL, dtype=torch.int64, device=dev)], 1)
    ids = _long_ids(rank, BL)
    it = torch.as_tensor(ids, device=dev)
    ref = embedding_lookup_sparse_multi(full, [SparseTensor(indl, it[t], (BL, 1))
                                               for t in range(T)], combiner="sum")
    out = eng.forward(it, combiner="sum", need_grad=True)
    torch.cuda.synchronize()
    check("long_fwd", out.cpu().numpy(), ref.detach().cpu().numpy())
    g = _grad(200, rank, BL)
    slices = eng.backward(torch.as_tensor(g, device=dev))
    for t in range(T):
        k, v = slices[t]
        kk, vv = [], []
        for p in range(world):
            idp = _long_ids(p, BL)[t]
            gp = _grad(200, p, BL)[:, t * D:(t + 1) * D]
            u, idx = orc.unique(idp)
            gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(gp), idx,
                                                np.arange(BL, dtype=np.int32), u.size, "sum")
            own = u % world == rank
            kk.append(u[own])
            vv.append(gu[own])
        check("long_bwd_keys_%d" % t, k.cpu().numpy(), np.concatenate(kk))
        check("long_bwd_grads_%d" % t, v.cpu().numpy(), np.concatenate(vv))
    for e in shard:
        e.pending_grads.clear()
    # -- bf16 EVs: bf16 rows on the wire, fp32 and bf16 outputs --
    sb = evset("bs", torch.bfloat16)
    fb = evset("bf", torch.bfloat16, full=True)
    eb = NativeShardedLookup(comm, sb, dev)
    ids = _onehot_ids(9, rank)
    it = torch.as_tensor(ids, device=dev)
    sps = [SparseTensor(ind1, it[t], (B, 1)) for t in range(T)]
    with torch.no_grad():
        ref32 = embedding_lookup_sparse_multi(fb, sps, combiner="sum")
        ref16 = embedding_lookup_sparse_multi(fb, sps, combiner="sum", out_dtype=torch.bfloat16)
    o32 = eb.forward(it, combiner="sum")
    check("bf16_fwd_fp32", o32.cpu().numpy(), ref32.float().cpu().numpy())
    o16 = eb.forward(it, combiner="sum", out_dtype=torch.bfloat16)
    check("bf16_fwd_bf16", o16.view(torch.int16).cpu().numpy(),
          ref16.view(torch.int16).cpu().numpy())
    dr.status_check()
    eng.close()
    eb.close()
    # -- the host-read-free kinds (dr_sharded_create_ex): XGMI peer writes and
    # the fixed-capacity all-to-all, on the same shards and batches --
    for kind in ("xgmi", "fixed"):
        ek = NativeShardedLookup(comm, shard, dev, kind=kind, batch=B, max_ids=70000)
        for step in range(2):
            ids = _onehot_ids(step, rank)
            it = torch.as_tensor(ids, device=dev)
            ref = embedding_lookup_sparse_multi(full, [SparseTensor(ind1, it[t], (B, 1))
                                                       for t in range(T)], combiner="sum")
            out = ek.forward(it, combiner="sum", need_grad=False)
            torch.cuda.synchronize()
            check("%s_onehot_fwd_%d" % (kind, step), out.cpu().numpy(), ref.detach().cpu().numpy())
            out = ek.forward(it, combiner="sum", need_grad=True)
            check("%s_onehot_fwd_grad_%d" % (kind, step), out.cpu().numpy(),
                  ref.detach().cpu().numpy())
            g = _grad(step, rank, B)
            slices = ek.backward(torch.as_tensor(g, device=dev))
            for t in range(T):
                k, v, n = slices[t]
                n = int(n.item())
                kk, vv = [], []
                for p in range(world):
                    idp = _onehot_ids(step, p)[t]
                    gp = _grad(step, p, B)[:, t * D:(t + 1) * D]
                    if kind == "xgmi":   # every position, in source-slot order
                        own = idp % world == rank
                        kk.append(idp[own])
                        vv.append(gp[own])
                        continue
                    u, idx = orc.unique(idp)
                    gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(gp), idx,
                                                        np.arange(B, dtype=np.int32), u.size, "sum")
                    own = u % world == rank
                    kk.append(u[own])
                    vv.append(gu[own])
                check("%s_onehot_bwd_keys_%d_%d" % (kind, step, t), k[:n].cpu().numpy(),
                      np.concatenate(kk))
                check("%s_onehot_bwd_grads_%d_%d" % (kind, step, t), v[:n].cpu().numpy(),
                      np.concatenate(vv))
            for e in shard:
                e.pending_grads.clear()
        if kind == "fixed":
            # multi-hot mean bags through the fixed regions
            ids, offs, lens = _bags(0, rank)
            it = [torch.as_tensor(x, device=dev) for x in ids]
            ot = [torch.as_tensor(o, device=dev) for o in offs]
            sps = []
            for t in range(T):
                rows = np.repeat(np.arange(B), lens[t])
                ind = np.stack([rows, np.zeros_like(rows)], 1).astype(np.int64)
                sps.append(SparseTensor(torch.as_tensor(ind, device=dev), it[t], (B, 5)))
            ref = embedding_lookup_sparse_multi(full, sps, combiner="mean")
            out = ek.forward(it, bag_offs=ot, combiner="mean", need_grad=True)
            torch.cuda.synchronize()
            check("fixed_bags_fwd", out.cpu().numpy(), ref.detach().cpu().numpy())
            g = _grad(100, rank, B)
            slices = ek.backward(torch.as_tensor(g, device=dev))
            for t in range(T):
                k, v, n = slices[t]
                n = int(n.item())
                kk, vv = [], []
                for p in range(world):
                    idp, offp, lenp = _bags(0, p)
                    u, idx = orc.unique(idp[t])
                    seg = np.repeat(np.arange(B), lenp[t]).astype(np.int32)
                    gp = _grad(100, p, B)[:, t * D:(t + 1) * D]
                    gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(gp), idx, seg, u.size,
                                                        "mean")
                    own = u % world == rank
                    kk.append(u[own])
                    vv.append(gu[own])
                check("fixed_bags_bwd_keys_%d" % t, k[:n].cpu().numpy(), np.concatenate(kk))
                check("fixed_bags_bwd_grads_%d" % t, v[:n].cpu().numpy(), np.concatenate(vv))
            for e in shard:
                e.pending_grads.clear()
        ek.close()
        # bf16 EVs: fp32 and bf16 outputs
        ekb = NativeShardedLookup(comm, sb, dev, kind=kind, batch=B, max_ids=B)
        ids = _onehot_ids(9, rank)
        it = torch.as_tensor(ids, device=dev)
        o32 = ekb.forward(it, combiner="sum")
        check("%s_bf16_fwd_fp32" % kind, o32.cpu().numpy(), ref32.float().cpu().numpy())
        o16 = ekb.forward(it, combiner="sum", out_dtype=torch.bfloat16)
        check("%s_bf16_fwd_bf16" % kind, o16.view(torch.int16).cpu().numpy(),
              ref16.view(torch.int16).cpu().numpy())
        ekb.close()
    dr.status_check()
    comm.close()
    res["ok"] = ok
    q.put(json.dumps(res))   # the parent prints: one whole line per rank
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    import multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, args.world, port, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    import queue
    for _ in procs:
        try:
            print(q.get(timeout=300), flush=True)
        except queue.Empty:
            break
    for p in procs:
        p.join(60)
    codes = [p.exitcode for p in procs]
    sys.exit(0 if all(c == 0 for c in codes) else 1)


if __name__ == "__main__":
    main()
