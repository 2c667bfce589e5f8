"""Data-parallel DLRM with row-sharded embeddings, across PROCESSES on one GPU
(the N > 1 model step of modelzoo/SOK/DLRM, rehearsed with gloo):

  python tools/dlrm_sharded_check.py [--world 2] [--engine a2a|xgmi]

Every rank holds the EV shards of the keys it owns (key % world == rank),
the same dense initialisation, and its slice of one global batch.  Each step
is modelzoo.train_step_sharded: DLRM forward with the sharded lookup
(ShardedLookup, all-to-alls staged through host memory over gloo, or the
peer-write engine over HIP IPC), local mean loss / world, backward (dense
gradients all-reduced; embedding gradient rows delivered to their owners),
SGD on the dense weights and KV SGD on the shards.  Reference: one process
with the full tables training the same DLRM on the whole global batch
(modelzoo.train_step, global mean loss).  After each step every rank checks
its dense weights and its owned EV rows against the reference (fp32
tolerance: the towers' GEMMs and the gradient sums associate differently).
--model dcn: DCN-v2 (BASELINE configs[4], bf16 cross layers on the MFMA
kernel) instead of DLRM; its tolerance is the bf16 one (1/64 of the
reference's magnitude, as tests/test_gpu_dcn.py).
--hybrid: features 0 and 2 replicated on every rank (local lookups, their
gradient slices gathered by sharded.sync_replicated_grads), 1 and 3 sharded;
every replica must equal the reference's whole table.
The parent prints one JSON line per rank (sent through a queue)."""
import argparse
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T, D, B, KEYS, LR = 4, 16, 256, 3000, 0.1


def _vals(t, keys):
    k = np.asarray(keys, np.float64)[:, None]
    return (0.1 * np.cos(0.017 * k + 0.9 * t + 0.07 * np.arange(D)[None, :])).astype(np.float32)


def worker(rank, world, port, engine_kind, hybrid, model_kind, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    from deeprec_amd.sharded import ShardedLookup, XgmiShardedLookup
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dr.load()
    allk = np.arange(KEYS, dtype=np.int64)

    def evset(tag, keys):
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("%s%d_%d" % (tag, rank, t), D, 0.0, capacity=2 * KEYS,
                                      device=dev)
            ev.insert(torch.as_tensor(keys, device=dev), torch.as_tensor(_vals(t, keys), device=dev))
            evs.append(ev)
        return evs

    own = allk[allk % world == rank]
    # hybrid: features 0 and 2 replicated (the whole table on every rank),
    # 1 and 3 row-sharded
    rep = [0, 2] if hybrid else []
    shard = evset("sh", own)
    full = evset("fu", allk)
    if rep:
        repl = evset("rp", allk)
        model_evs = [repl[t] if t in rep else shard[t] for t in range(T)]
        eng_evs = [shard[t] for t in range(T) if t not in rep]
    else:
        model_evs, eng_evs = shard, shard

    def staged_a2a(out, inp, out_splits=None, in_splits=None):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
        out.copy_(o)
        return out

    if engine_kind == "xgmi":
        def barrier():
            torch.cuda.synchronize()
            dist.barrier()
        engine = XgmiShardedLookup(eng_evs, world, rank, B, dev, barrier=barrier)
    else:
        engine = ShardedLookup(eng_evs, world, rank, B, dev)
        engine._a2a = staged_a2a
    torch.manual_seed(0)
    if model_kind == "dcn":
        model = mz.DCNv2(model_evs, 13, layers=2, deep=(64, 32), engine=engine).to(dev)
        torch.manual_seed(0)
        ref = mz.DCNv2(full, 13, layers=2, deep=(64, 32)).to(dev)
    else:
        model = mz.DLRM(model_evs, 13, mlp_bot=(64,), mlp_top=(64, 32), engine=engine,
                        replicated=rep).to(dev)
        torch.manual_seed(0)
        ref = mz.DLRM(full, 13, mlp_bot=(64,), mlp_top=(64, 32)).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=LR)
    ropt = torch.optim.SGD(ref.parameters(), lr=LR)
    ev_opt, rev_opt = dr.GradientDescentOptimizer(LR), dr.GradientDescentOptimizer(LR)
    res = {"rank": rank, "world": world, "engine": engine_kind, "hybrid": bool(rep),
           "model": model_kind, "checks": []}
    ok = True
    for step in range(3):
        rng = np.random.default_rng(100 + step)           # the same global batch on every rank
        ids_all = (rng.zipf(1.2, size=(T, world * B)) - 1) % KEYS
        dense_all = rng.standard_normal((world * B, 13)).astype(np.float32)
        lab_all = (rng.random(world * B) > 0.5).astype(np.float32)
        sl = slice(rank * B, (rank + 1) * B)
        ids = torch.as_tensor(np.ascontiguousarray(ids_all[:, sl]), device=dev)
        loss = mz.train_step_sharded(model, torch.as_tensor(dense_all[sl], device=dev), ids,
                                     torch.as_tensor(lab_all[sl], device=dev), opt, ev_opt, world,
                                     staged=True)
        rloss = mz.train_step(ref, torch.as_tensor(dense_all, device=dev),
                              torch.as_tensor(ids_all, device=dev),
                              torch.as_tensor(lab_all, device=dev), ropt, rev_opt)
        lt = torch.tensor([float(loss)], dtype=torch.float64)
        dist.all_reduce(lt)
        gl = lt.item() / world
        tol = 1e-5 if model_kind == "dlrm" else 1.0 / 64     # bf16 layers: bf16 tolerance
        c_loss = abs(gl - float(rloss)) <= tol * abs(float(rloss)) + 1e-6
        errs = []
        for (n, p), (_, rp) in zip(model.named_parameters(), ref.named_parameters()):
            errs.append((p.detach() - rp.detach()).abs().max().item()
                        / (rp.detach().abs().max().item() + 1e-12))
        c_dense = max(errs) <= tol
        c_rows = True
        emax = 0.0
        for t in range(T):
            k, v = model_evs[t].export()[:2]
            rk, rv = full[t].export()[:2]
            order = torch.argsort(k)
            k, v = k[order], v[order]
            sel = (rk % world) == rank if t not in rep else torch.ones_like(rk, dtype=torch.bool)
            rk, rv = rk[sel], rv[sel]
            ro = torch.argsort(rk)
            rk, rv = rk[ro], rv[ro]
            same_keys = torch.equal(k, rk)
            e = (v - rv).abs().max().item() / (rv.abs().max().item() + 1e-12)
            emax = max(emax, e)
            c_rows = c_rows and same_keys and e <= tol
        res["checks"].append({"step": step, "loss": [gl, float(rloss)], "loss_ok": c_loss,
                              "dense_rel_err": max(errs), "rows_rel_err": emax,
                              "ok": bool(c_loss and c_dense and c_rows)})
        ok = ok and c_loss and c_dense and c_rows
    dr.status_check()
    if hasattr(engine, "close"):
        engine.close()
    res["ok"] = bool(ok)
    q.put(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--engine", default="a2a", choices=["a2a", "xgmi"])
    ap.add_argument("--model", default="dlrm", choices=["dlrm", "dcn"])
    ap.add_argument("--hybrid", action="store_true",
                    help="features 0 and 2 replicated, 1 and 3 sharded")
    args = ap.parse_args()
    import multiprocessing as mp
    import queue
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, args.world, port, args.engine, args.hybrid,
                                                  args.model, q))
             for r in range(args.world)]
    for p in procs:
        p.start()
    for _ in procs:
        try:
            print(q.get(timeout=300), flush=True)
        except queue.Empty:
            break
    for p in procs:
        p.join(60)
    sys.exit(0 if all(p.exitcode == 0 for p in procs) else 1)


if __name__ == "__main__":
    main()
