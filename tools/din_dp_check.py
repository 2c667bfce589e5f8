"""Data-parallel DIN (BASELINE configs[3], 1 -> N GPUs) across PROCESSES on
one GPU, rehearsed with gloo:

  python tools/din_dp_check.py [--world 2]

Every rank holds the whole uid / mid / cat EVs (replicated), the same dense
initialisation and its slice of one global batch (each slice padded to the
same history length).  A step is modelzoo.din_train_step(..., world=N):
local loss / N, dense gradients all-reduced, every EV's gradient slices
gathered in rank order (sharded.sync_replicated_grads), SGD + KV SGD.
Reference: one process running the same data-parallel step (every slice's
forward on its own -- DIN's Dice normalises over the batch a replica sees --
gradients of all slices accumulated, one optimizer step).
After each of three steps every rank checks its loss share, dense weights
and all three tables against the reference (1e-5 relative), and the
replicas against each other (bit-identical).  The parent prints one JSON
line per rank (through a queue)."""
import argparse
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, TMAX, D, LR = 128, 12, 8, 0.05
R = (300, 200, 20)


def worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import deeprec_amd as dr
    from deeprec_amd import modelzoo as mz
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dr.load()

    def evset(tag):
        evs = []
        for i, r in enumerate(R):
            ev = dr.EmbeddingVariable("%s%d_%d" % (tag, rank, i), D, 0.0, capacity=4 * r,
                                      device=dev)
            k = np.arange(r, dtype=np.int64)
            v = (0.1 * np.sin(0.3 * k[:, None] + i + 0.2 * np.arange(D)[None, :])).astype(np.float32)
            ev.insert(torch.as_tensor(k, device=dev), torch.as_tensor(v, device=dev))
            evs.append(ev)
        return evs

    mine, full = evset("dp"), evset("rf")
    torch.manual_seed(0)
    model = mz.DIN(*mine).to(dev)
    torch.manual_seed(0)
    ref = mz.DIN(*full).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=LR)
    ropt = torch.optim.SGD(ref.parameters(), lr=LR)
    eo, reo = dr.GradientDescentOptimizer(LR), dr.GradientDescentOptimizer(LR)
    res = {"rank": rank, "world": world, "checks": []}
    ok = True
    for step in range(3):
        rng = np.random.default_rng(40 + step)                # one global batch
        n = world * B
        lens = rng.integers(1, TMAX + 1, n)
        lens[::B] = TMAX                                       # every slice pads to TMAX
        mask = (np.arange(TMAX)[None, :] < lens[:, None]).astype(np.float32)
        mh = rng.integers(1, R[1], (n, TMAX)) * mask.astype(np.int64)
        ch = rng.integers(1, R[2], (n, TMAX)) * mask.astype(np.int64)
        lab = (rng.random(n) > 0.5).astype(np.int64)
        glob = [rng.integers(0, R[0], n), rng.integers(0, R[1], n), rng.integers(0, R[2], n),
                mh, ch, mask, np.stack([lab, 1 - lab], 1).astype(np.float32)]
        tg = [torch.as_tensor(x, device=dev) for x in glob]
        sl = slice(rank * B, (rank + 1) * B)
        loss = mz.din_train_step(model, [x[sl].contiguous() for x in tg], opt, eo, step,
                                 world=world, staged=True)
        # reference: the same data-parallel step in one process -- DIN's
        # Dice activations normalise over the batch a replica sees, so each
        # slice's forward is its own; the slices' gradients accumulate
        # (dense: autograd sums, EVs: slices queued in rank order) before one
        # optimizer step
        ropt.zero_grad(set_to_none=True)
        rl = []
        for r in range(world):
            rs = slice(r * B, (r + 1) * B)
            part = [x[rs].contiguous() for x in tg]
            y = ref(*part[:6])
            lr_ = -(torch.log(y) * part[6]).mean()
            (lr_ / world).backward()
            rl.append(float(lr_.detach()))
        ropt.step()
        reo.apply_gradients(ref.evs, global_step=step)
        rloss = sum(rl) / world
        lt = torch.tensor([float(loss.detach())], dtype=torch.float64)
        dist.all_reduce(lt)
        gl = lt.item() / world
        c_loss = abs(gl - float(rloss)) <= 1e-5 * abs(float(rloss)) + 1e-7
        derr = max((p.detach() - rp.detach()).abs().max().item()
                   / (rp.detach().abs().max().item() + 1e-12)
                   for p, rp in zip(model.parameters(), ref.parameters()))
        terr, same = 0.0, True
        for e, re_ in zip(mine, full):
            k, v = e.export()[:2]
            rk, rv = re_.export()[:2]
            o, ro = torch.argsort(k), torch.argsort(rk)
            same = same and torch.equal(k[o], rk[ro])
            terr = max(terr, (v[o] - rv[ro]).abs().max().item() / (rv.abs().max().item() + 1e-12))
        # the replicas are bit-identical across ranks
        vals = torch.cat([e.export()[1][torch.argsort(e.export()[0])].reshape(-1) for e in mine])
        h = vals.cpu().double()
        s = torch.tensor([float(h.sum()), float((h * h).sum())], dtype=torch.float64)
        s0 = s.clone()
        dist.broadcast(s0, 0)
        rep_same = bool(torch.equal(s, s0))
        good = c_loss and derr <= 1e-5 and terr <= 1e-5 and same and rep_same
        res["checks"].append({"step": step, "loss": [gl, float(rloss)], "dense_rel_err": derr,
                              "tables_rel_err": terr, "replicas_identical": rep_same,
                              "ok": bool(good)})
        ok = ok and good
    dr.status_check()
    res["ok"] = bool(ok)
    q.put(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    import multiprocessing as mp
    import queue
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, args.world, port, q)) for r in range(args.world)]
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
