"""Debug helper: capture each engine op in a CUDA graph and replay it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
import torch  # noqa: E402

import deeprec_amd as dr  # noqa: E402
from deeprec_amd import ops  # noqa: E402


def log(*a):
    print("[dbg]", *a, file=sys.stderr, flush=True)


def trial(name, fn, reps=3):
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    log(name, "captured")
    for r in range(reps):
        t = time.time()
        g.replay()
        torch.cuda.synchronize()
        log(name, "replay", r, "%.4fs" % (time.time() - t))


def main():
    import faulthandler
    faulthandler.dump_traceback_later(25, exit=True)
    dev = torch.device("cuda", 0)
    dr.load()
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    T, B, R = 4, 4096, 200000
    ids = torch.randint(0, R, (T, B), device=dev)
    koff = [t * B for t in range(T + 1)]
    if which in ("all", "unique"):
        trial("unique_grouped", lambda: ops.unique_grouped(ids.reshape(-1), koff))
        trial("unique", lambda: ops.unique_device(ids[0]))
    if which in ("all", "bag"):
        seg = torch.arange(B, dtype=torch.int32, device=dev)
        trial("bag_offsets", lambda: ops.bag_offsets(seg, B))
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("dbg%d" % t, 128, 0.0, capacity=R + (1 << 19), device=dev)
        ev.insert_synthetic(0, R, seed=t)
        evs.append(ev)
    torch.cuda.synchronize()
    if which in ("all", "resolve"):
        u, idx, _, U = ops.unique_device(ids[0])
        trial("resolve", lambda: evs[0].resolve(u, n_dev=U))
    if which in ("all", "multi"):
        from deeprec_amd.embedding_ops import SparseTensor
        ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64,
                                                                    device=dev)], 1)
        sps = [SparseTensor(ind, ids[t], (B, 1)) for t in range(T)]
        with torch.no_grad():
            trial("multi", lambda: dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum"))
    if which == "uniq_check":
        static = ids.clone()
        datas = [torch.randint(0, R, (T, B), device=dev) for _ in range(4)]
        res = {}

        def fn():
            res["o"] = ops.unique_grouped(static.reshape(-1), koff)

        fn()
        static.copy_(datas[1])
        fn()
        torch.cuda.synchronize()
        static.copy_(ids)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        out = res["o"]
        for r in range(4):
            static.copy_(datas[r])
            torch.cuda.synchronize()
            log("uniq_check copied", r)
            g.replay()
            torch.cuda.synchronize()
            y, idx, _, U = out
            ey, eidx, _, eU = ops.unique_grouped(static.reshape(-1), koff)
            torch.cuda.synchronize()
            ok = torch.equal(U, eU) and torch.equal(idx, eidx)
            log("uniq_check replay", r, "match" if ok else "MISMATCH", U.tolist(), eU.tolist())
    if which.startswith("iso"):
        # extra eager call on other data, capture, replay twice with syncs
        static = ids.clone()
        other = torch.randint(0, R, (T, B), device=dev)
        U0 = None

        def run_unique():
            return ops.unique_grouped(static.reshape(-1), koff)

        u_keep = {}

        def run_resolve():
            y, idx, _, U = u_keep["u"]
            return evs[0].resolve(y[:B], n_dev=U[:1])

        from deeprec_amd.embedding_ops import _Feature, _prepare_group, _pool_all
        seg = torch.arange(B, dtype=torch.int32, device=dev)
        feats = [_Feature(evs[t], static[t], seg, B, None, "sum", None) for t in range(T)]

        def run_prep():
            _prepare_group(feats)

        def run_pool():
            return _pool_all(feats, 0)

        def run_both():
            _prepare_group(feats)
            return _pool_all(feats, 0)

        def run_temp():
            fs = [_Feature(evs[t], static[t], seg, B, None, "sum", None) for t in range(T)]
            _prepare_group(fs)
            return _pool_all(fs, 0)

        def run_temp_seg():
            fs = [_Feature(evs[t], static[t], seg.to(torch.int32).contiguous() + 0, B, None,
                           "sum", None) for t in range(T)]
            _prepare_group(fs)
            return _pool_all(fs, 0)

        fn = {"iso_unique": run_unique, "iso_resolve": run_resolve, "iso_prep": run_prep,
              "iso_pool": run_pool, "iso_both": run_both, "iso_temp": run_temp,
              "iso_tempseg": run_temp_seg}[which]
        _prepare_group(feats)
        u_keep["u"] = ops.unique_grouped(static.reshape(-1), koff)
        torch.cuda.synchronize()
        static.copy_(other)
        if which == "iso_resolve_fixed":
            pass
        fn()
        torch.cuda.synchronize()
        static.copy_(ids)
        u_keep["u"] = ops.unique_grouped(static.reshape(-1), koff)
        torch.cuda.synchronize()
        log(which, "eager ok")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for r in range(3):
            if os.environ.get("DBG_CHANGE") == "1":
                static.copy_(torch.randint(0, R, (T, B), device=dev))
                torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            log(which, "replay", r)
    if which == "multi2":
        from deeprec_amd.embedding_ops import SparseTensor
        ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64,
                                                                    device=dev)], 1)
        static = torch.empty_like(ids)
        static.copy_(ids)
        sps = [SparseTensor(ind, static[t], (B, 1)) for t in range(T)]
        batches = [torch.randint(0, R, (T, B), device=dev) for _ in range(4)]
        with torch.no_grad():
            f = lambda: dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
            f()
            torch.cuda.synchronize()
            if os.environ.get("DBG_EXTRA") == "1":
                static.copy_(batches[1])
                f()
                torch.cuda.synchronize()
                static.copy_(ids)
                log("extra eager step ok")
            if os.environ.get("DBG_STATUS") == "1":
                dr.status_check(dev)
                log("status ok")
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                f()
            g.replay()
            torch.cuda.synchronize()
            log("multi2 first replay ok")
            for i in range(6):
                static.copy_(batches[i % 4])
                torch.cuda.synchronize()
                log("copied", i)
                g.replay()
                torch.cuda.synchronize()
                log("replayed", i)
            for i in range(6):
                static.copy_(batches[i % 4])
                g.replay()
            torch.cuda.synchronize()
            log("multi2 back-to-back ok")
    log("done")


if __name__ == "__main__":
    main()
