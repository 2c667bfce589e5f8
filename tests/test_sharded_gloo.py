"""World-size-2 test of the row-sharded exchange protocol (sharded.py) on CPU.

The ShardedLookup engine (routing, counts / keys / rows all-to-all, requester
pooling) runs unchanged over torch.distributed gloo; its local steps go
through a backend object, here `OracleLocal`, built from the CPU oracle
(test infrastructure; the product backend is HipLocal, exercised on the GPU).
Each rank's pooled output must equal -- bit for bit -- a single-process
lookup of the same batch against one EV that holds every key
(embedding_ops.py:480-675 over embedding_var.h LookupOrCreate).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

T, D, B = 3, 8, 40
KEYSPACE = 200
DEFAULT = 0.25


def _row_values(t, keys):
    k = np.asarray(keys, np.float64)[:, None]
    c = np.arange(D)[None, :]
    return np.sin(0.37 * k + 1.3 * t + 0.11 * c).astype(np.float32)


class OracleLocal(object):
    """CPU restatement of HipLocal's four local steps."""

    def __init__(self, orc, evs):
        self.orc = orc
        self.evs = evs
        self.T = len(evs)
        self.dim = D
        self.filter = False

    def unique_grouped(self, vals, koff):
        v = vals.numpy()
        n = v.shape[0]
        y = np.zeros(n, np.int64)
        idx = np.zeros(n, np.int32)
        cnt = np.zeros(n, np.int32)
        U = []
        for t in range(self.T):
            u, i, c = self.orc.unique(v[koff[t]:koff[t + 1]], with_counts=True)
            y[koff[t]:koff[t] + u.shape[0]] = u
            idx[koff[t]:koff[t + 1]] = i
            cnt[koff[t]:koff[t] + u.shape[0]] = c
            U.append(u.shape[0])
        return (torch.from_numpy(y), torch.from_numpy(idx), torch.from_numpy(cnt),
                torch.tensor(U, dtype=torch.int64))

    def route(self, uniq, koff, U, world):
        """Stable (owner, feature) order (dr_route_by_owner's contract)."""
        u = uniq.numpy()
        n = u.shape[0]
        items = []
        for t in range(self.T):
            m = (koff[t + 1] - koff[t]) if U is None else int(U[t])
            for i in range(koff[t], koff[t] + m):
                items.append((int(u[i]) % world * self.T + t, i))
        items.sort(key=lambda x: x[0])            # Python sort is stable
        keys = np.zeros(n, np.int64)
        tags = np.zeros(n, np.int32)
        perm = np.zeros(n, np.int32)
        counts = np.zeros((world, self.T), np.int64)
        for j, (k, i) in enumerate(items):
            keys[j], tags[j], perm[j] = u[i], k % self.T, i
            counts[k // self.T, k % self.T] += 1
        return (torch.from_numpy(keys), torch.from_numpy(tags), torch.from_numpy(perm),
                torch.from_numpy(counts))

    def resolve_pack(self, keys, tags, n, per_table):
        out = np.zeros((n, D), np.float32)
        k, tg = keys.numpy(), tags.numpy()
        for t in range(self.T):
            m = tg == t
            assert int(m.sum()) == per_table[t]
            if m.any():
                out[m] = self.evs[t].gather(k[m])
        return torch.from_numpy(out)

    def pool_grad(self, grad, idx, koff, U, bag_offs, batch, combiner):
        g = grad.numpy()
        out = np.zeros((koff[-1], D), np.float32)
        for t in range(self.T):
            it = idx.numpy()[koff[t]:koff[t + 1]]
            if bag_offs is None:
                seg = np.arange(batch, dtype=np.int32)
            else:
                seg = np.repeat(np.arange(batch, dtype=np.int32), np.diff(bag_offs[t].numpy()))
            u = int(U[t])
            out[koff[t]:koff[t] + u] = self.orc.sparse_segment_reduce_grad(
                np.ascontiguousarray(g[:, t * D:(t + 1) * D]), it, seg, u, combiner)
        return torch.from_numpy(out)

    def pack(self, src, perm):
        return torch.from_numpy(np.ascontiguousarray(src.numpy()[perm.numpy().astype(np.int64)]))

    def pool(self, rows_recv, rowsel, idx, koff, bag_offs, batch, combiner):
        rr, rs = rows_recv.numpy(), rowsel.numpy()
        out = np.zeros((batch, self.T * D), np.float32)
        for t in range(self.T):
            if idx is None:                        # direct one-hot: bag b = nnz b
                rows = rr[rs[koff[t]:koff[t + 1]]]
                seg = np.arange(batch, dtype=np.int32)
                pooled = self.orc.sparse_segment_reduce(rows, np.arange(batch, dtype=np.int32),
                                                        seg, combiner, num_segments=batch)
            else:
                it = idx.numpy()[koff[t]:koff[t + 1]]
                U = int(it.max()) + 1
                emb = rr[rs[koff[t]:koff[t] + U]]
                off = (np.arange(batch + 1) if bag_offs is None else bag_offs[t].numpy())
                seg = np.repeat(np.arange(batch, dtype=np.int32), np.diff(off))
                pooled = self.orc.sparse_segment_reduce(emb, it, seg, combiner,
                                                        num_segments=batch)
            out[:, t * D:(t + 1) * D] = pooled
        return torch.from_numpy(out)


def _batches(rank, onehot):
    rng = np.random.default_rng(100 + rank)
    ids, offs = [], []
    for t in range(T):
        if onehot:
            lens = np.ones(B, np.int64)
        else:
            lens = rng.integers(0, 4, B)
            lens[0] = 0                              # an empty bag
        v = rng.integers(0, KEYSPACE, int(lens.sum())).astype(np.int64)
        v[:3] = 7                                    # duplicates across the batch
        ids.append(v)
        offs.append(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32))
    return ids, offs


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                        "deeprec-1_amd"))
        from oracle import oracle as orc
        from deeprec_amd.sharded import ShardedLookup
        # rank's shard: keys k % world == rank, pre-populated for half the keyspace
        own = np.arange(rank, KEYSPACE // 2, world, dtype=np.int64)
        sh_evs = []
        for t in range(T):
            ev = orc.EV(D, DEFAULT)
            ev.insert(own, _row_values(t, own))
            sh_evs.append(ev)
        be = OracleLocal(orc, sh_evs)
        eng = ShardedLookup(None, world, rank, B, torch.device("cpu"), backend=be)
        for onehot in (True, False):
            ids, offs = _batches(rank, onehot)
            # one reference EV per table holding every key (pre-populated half)
            allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
            for combiner in (("sum",) if onehot else ("sum", "mean", "sqrtn")):
                nnz = ids[0].shape[0]
                if not onehot and any(v.shape[0] != nnz for v in ids):
                    # ShardedLookup takes [T, nnz]: pad tables to equal nnz by
                    # giving every table table-0's bag structure
                    ids = [ids[0] for _ in range(T)]
                    offs = [offs[0] for _ in range(T)]
                    nnz = ids[0].shape[0]
                idm = torch.from_numpy(np.stack(ids))
                bo = None if onehot else [torch.from_numpy(o) for o in offs]
                out = eng.forward(idm, bag_offs=bo, combiner=combiner).numpy()
                assert eng.last_stats["direct"] == onehot
                for t in range(T):
                    ref_ev = orc.EV(D, DEFAULT)
                    ref_ev.insert(allk, _row_values(t, allk))
                    seg = np.repeat(np.arange(B), np.diff(offs[t]))
                    ind = np.stack([seg, np.zeros_like(seg)], 1)
                    ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[t], B, combiner=combiner)
                    np.testing.assert_array_equal(out[:, t * D:(t + 1) * D], ref)
        # backward: the owner receives, per feature, the rank-order
        # concatenation of every rank's (unique ids it owns, partial grads)
        for onehot in (True, False):
            for combiner in (("sum",) if onehot else ("sum", "mean")):
                allb = [_batches(p, onehot) for p in range(world)]
                if not onehot:
                    allb = [([b[0][0]] * T, [b[1][0]] * T) for b in allb]
                grads = [np.random.default_rng(300 + p).standard_normal((B, T * D))
                         .astype(np.float32) for p in range(world)]
                ids, offs = allb[rank]
                bo = None if onehot else [torch.from_numpy(o) for o in offs]
                eng.forward(torch.from_numpy(np.stack(ids)), bag_offs=bo, combiner=combiner,
                            need_grad=True)
                got = eng.backward(torch.from_numpy(grads[rank]))
                for t in range(T):
                    ek, ev_ = [], []
                    for p in range(world):
                        pid, poff = allb[p]
                        u, idx = orc.unique(pid[t])
                        seg = np.repeat(np.arange(B, dtype=np.int32), np.diff(poff[t]))
                        gu = orc.sparse_segment_reduce_grad(
                            np.ascontiguousarray(grads[p][:, t * D:(t + 1) * D]), idx, seg,
                            u.shape[0], combiner)
                        m = u % world == rank
                        ek.append(u[m])
                        ev_.append(gu[m])
                    np.testing.assert_array_equal(got[t][0].numpy(), np.concatenate(ek))
                    np.testing.assert_array_equal(got[t][1].numpy(), np.concatenate(ev_))
        # every key looked up anywhere is now owned by exactly its owner shard
        for t in range(T):
            keys = sh_evs[t].export()[0]
            assert np.all(keys % world == rank)
        open(os.path.join(outdir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [1, 2])
def test_sharded_exchange_gloo(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            assert os.path.exists(os.path.join(d, "ok%d" % r))


class _FakeEV(object):
    """What XgmiShardedLookup reads from an EV before its buffers exist."""
    filter_freq = 0
    dim = D
    value_dtype = torch.float32

    def __init__(self):
        import ctypes
        self.handle = ctypes.c_void_p(0)


class _CpuBuffers(object):
    cap = T * B

    def __init__(self, *a, **k):
        self.t = [torch.zeros(4) for _ in range(5)]

    def tensors(self):
        return self.t


class _ExportOk(object):
    @staticmethod
    def dr_ipc_export(p, h, off):
        return 0


def _setup_fail_worker(rank, world, port, outdir):
    """Rank 1's buffer allocation fails, rank 0's export succeeds: both must
    leave the handle exchange and raise the same error (before: rank 1 raised
    ahead of the all-gather rank 0 waited in -- a hang)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                        "deeprec-1_amd"))
        from deeprec_amd import sharded

        def failing(*a, **k):
            raise MemoryError("injected allocation failure")
        sharded.XgmiBuffers = failing if rank == 1 else _CpuBuffers
        sharded.lib = lambda: _ExportOk
        with pytest.raises(RuntimeError) as ei:
            sharded.XgmiShardedLookup([_FakeEV() for _ in range(T)], world, rank, B,
                                      torch.device("cpu"))
        msg = str(ei.value)
        assert "xgmi IPC setup failed" in msg and "rank 1" in msg and "injected" in msg
        assert "rank 0" not in msg
        open(os.path.join(outdir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


def test_xgmi_setup_failure_is_collective():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_setup_fail_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        for r in range(2):
            assert os.path.exists(os.path.join(d, "ok%d" % r))


def _hybrid_worker(rank, world, port, outdir):
    """HybridShardedLookup over gloo: features 0 and 2 replicated (every rank
    holds the whole table, looked up locally), feature 1 row-sharded through
    ShardedLookup (oracle backend).  Both output blocks equal the
    single-process lookup of every feature bit for bit."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                        "deeprec-1_amd"))
        from oracle import oracle as orc
        from deeprec_amd.sharded import HybridShardedLookup, ShardedLookup, hybrid_split
        cards = [30, KEYSPACE, 12]                 # features 0, 2 small; 1 large
        rep, shard = hybrid_split(cards, 40)
        assert rep == [0, 2] and shard == [1]
        allk = [np.arange(c, dtype=np.int64) for c in cards]
        full = []
        for t in range(3):
            ev = orc.EV(D, DEFAULT)
            ev.insert(allk[t][:cards[t] // 2], _row_values(t, allk[t][:cards[t] // 2]))
            full.append(ev)
        own = allk[1][:cards[1] // 2]
        own = own[own % world == rank]
        sev = orc.EV(D, DEFAULT)
        sev.insert(own, _row_values(1, own))
        be = OracleLocal(orc, [sev])
        eng = ShardedLookup(None, world, rank, B, torch.device("cpu"), backend=be)
        rep_evs = [full[t] for t in rep]

        def local_lookup(ids_rep):
            cols = []
            for j in range(len(rep)):
                ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
                cols.append(orc.embedding_lookup_sparse(rep_evs[j], ind, ids_rep[j].numpy(), B,
                                                        combiner="sum"))
            return torch.from_numpy(np.concatenate(cols, 1))

        hyb = HybridShardedLookup(local_lookup, eng, device=None)
        rng = np.random.default_rng(500 + rank)
        for step in range(2):
            ids = np.stack([rng.integers(0, c, B) for c in cards]).astype(np.int64)
            out_r, out_s = hyb.forward(torch.from_numpy(ids[rep]), torch.from_numpy(ids[shard]))
            ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
            for j, t in enumerate(rep):
                ref_ev = orc.EV(D, DEFAULT)
                ref_ev.insert(allk[t][:cards[t] // 2], _row_values(t, allk[t][:cards[t] // 2]))
                ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[t], B, combiner="sum")
                np.testing.assert_array_equal(out_r[:, j * D:(j + 1) * D].numpy(), ref)
            for j, t in enumerate(shard):
                ref_ev = orc.EV(D, DEFAULT)
                ref_ev.insert(allk[t][:cards[t] // 2], _row_values(t, allk[t][:cards[t] // 2]))
                ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[t], B, combiner="sum")
                np.testing.assert_array_equal(out_s[:, j * D:(j + 1) * D].numpy(), ref)
        open(os.path.join(outdir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_hybrid_placement_gloo(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_hybrid_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            assert os.path.exists(os.path.join(d, "ok%d" % r))


class _TinyDense(torch.nn.Module):
    """A dense-only stand-in for the model side of train_step_sharded (no
    EVs: the sharded embedding half is the GPU test
    tests/test_gpu_dlrm_sharded.py)."""

    def __init__(self):
        super().__init__()
        self.evs = []
        self.l1 = torch.nn.Linear(13, 8)
        self.l2 = torch.nn.Linear(8, 1)

    def forward(self, dense, ids):
        return torch.sigmoid(self.l2(torch.relu(self.l1(dense)))).squeeze(1)


class _NoKv(object):
    def apply_gradients(self, evs, global_step=None):
        assert not evs


def _dp_batch():
    g = torch.Generator().manual_seed(5)
    return torch.randn(4 * 32, 13, generator=g), (torch.rand(4 * 32, generator=g) > 0.5).float()


def _dp_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deeprec-1_amd"))
    from deeprec_amd import modelzoo as mz
    torch.manual_seed(0)
    model = _TinyDense()
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    dense, lab = _dp_batch()
    n = dense.shape[0] // world
    for _ in range(3):
        mz.train_step_sharded(model, dense[rank * n:(rank + 1) * n], None,
                              lab[rank * n:(rank + 1) * n], opt, _NoKv(), world)
    torch.save({k: v.clone() for k, v in model.state_dict().items()},
               os.path.join(outdir, "dp%d.pt" % rank))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_data_parallel_dense_step_gloo(world):
    """train_step_sharded's dense half (loss / world, gradient all-reduce,
    identical optimizer step on every rank) over gloo equals one process
    training on the whole global batch (fp32 summation order aside)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deeprec-1_amd"))
    from deeprec_amd import modelzoo as mz
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        got = [torch.load(os.path.join(d, "dp%d.pt" % r), weights_only=True) for r in range(world)]
    torch.manual_seed(0)
    ref = _TinyDense()
    opt = torch.optim.SGD(ref.parameters(), lr=0.5)
    dense, lab = _dp_batch()
    for _ in range(3):
        mz.train_step(ref, dense, None, lab, opt, _NoKv())
    for r in range(world):
        for k, v in ref.state_dict().items():
            assert torch.equal(got[r][k], got[0][k]), (r, k)        # replicas stay identical
            assert (got[r][k] - v).abs().max().item() <= 1e-6 * (v.abs().max().item() + 1), k


class _FakeEv(object):
    def __init__(self, dim):
        self.dim = dim
        self.device = torch.device("cpu")
        self.pending_grads = []


def _repl_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deeprec-1_amd"))
    from deeprec_amd.kv_variable_ops import IndexedSlices
    from deeprec_amd.sharded import sync_replicated_grads
    evs = [_FakeEv(4), _FakeEv(4)]
    g = torch.Generator().manual_seed(rank)
    # EV 0: two slices, the second with a device-count prefix; EV 1: rank 1 has none
    n0 = 3 + rank
    evs[0].pending_grads.append(IndexedSlices(torch.randn(n0, 4, generator=g),
                                              torch.arange(n0) * (rank + 1)))
    evs[0].pending_grads.append(IndexedSlices(torch.randn(5, 4, generator=g),
                                              torch.arange(5) + 100, num_valid=torch.tensor([2])))
    if rank != 1:
        evs[1].pending_grads.append(IndexedSlices(torch.randn(2, 4, generator=g),
                                                  torch.tensor([7, 7])))
    mine = [[(s.indices[:int(s.num_valid[0])] if s.num_valid is not None else s.indices,
              s.values[:int(s.num_valid[0])] if s.num_valid is not None else s.values)
             for s in ev.pending_grads] for ev in evs]
    sync_replicated_grads(evs)
    out = [[(s.indices, s.values) for s in ev.pending_grads] for ev in evs]
    torch.save({"mine": mine, "out": out}, os.path.join(outdir, "r%d.pt" % rank))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sync_replicated_grads_gloo(world):
    """sharded.sync_replicated_grads: every rank ends with the same slice per
    EV, the rank-order concatenation of every rank's pending slices (device
    counts honoured, empty contributions skipped)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_repl_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=True) for r in range(world)]
    for e in range(2):
        want_k = torch.cat([k for r in range(world) for k, _ in res[r]["mine"][e]] or
                           [torch.empty(0, dtype=torch.int64)])
        want_v = torch.cat([v for r in range(world) for _, v in res[r]["mine"][e]] or
                           [torch.empty(0, 4)])
        for r in range(world):
            out = res[r]["out"][e]
            assert len(out) == (1 if want_k.numel() else 0)
            if out:
                assert torch.equal(out[0][0], want_k) and torch.equal(out[0][1], want_v)


def _unused_param_worker(rank, world, port, outdir):
    import datetime
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deeprec-1_amd"))
    from deeprec_amd import modelzoo as mz
    a = torch.nn.Parameter(torch.ones(3))
    b = torch.nn.Parameter(torch.ones(5))
    loss = (a * (rank + 1)).sum()
    if rank == 0:                       # b gets a gradient on rank 0 only
        loss = loss + (b * 2.0).sum()
    loss.backward()
    mz.allreduce_dense_grads([a, b])
    torch.save({"a": a.grad.clone(), "b": b.grad.clone()}, os.path.join(outdir, "u%d.pt" % rank))
    dist.destroy_process_group()


def test_allreduce_dense_grads_param_unused_on_one_rank():
    """A parameter without a gradient on one rank (unused by its batch after
    zero_grad(set_to_none=True)) reduces as zeros there: every rank reduces
    buckets of the same size and ends with the same summed gradients."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_unused_param_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        got = [torch.load(os.path.join(d, "u%d.pt" % r), weights_only=True) for r in range(world)]
    for g in got:
        assert torch.equal(g["a"], torch.full((3,), 3.0))
        assert torch.equal(g["b"], torch.full((5,), 2.0))
