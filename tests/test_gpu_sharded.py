"""Row-sharded engine with the HIP backend (HipLocal) on one GPU.

World sizes 1 and 2 are emulated inside one process: every rank is a thread
with its own ShardedLookup and its own EV shards, and the all-to-all is an
in-memory exchange between the threads (same device, same stream order), so
routing, tagged owner resolve, row pack and requester pooling all run as
HIP kernels through the C ABI.  The RCCL transport itself is not under test
here (the driver's multi-GPU run exercises it); the CPU gloo test covers the
protocol over a real process group.  Outputs must equal the single-process
oracle bit for bit.
"""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
T, D, B = 4, 64, 512
KEYSPACE = 3000
DEFAULT = 0.5


def _vals(t, keys):
    k = np.asarray(keys, np.float64)[:, None]
    return np.cos(0.013 * k + 0.7 * t + 0.05 * np.arange(D)[None, :]).astype(np.float32)


class _Exchange(object):
    """all_to_all_single between threads of one process."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.box = [None] * world

    def a2a(self, rank, out, inp, out_splits, in_splits):
        W = self.world
        if in_splits is None:
            in_splits = [inp.shape[0] // W] * W
        if out_splits is None:
            out_splits = [out.shape[0] // W] * W
        self.box[rank] = list(torch.split(inp, list(in_splits)))
        self.bar.wait()
        pieces = [self.box[p][rank] for p in range(W)]
        assert [x.shape[0] for x in pieces] == list(out_splits)
        if out.shape[0]:
            torch.cat(pieces, out=out)
        self.bar.wait()
        return out


def _run_world(world, onehot, combiner):
    import deeprec_amd as dr
    from oracle import oracle as orc
    from deeprec_amd.sharded import ShardedLookup
    dr.load()
    ex = _Exchange(world)
    engines, batches = [], []
    rng = np.random.default_rng(5 + world)
    for r in range(world):
        evs = []
        own = np.arange(r, KEYSPACE // 2, world, dtype=np.int64)
        for t in range(T):
            ev = dr.EmbeddingVariable("sh%d_%d_%d_%d" % (world, int(onehot), r, t), D, DEFAULT,
                                      device=DEV)
            ev.insert(torch.as_tensor(own, device=DEV), torch.as_tensor(_vals(t, own), device=DEV))
            evs.append(ev)
        eng = ShardedLookup(evs, world, r, B, torch.device(DEV))
        eng._a2a = (lambda rr: (lambda out, inp, os_=None, is_=None:
                                ex.a2a(rr, out, inp, os_, is_)))(r)
        engines.append(eng)
        if onehot:
            lens = np.ones(B, np.int64)
        else:
            lens = rng.integers(0, 5, B)
            lens[3] = 0
        nnz = int(lens.sum())
        ids = rng.integers(0, KEYSPACE, (T, nnz)).astype(np.int64)
        ids[:, :4] = 11                       # duplicates inside the batch
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        batches.append((ids, off))
    outs = [None] * world
    errs = []

    def run(r):
        try:
            ids, off = batches[r]
            bo = None if onehot else [torch.as_tensor(off, device=DEV)] * T
            with torch.no_grad():
                outs[r] = engines[r].forward(torch.as_tensor(ids, device=DEV), bag_offs=bo,
                                             combiner=combiner).cpu().numpy()
        except Exception as e:  # surfaced below
            errs.append(e)
            ex.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    if errs:
        raise errs[0]
    dr.status_check()
    allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    for r in range(world):
        ids, off = batches[r]
        assert engines[r].last_stats["direct"] == onehot
        seg = np.repeat(np.arange(B), np.diff(off))
        ind = np.stack([seg, np.zeros_like(seg)], 1)
        for t in range(T):
            ref_ev = orc.EV(D, DEFAULT)
            ref_ev.insert(allk, _vals(t, allk))
            ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[t], B, combiner=combiner)
            np.testing.assert_array_equal(outs[r][:, t * D:(t + 1) * D], ref)
    # each shard holds only its own keys
    for r in range(world):
        for ev in engines[r].evs:
            k = ev.export()[0].cpu().numpy()
            assert np.all(k % world == r)


@pytest.mark.parametrize("world", [1, 2])
def test_sharded_onehot_direct(world):
    _run_world(world, True, "sum")


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("combiner", ["sum", "mean"])
def test_sharded_multihot_unique(world, combiner):
    _run_world(world, False, combiner)


# ---------------------------------------------------------------------------
# Peer-write engine (dr_xgmi_route / dr_xgmi_serve), ranks as threads sharing
# one GPU: "peer" buffers are plain same-device allocations here (the IPC
# mapping is exercised by tools/xgmi_ipc_check.py as separate processes).
# ---------------------------------------------------------------------------
def _run_xgmi(world, steps=2):
    import deeprec_amd as dr
    from oracle import oracle as orc
    from deeprec_amd.sharded import XgmiBuffers, XgmiShardedLookup
    dr.load()
    rng = np.random.default_rng(17 + world)
    evs_all, bufs = [], []
    for r in range(world):
        own = np.arange(r, KEYSPACE // 2, world, dtype=np.int64)
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("xg%d_%d_%d" % (world, r, t), D, DEFAULT, device=DEV)
            ev.insert(torch.as_tensor(own, device=DEV), torch.as_tensor(_vals(t, own), device=DEV))
            evs.append(ev)
        evs_all.append(evs)
        bufs.append(XgmiBuffers(world, T, B, D, DEV))
    bar = threading.Barrier(world)
    engines = [XgmiShardedLookup(evs_all[r], world, r, B, torch.device(DEV), peer_buffers=bufs,
                                 barrier=bar.wait, buffers=bufs[r]) for r in range(world)]
    allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    for step in range(steps):
        ids = [rng.integers(0, KEYSPACE, (T, B)).astype(np.int64) for _ in range(world)]
        for r in range(world):
            ids[r][:, :5] = 13 + step                 # duplicates across ranks and rows
        outs = [None] * world
        errs = []

        def run(r):
            try:
                o = engines[r].forward(torch.as_tensor(ids[r], device=DEV))
                bar.wait()                           # every owner has written every output
                outs[r] = o.cpu().numpy()
            except Exception as e:
                errs.append(e)
                bar.abort()

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        if errs:
            raise errs[0]
        dr.status_check()
        for r in range(world):
            for t in range(T):
                ref_ev = orc.EV(D, DEFAULT)
                ref_ev.insert(allk, _vals(t, allk))
                ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[r][t], B, combiner="sum")
                np.testing.assert_array_equal(outs[r][:, t * D:(t + 1) * D], ref)
        # backward: every owner pulls its keys' gradient rows from the
        # requesters, in (table, source rank, batch row) order -- exact copies
        grads = [rng.standard_normal((B, T * D)).astype(np.float32) for _ in range(world)]
        pulled = [None] * world

        def run_bwd(r):
            try:
                got = engines[r].backward(torch.as_tensor(grads[r], device=DEV))
                pulled[r] = []
                for k, v, n in got:                  # fixed regions + device counts
                    m = int(n.item())
                    pulled[r].append((k[:m].cpu().numpy(), v[:m].cpu().numpy()))
            except Exception as e:
                errs.append(e)
                bar.abort()

        th = [threading.Thread(target=run_bwd, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        if errs:
            raise errs[0]
        for r in range(world):
            for t in range(T):
                wk, wg = [], []
                for s in range(world):
                    sel = np.nonzero(ids[s][t] % world == r)[0]
                    wk.append(ids[s][t][sel])
                    wg.append(grads[s][sel, t * D:(t + 1) * D])
                k, v = pulled[r][t]
                np.testing.assert_array_equal(k, np.concatenate(wk))
                np.testing.assert_array_equal(v, np.concatenate(wg).reshape(-1, D))
                sl = evs_all[r][t].pending_grads.pop()
                assert int(sl.num_valid.item()) == k.shape[0]
                evs_all[r][t].pending_grads.clear()
    for r in range(world):
        for ev in evs_all[r]:
            k = ev.export()[0].cpu().numpy()
            assert np.all(k % world == r)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_xgmi_peer_write_engine(world):
    _run_xgmi(world)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_xgmi_dedup_engine(world):
    """Peer-write engine with per-destination dedup (dr_xgmi_route_ex over
    the grouped Unique, local expansion): Zipf-skewed ids with hot keys
    shared across ranks.  Forward bit-exact vs the oracle (and hence vs the
    plain engine); backward: each owner pulls, per table and source rank,
    the source's unique keys in first-occurrence order with their summed
    gradient (SparseSegmentSumGrad over ascending positions) -- each
    worker's IndexedSlices, concatenated in rank order."""
    import deeprec_amd as dr
    from oracle import oracle as orc
    from deeprec_amd.sharded import XgmiBuffers, XgmiShardedLookup
    dr.load()
    rng = np.random.default_rng(71 + world)
    evs_all, bufs = [], []
    for r in range(world):
        own = np.arange(r, KEYSPACE // 2, world, dtype=np.int64)
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("xgd%d_%d_%d" % (world, r, t), D, DEFAULT, device=DEV)
            ev.insert(torch.as_tensor(own, device=DEV), torch.as_tensor(_vals(t, own), device=DEV))
            evs.append(ev)
        evs_all.append(evs)
        bufs.append(XgmiBuffers(world, T, B, D, DEV))
    bar = threading.Barrier(world)
    engines = [XgmiShardedLookup(evs_all[r], world, r, B, torch.device(DEV), peer_buffers=bufs,
                                 barrier=bar.wait, buffers=bufs[r], dedup=True)
               for r in range(world)]
    allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    for step in range(2):
        ids = [((rng.zipf(1.2, size=(T, B)) - 1) % KEYSPACE).astype(np.int64)
               for _ in range(world)]
        grads = [rng.standard_normal((B, T * D)).astype(np.float32) for _ in range(world)]
        outs, pulled, errs = [None] * world, [None] * world, []

        def run(r):
            try:
                o = engines[r].forward(torch.as_tensor(ids[r], device=DEV))
                outs[r] = o.cpu().numpy()
                got = engines[r].backward(torch.as_tensor(grads[r], device=DEV))
                pulled[r] = []
                for k, v, n in got:
                    m = int(n.item())
                    pulled[r].append((k[:m].cpu().numpy(), v[:m].cpu().numpy()))
            except Exception as e:
                errs.append(e)
                bar.abort()

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        if errs:
            raise errs[0]
        dr.status_check()
        for r in range(world):
            for t in range(T):
                ref_ev = orc.EV(D, DEFAULT)
                ref_ev.insert(allk, _vals(t, allk))
                ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[r][t], B, combiner="sum")
                np.testing.assert_array_equal(outs[r][:, t * D:(t + 1) * D], ref)
                wk, wg = [], []
                for src in range(world):
                    uids, idx = orc.unique(ids[src][t])
                    gu = orc.sparse_segment_reduce_grad(
                        np.ascontiguousarray(grads[src][:, t * D:(t + 1) * D]), idx,
                        np.arange(B, dtype=np.int32), uids.size, "sum")
                    sel = uids % world == r
                    wk.append(uids[sel])
                    wg.append(gu[sel])
                k, v = pulled[r][t]
                np.testing.assert_array_equal(k, np.concatenate(wk))
                np.testing.assert_array_equal(v, np.concatenate(wg).reshape(-1, D))
                evs_all[r][t].pending_grads.clear()


@pytest.mark.parametrize("world,combiner", [(1, "sum"), (2, "mean"), (3, "sqrtn"), (2, "sum")])
def test_xgmi_multihot_engine(world, combiner):
    """Multi-hot bags on the peer-write engine (Unique -> route unique keys
    -> owners serve one row per unique key -> ALI-order pooling over the
    bags): bags of 0..4 Zipf-skewed ids, empty bags, per-table key capacity
    4 x the bag count.  Forward bit-exact vs the oracle's
    embedding_lookup_sparse; backward: each owner pulls, per table and
    source rank, the source's unique keys in first-occurrence order with
    their SparseSegment{Sum,Mean,SqrtN}Grad rows."""
    import deeprec_amd as dr
    from oracle import oracle as orc
    from deeprec_amd.sharded import XgmiBuffers, XgmiShardedLookup
    dr.load()
    rng = np.random.default_rng(97 + world)
    CAP = 4 * B
    evs_all, bufs = [], []
    for r in range(world):
        own = np.arange(r, KEYSPACE // 2, world, dtype=np.int64)
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("xgm%d_%s_%d_%d" % (world, combiner, r, t), D, DEFAULT,
                                      device=DEV)
            ev.insert(torch.as_tensor(own, device=DEV), torch.as_tensor(_vals(t, own), device=DEV))
            evs.append(ev)
        evs_all.append(evs)
        bufs.append(XgmiBuffers(world, T, CAP, D, DEV))
    bar = threading.Barrier(world)
    engines = [XgmiShardedLookup(evs_all[r], world, r, CAP, torch.device(DEV), peer_buffers=bufs,
                                 barrier=bar.wait, buffers=bufs[r]) for r in range(world)]
    allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    for step in range(2):
        lens = [rng.integers(0, 5, B) for _ in range(world)]
        for ln in lens:
            ln[3] = 0
        offs = [np.concatenate([[0], np.cumsum(ln)]).astype(np.int32) for ln in lens]
        ids = [((rng.zipf(1.3, size=(T, int(ln.sum()))) - 1) % KEYSPACE).astype(np.int64)
               for ln in lens]
        grads = [rng.standard_normal((B, T * D)).astype(np.float32) for _ in range(world)]
        outs, pulled, errs = [None] * world, [None] * world, []

        def run(r):
            try:
                bo = [torch.as_tensor(offs[r], device=DEV)] * T
                o = engines[r].forward(torch.as_tensor(ids[r], device=DEV), bag_offs=bo,
                                       combiner=combiner)
                outs[r] = o.cpu().numpy()
                got = engines[r].backward(torch.as_tensor(grads[r], device=DEV))
                pulled[r] = []
                for k, v, n in got:
                    m = int(n.item())
                    pulled[r].append((k[:m].cpu().numpy(), v[:m].cpu().numpy()))
            except Exception as e:
                errs.append(e)
                bar.abort()

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        if errs:
            raise errs[0]
        dr.status_check()
        for r in range(world):
            seg = np.repeat(np.arange(B), lens[r])
            ind = np.stack([seg, np.zeros_like(seg)], 1)
            for t in range(T):
                ref_ev = orc.EV(D, DEFAULT)
                ref_ev.insert(allk, _vals(t, allk))
                ref = orc.embedding_lookup_sparse(ref_ev, ind, ids[r][t], B, combiner=combiner)
                np.testing.assert_array_equal(outs[r][:, t * D:(t + 1) * D], ref)
                wk, wg, wl = [], [], []
                for src in range(world):
                    uids, idx = orc.unique(ids[src][t])
                    sseg = np.repeat(np.arange(B), lens[src]).astype(np.int32)
                    gu = orc.sparse_segment_reduce_grad(
                        np.ascontiguousarray(grads[src][:, t * D:(t + 1) * D]), idx, sseg,
                        uids.size, combiner)
                    sel = uids % world == r
                    wk.append(uids[sel])
                    wg.append(gu[sel])
                    # > 256 positions: ordered chunk partials (fp32 tolerance)
                    wl.append(np.bincount(idx, minlength=uids.size)[sel] > 256)
                k, v = pulled[r][t]
                np.testing.assert_array_equal(k, np.concatenate(wk))
                ref_g = np.concatenate(wg).reshape(-1, D)
                hot = np.concatenate(wl)
                np.testing.assert_array_equal(v[~hot], ref_g[~hot])
                for i in np.where(hot)[0]:
                    err = np.abs(v[i] - ref_g[i]).max()
                    assert err <= 1e-5 * np.abs(ref_g[i]).max(), (i, err)
                evs_all[r][t].pending_grads.clear()


@pytest.mark.parametrize("world", [1, 2])
def test_xgmi_serve_grows_small_tables(world):
    """Owners whose EVs start with room for 256 rows receive ~3x that many new
    keys over three steps: dr_xgmi_serve reserves before its insert-on-miss
    (ADVICE round 1), so nothing is served from a dead row, the status word
    stays clean and every key is stored exactly once."""
    import deeprec_amd as dr
    from deeprec_amd.sharded import XgmiBuffers, XgmiShardedLookup
    dr.load()
    evs_all = [[dr.EmbeddingVariable("xgrow%d_%d_%d" % (world, r, t), D, DEFAULT, device=DEV,
                                     capacity=256) for t in range(T)] for r in range(world)]
    bufs = [XgmiBuffers(world, T, B, D, DEV) for _ in range(world)]
    bar = threading.Barrier(world)
    engines = [XgmiShardedLookup(evs_all[r], world, r, B, torch.device(DEV), peer_buffers=bufs,
                                 barrier=bar.wait, buffers=bufs[r]) for r in range(world)]
    seen = [set() for _ in range(T)]
    for step in range(3):
        # distinct new keys every step, each rank's spread over every owner
        allk = np.random.default_rng(step).permutation(T * B * world).astype(np.int64)
        allk += step * T * B * world
        ids = [allk[r * T * B:(r + 1) * T * B].reshape(T, B) for r in range(world)]
        for r in range(world):
            for t in range(T):
                seen[t].update(ids[r][t].tolist())
        outs, errs = [None] * world, []

        def run(r):
            try:
                with torch.no_grad():
                    o = engines[r].forward(torch.as_tensor(ids[r], device=DEV))
                bar.wait()
                outs[r] = o.cpu().numpy()
            except Exception as e:
                errs.append(e)
                bar.abort()

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        if errs:
            raise errs[0]
        dr.status_check()
        for r in range(world):
            if not np.all(outs[r] == np.float32(DEFAULT)):
                ob = outs[r].reshape(B, T, D)
                badbt = np.argwhere(~(ob == np.float32(DEFAULT)).all(2))
                stored = []
                for t in range(T):
                    vals = [evs_all[o][t].export()[1].cpu().numpy() for o in range(world)]
                    stored.append(int(sum((v != np.float32(DEFAULT)).any(1).sum() for v in vals)))
                raise AssertionError(
                    "step %d rank %d: %d (bag, table) outputs differ, first %s (key %d, "
                    "values %s); stored rows != default per table: %s" % (
                        step, r, badbt.shape[0], badbt[:4].tolist(),
                        ids[r][badbt[0][1], badbt[0][0]],
                        ob[badbt[0][0], badbt[0][1], :6].tolist(), stored))
    for r in range(world):
        for t in range(T):
            k = evs_all[r][t].export()[0].cpu().numpy()
            want = np.array(sorted(x for x in seen[t] if x % world == r), np.int64)
            np.testing.assert_array_equal(np.sort(k), want)


# ---------------------------------------------------------------------------
# Sharded backward (ShardedLookup.backward): grad rows to the owners, then the
# KV optimizer on each shard.  Reference: one EV per feature holding every
# key, updated with the rank-order concatenation of each rank's (unique ids,
# partial grads) -- deduplicated (Adagrad, optimizer.py:68-83) or applied in
# order (SGD, gradient_descent.py:71-76).
# ---------------------------------------------------------------------------
def _run_sharded_train(world, onehot, opt_name, combiner):
    import deeprec_amd as dr
    from oracle import oracle as orc
    from deeprec_amd.sharded import ShardedLookup
    dr.load()
    ex = _Exchange(world)
    rng = np.random.default_rng(41 + world)
    lr = np.float32(0.3)
    engines, batches, grads = [], [], []
    for r in range(world):
        own = np.arange(r, KEYSPACE // 2, world, dtype=np.int64)
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("tr%d_%d_%s_%s_%d_%d" % (world, int(onehot), opt_name,
                                                              combiner, r, t), D, DEFAULT,
                                      device=DEV)
            ev.insert(torch.as_tensor(own, device=DEV), torch.as_tensor(_vals(t, own), device=DEV))
            evs.append(ev)
        eng = ShardedLookup(evs, world, r, B, torch.device(DEV))
        eng._a2a = (lambda rr: (lambda out, inp, os_=None, is_=None:
                                ex.a2a(rr, out, inp, os_, is_)))(r)
        engines.append(eng)
        lens = np.ones(B, np.int64) if onehot else rng.integers(0, 5, B)
        if not onehot:
            lens[3] = 0
        nnz = int(lens.sum())
        ids = rng.integers(0, KEYSPACE, (T, nnz)).astype(np.int64)
        ids[:, :4] = 11 + r % 2                  # duplicates inside and across ranks
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        batches.append((ids, off))
        grads.append(rng.standard_normal((B, T * D)).astype(np.float32))
    opts = [dr.GradientDescentOptimizer(lr) if opt_name == "sgd" else dr.AdagradOptimizer(lr, 0.1)
            for _ in range(world)]
    errs = []

    def run(r):
        try:
            ids, off = batches[r]
            bo = None if onehot else [torch.as_tensor(off, device=DEV)] * T
            engines[r].forward(torch.as_tensor(ids, device=DEV), bag_offs=bo, combiner=combiner,
                               need_grad=True)
            engines[r].backward(torch.as_tensor(grads[r], device=DEV))
            opts[r].apply_gradients(engines[r].evs, global_step=1)
        except Exception as e:
            errs.append(e)
            ex.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    if errs:
        raise errs[0]
    dr.status_check()
    allk = np.arange(0, KEYSPACE // 2, dtype=np.int64)
    for t in range(T):
        ref = orc.EV(D, DEFAULT)
        ref.insert(allk, _vals(t, allk))
        ks, gs = [], []
        for p in range(world):
            ids, off = batches[p]
            u, idx = orc.unique(ids[t])
            ref.gather(u)                                    # forward's insert-on-miss
            seg = np.repeat(np.arange(B, dtype=np.int32), np.diff(off))
            ks.append(u)
            gs.append(orc.sparse_segment_reduce_grad(
                np.ascontiguousarray(grads[p][:, t * D:(t + 1) * D]), idx, seg, u.shape[0],
                combiner))
        if opt_name == "sgd":
            for k, g in zip(ks, gs):                          # repeated ids in order
                ref.apply_sgd(lr, g, k, 1)
        else:
            acc = ref.create_slot(1, 0.1)
            k, g = np.concatenate(ks), np.concatenate(gs)
            u, pos = orc.unique(k)
            ref.apply_adagrad(acc, lr, orc.unsorted_segment_sum(g, pos, u.shape[0]), u, 1)
        rk, rv = ref.export()[:2]
        for r in range(world):
            k, v = [x.cpu().numpy() for x in engines[r].evs[t].export()[:2]]
            o = np.argsort(k)
            m = rk % world == r
            ro = np.argsort(rk[m])
            np.testing.assert_array_equal(k[o], rk[m][ro])
            np.testing.assert_array_equal(v[o], rv[m][ro])


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("opt_name", ["sgd", "adagrad"])
@pytest.mark.parametrize("onehot,combiner", [(True, "sum"), (False, "mean")])
def test_sharded_backward_apply(world, opt_name, onehot, combiner):
    _run_sharded_train(world, onehot, opt_name, combiner)
