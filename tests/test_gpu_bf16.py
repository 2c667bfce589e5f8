"""GPU: bf16 EmbeddingVariables (value_bits 16; BASELINE configs[4] "DCN-v2
CrossNet with bf16 embeddings").

The reference registers float and double EVs only (kv_variable_ops.cc:368-388),
so the bf16 EV is build-defined; its contract (include/deeprec_amd.h
dr_ev_config.value_bits, DESIGN.md "bf16 EVs") is restated by the oracle
(oracle.EV(bf16=True), oracle.bf16_round):
  * values are bf16; the fp32 default row is rounded to nearest even;
  * lookups pool the widened values in fp32 in the reference association
    order into an fp32 output (the reference casts bf16 embeddings to
    float32 before pooling, embedding_ops.py:606-607), or -- out_dtype
    bfloat16, the DCN-v2 input path -- round each bag once into a bf16
    output (a one-id bag is then a bitwise copy);
  * gradients are fp32; an apply computes the reference's fp32 formula on
    the widened value and rounds the updated value once; optimizer slots
    stay fp32.
Everything is compared bit for bit.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    deeprec_amd.set_validate(True)
    assert torch.cuda.is_available()
    return deeprec_amd


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


def bits(t):
    """bf16 tensor -> uint16 bit patterns (numpy)."""
    return t.detach().contiguous().view(torch.int16).cpu().numpy().view(np.uint16)


def f32(t):
    return t.detach().float().cpu().numpy()


def _ev_pair(dr, orc, name, D, init, rng=None, keys=None):
    ev = dr.EmbeddingVariable(name, D, init, value_dtype=torch.bfloat16)
    oev = orc.EV(D, init, bf16=True)
    if keys is not None:
        vals = orc.bf16_round(rng.standard_normal((keys.size, D)).astype(np.float32))
        ev.insert(T(keys), T(vals).to(torch.bfloat16))
        oev.insert(keys, vals)
    return ev, oev


def test_bf16_ev_default_insert_gather_export(dr, orc):
    rng = np.random.default_rng(1)
    D = 24
    ev, oev = _ev_pair(dr, orc, "bf_basic", D, 0.3, rng, np.arange(0, 200, 2, dtype=np.int64))
    assert ev.value_dtype == torch.bfloat16
    assert torch.equal(ev.default_value.float().cpu(),
                       torch.full((D,), orc.bf16_round(np.float32(0.3)).item()))
    keys = rng.integers(0, 300, 500).astype(np.int64)       # hits and insert-on-miss
    got = ev.sparse_read(T(keys))
    assert got.dtype == torch.bfloat16
    np.testing.assert_array_equal(f32(got), oev.gather(keys))
    k, v, _, _ = ev.export()
    ok, ov, _, _ = oev.export()
    np.testing.assert_array_equal(k.cpu().numpy(), ok)
    np.testing.assert_array_equal(f32(v), ov)
    assert int(ev.total_count()[0]) == oev.size()


def test_bf16_synthetic_rows(dr, orc):
    D = 64
    ev = dr.EmbeddingVariable("bf_synth", D, 0.0, value_dtype=torch.bfloat16)
    ev.insert_synthetic(100, 1000, seed=7, key_stride=3)
    keys = 100 + 3 * np.arange(1000, dtype=np.int64)
    got = ev.sparse_read(T(keys))
    want = orc.bf16_bits(orc.synth_rows(7, keys, D))
    np.testing.assert_array_equal(bits(got), want)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [64, 128])
def test_bf16_onehot_lookup(dr, orc, D, out_dtype):
    """Forward-only fused one-hot lookup (dr_ev_lookup_onehot_ex): the bf16
    rows widened into an fp32 output, or copied bitwise into a bf16 output;
    misses created with the (rounded) default."""
    rng = np.random.default_rng(D)
    F, B = 5, 700
    evs, oevs = [], []
    for f in range(F):
        e, o = _ev_pair(dr, orc, "bf_oh_%d_%d" % (D, f), D, 0.05 * (f + 1), rng,
                        np.arange(400, dtype=np.int64))
        evs.append(e)
        oevs.append(o)
    ids = rng.integers(0, 600, (F, B)).astype(np.int64)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    sps = [dr.SparseTensor(T(ind), T(ids[f]), (B, 1)) for f in range(F)]
    with torch.no_grad():
        out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum", out_dtype=out_dtype)
    assert out.dtype == out_dtype and tuple(out.shape) == (B, F * D)
    want = np.concatenate([oevs[f].gather(ids[f]) for f in range(F)], 1)
    np.testing.assert_array_equal(f32(out), want)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
@pytest.mark.parametrize("weighted,out_dtype", [(False, torch.float32), (True, torch.float32),
                                                (False, torch.bfloat16)])
def test_bf16_multihot_pool(dr, orc, comb, weighted, out_dtype):
    """Multi-hot bags (and weights, empty bags): fp32 pooling of the widened
    rows in the ALI order (DR_POOL_BF16 kernels), fp32 out or each bag
    rounded once to bf16.  Weighted mean / sqrtn of an empty bag is the
    reference's 0 / 0."""
    rng = np.random.default_rng(3 + int(weighted))
    B, D, H_ = 300, 32, 13
    ev, oev = _ev_pair(dr, orc, "bf_mh_%s_%d" % (comb, weighted), D, 0.1, rng,
                       np.arange(150, dtype=np.int64))
    lens = rng.integers(0, H_ + 1, B)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(n) for n in lens])
    ind = np.stack([rows, cols], 1).astype(np.int64)
    v = rng.integers(0, 200, rows.size).astype(np.int64)
    w = rng.uniform(0.5, 2.0, v.size).astype(np.float32) if weighted else None
    sp = dr.SparseTensor(T(ind), T(v), (B, H_))
    spw = dr.SparseTensor(T(ind), T(w), (B, H_)) if weighted else None
    with torch.no_grad():
        if out_dtype == torch.bfloat16:       # (the multi-feature API carries no weights)
            out = dr.embedding_lookup_sparse_multi([ev], [sp], combiner=comb, out_dtype=out_dtype)
        else:
            out = dr.embedding_lookup_sparse(ev, sp, sp_weights=spw, combiner=comb)
    assert out.dtype == out_dtype
    want = orc.embedding_lookup_sparse(oev, ind, v, B, weights=w, combiner=comb)
    if out_dtype == torch.bfloat16:
        want = orc.bf16_round(want)
    np.testing.assert_array_equal(f32(out), want)


@pytest.mark.parametrize("opt", ["sgd", "adagrad", "adam", "adam_async", "adagrad_decay"])
def test_bf16_training_steps_match_oracle(dr, orc, opt):
    """Three training steps of one-hot bf16 EVs (fused lookup recording rows
    -> row-grouped backward with fp32 gradients -> KV apply on bf16 values
    with fp32 slots) against the oracle's bf16 EV."""
    rng = np.random.default_rng(11)
    F, B, D = 3, 256, 64
    evs, oevs = [], []
    for f in range(F):
        e, o = _ev_pair(dr, orc, "bf_tr_%s_%d" % (opt, f), D, 0.02 * (f + 1), rng,
                        np.arange(100, dtype=np.int64))
        evs.append(e)
        oevs.append(o)
    lr = 0.05
    if opt == "sgd":
        o = dr.GradientDescentOptimizer(lr)
    elif opt == "adagrad":
        o = dr.AdagradOptimizer(lr, 0.1)
        oslots = [(oe.create_slot(1, np.float32(0.1)),) for oe in oevs]
    elif opt == "adam":
        o = dr.AdamOptimizer(lr)
        oslots = [(oe.create_slot(1, np.float32(0)), oe.create_slot(2, np.float32(0)))
                  for oe in oevs]
    elif opt == "adam_async":
        o = dr.AdamAsyncOptimizer(lr)
        oslots = [(oe.create_slot(1, np.float32(0)), oe.create_slot(2, np.float32(0)))
                  for oe in oevs]
    else:
        o = dr.AdagradDecayOptimizer(lr, initial_accumulator_value=0.1, accumulator_decay_step=2,
                                     accumulator_decay_rate=0.5)
        oslots = [(oe.create_slot(1, np.float32(0.1)), oe.create_slot(2, np.float32(0)))
                  for oe in oevs]
    b1p, b2p = np.float32(0.9), np.float32(0.999)
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    for step in range(3):
        ids = rng.integers(0, 160, (F, B)).astype(np.int64)
        sps = [dr.SparseTensor(T(ind), T(ids[f]), (B, 1)) for f in range(F)]
        out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum",
                                               out_dtype=torch.bfloat16 if step % 2 else None)
        want = np.concatenate([oevs[f].gather(ids[f]) for f in range(F)], 1)
        np.testing.assert_array_equal(f32(out), want)
        g = rng.standard_normal((B, F * D)).astype(np.float32)
        if out.dtype == torch.bfloat16:
            out.backward(T(g).to(torch.bfloat16))
            g16 = orc.bf16_round(g)                   # the bf16 output's gradient, widened
        else:
            out.backward(T(g))
            g16 = g
        gs = step + 1
        o.apply_gradients(evs, global_step=gs)
        for f in range(F):
            uids, idx = orc.unique(ids[f])
            gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g16[:, f * D:(f + 1) * D]),
                                                idx, np.arange(B, dtype=np.int32), uids.size,
                                                "sum")
            if opt == "sgd":
                oevs[f].apply_sgd(np.float32(lr), gu, uids, gs)
            elif opt == "adagrad":
                oevs[f].apply_adagrad(oslots[f][0], np.float32(lr), gu, uids, gs)
            elif opt == "adam":
                oevs[f].apply_adam(oslots[f][0], oslots[f][1], b1p, b2p, np.float32(lr),
                                   np.float32(0.9), np.float32(0.999), np.float32(1e-8), gu,
                                   uids, gs)
            elif opt == "adam_async":
                oevs[f].apply_adam_async(oslots[f][0], oslots[f][1], b1p, b2p, np.float32(lr),
                                         np.float32(0.9), np.float32(0.999), np.float32(1e-8),
                                         gu, uids, gs=gs)
            else:
                oevs[f].apply_adagrad_decay(oslots[f][0], oslots[f][1], np.float32(lr), 2,
                                            np.float32(0.5), np.float32(0.1), gu, uids, gs + 1)
        b1p, b2p = np.float32(b1p * np.float32(0.9)), np.float32(b2p * np.float32(0.999))
    for f in range(F):
        k, v, _, _ = evs[f].export()
        ok, ov, _, _ = oevs[f].export()
        np.testing.assert_array_equal(k.cpu().numpy(), ok)
        np.testing.assert_array_equal(f32(v), ov)


def test_bf16_ftrl_refused(dr):
    ev = dr.EmbeddingVariable("bf_ftrl", 16, 0.0, value_dtype=torch.bfloat16)
    B = 32
    ind = T(np.stack([np.arange(B), np.zeros(B, np.int64)], 1))
    out = dr.embedding_lookup_sparse_multi([ev], [dr.SparseTensor(ind, T(np.arange(B)), (B, 1))],
                                           combiner="sum")
    out.float().sum().backward()
    with pytest.raises(dr.DeepRecError):
        dr.FtrlOptimizer(0.1).apply_gradients([ev], global_step=1)
    ev.pending_grads = []


def test_bf16_xgmi_engine_matches_local(dr, orc):
    """The peer-write engine moves bf16 rows bitwise (world 1 on itself): its
    output equals the local lookup's, half the bytes of an fp32 row."""
    from deeprec_amd.sharded import XgmiShardedLookup
    rng = np.random.default_rng(5)
    F, B, D = 4, 512, 128
    evs, oevs = [], []
    for f in range(F):
        e, o = _ev_pair(dr, orc, "bf_xg_%d" % f, D, 0.25, rng, np.arange(300, dtype=np.int64))
        evs.append(e)
        oevs.append(o)
    eng = XgmiShardedLookup(evs, 1, 0, B, torch.device(DEV))
    for step, odt in enumerate((torch.bfloat16, None)):
        ids = rng.integers(0, 500, (F, B)).astype(np.int64)
        out = eng.forward(T(ids), out_dtype=odt)
        torch.cuda.synchronize()
        assert out.dtype == (odt or torch.float32)
        want = np.concatenate([oevs[f].gather(ids[f]) for f in range(F)], 1)
        np.testing.assert_array_equal(f32(out), want)
    eng.close()


@pytest.mark.parametrize("world", [1, 2])
def test_bf16_alltoall_engine_multihot(dr, orc, world):
    """All-to-all engine data path with bf16 rows (ranks as threads, in-memory
    exchange, test_gpu_sharded's harness): Unique -> route -> owner resolve +
    bf16 row pack -> bf16 rows exchanged -> requester pool (DR_POOL_BF16)."""
    import threading
    from deeprec_amd.sharded import ShardedLookup
    from test_gpu_sharded import _Exchange
    rng = np.random.default_rng(21 + world)
    F, B, D, KS = 3, 256, 32, 900
    allk = np.arange(KS, dtype=np.int64)
    vals = [orc.bf16_round(rng.standard_normal((KS, D)).astype(np.float32)) for _ in range(F)]
    ex = _Exchange(world)
    engines, batches = [], []
    for r in range(world):
        own = allk[allk % world == r]
        evs = []
        for f in range(F):
            ev = dr.EmbeddingVariable("bf_a2a_%d_%d_%d" % (world, r, f), D, 0.5,
                                      value_dtype=torch.bfloat16)
            ev.insert(T(own), T(vals[f][own]).to(torch.bfloat16))
            evs.append(ev)
        eng = ShardedLookup(evs, world, r, B, torch.device(DEV))
        eng._a2a = (lambda rr: (lambda out, inp, os_=None, is_=None:
                                ex.a2a(rr, out, inp, os_, is_)))(r)
        engines.append(eng)
        lens = rng.integers(0, 6, B)
        ids = rng.integers(0, KS + 100, (F, int(lens.sum()))).astype(np.int64)
        batches.append((ids, np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)))
    outs, errs = [None] * world, []

    def run(r):
        try:
            ids, off = batches[r]
            with torch.no_grad():
                o = engines[r].forward(T(ids), bag_offs=[T(off)] * F, combiner="mean",
                                       out_dtype=torch.bfloat16 if r == 0 else None)
            outs[r] = o
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
    for r in range(world):
        ids, off = batches[r]
        assert outs[r].dtype == (torch.bfloat16 if r == 0 else torch.float32)
        seg = np.repeat(np.arange(B), np.diff(off))
        ind = np.stack([seg, np.zeros_like(seg)], 1)
        for f in range(F):
            oev = orc.EV(D, 0.5, bf16=True)
            oev.insert(allk, vals[f])
            want = orc.embedding_lookup_sparse(oev, ind, ids[f], B, combiner="mean")
            if r == 0:
                want = orc.bf16_round(want)
            np.testing.assert_array_equal(f32(outs[r][:, f * D:(f + 1) * D]), want)
