"""KvSparseApplyAdamAsync (training_ali_ops.cc:1404-1575, both modes) and
KvSparseApplyAdagradDecay (:703-823) on the GPU against the oracle's
restatements (themselves pinned by the reference's KATs,
tests/test_oracle_async_decay.py): 5 steps over first-touch and repeated
keys, several dims (VEC = 1 and 4 kernels), decay crossings every 2 steps,
and the by-address gradients of a row-grouped lookup backward.  The apply
kernels evaluate the oracle's scalar formulas with separate fp32 roundings:
weights, slots and decay counts are bit-identical to the oracle's."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd as dr
    dr.load()
    dr.set_validate(True)
    return dr


@pytest.mark.parametrize("D", [1, 3, 16, 64])
@pytest.mark.parametrize("rmsprop", [False, True])
def test_adam_async_matches_oracle(dr, orc, D, rmsprop):
    rng = np.random.default_rng(D * 7 + rmsprop)
    lr, b1, b2, eps = 0.01, 0.9, 0.999, 1e-8
    ev = dr.EmbeddingVariable("aa_%d_%d" % (D, rmsprop), D, 0.25)
    oev = orc.EV(D, 0.25)
    om, ov = oev.create_slot(1, 0.0), oev.create_slot(2, 0.0)
    opt = dr.AdamAsyncOptimizer(lr, b1, b2, eps, apply_sparse_rmsprop=rmsprop)
    b1p, b2p = np.float32(b1), np.float32(b2)
    for step in range(5):
        ids = rng.choice(300, 80, replace=False).astype(np.int64)
        g = (rng.standard_normal((80, D)) * 0.2).astype(np.float32)
        ev.pending_grads.append(dr.IndexedSlices(T(g), T(ids)))
        opt.apply_gradients([ev], global_step=step)
        oev.apply_adam_async(om, ov, float(b1p), float(b2p), lr, b1, b2, eps, g, ids,
                             rmsprop=rmsprop, gs=step)
        b1p, b2p = np.float32(b1p * np.float32(b1)), np.float32(b2p * np.float32(b2))
    keys = np.arange(300, dtype=np.int64)
    np.testing.assert_array_equal(ev.sparse_read(T(keys)).cpu().numpy(), oev.gather(keys),
    )
    np.testing.assert_array_equal(ev.slot("AdamAsync", 0.0).sparse_read(T(keys)).cpu().numpy(),
                               om.gather(keys))
    np.testing.assert_array_equal(ev.slot("AdamAsync_1", 0.0).sparse_read(T(keys)).cpu().numpy(),
                               ov.gather(keys))
    if not rmsprop:
        p = opt._power(ev)
        assert p[0] == float(b1p) and p[1] == float(b2p)


@pytest.mark.parametrize("D", [1, 3, 16, 64])
def test_adagrad_decay_matches_oracle(dr, orc, D):
    rng = np.random.default_rng(D + 100)
    lr, init, dstep, rate = 0.3, 0.1, 2, 0.8
    ev = dr.EmbeddingVariable("ad_%d" % D, D, 0.5)
    oev = orc.EV(D, 0.5)
    oacc, opw = oev.create_slot(1, init), oev.create_slot(2, 0.0)
    opt = dr.AdagradDecayOptimizer(lr, initial_accumulator_value=init,
                                   accumulator_decay_step=dstep, accumulator_decay_rate=rate)
    for step in range(6):
        ids = rng.choice(120, 50, replace=False).astype(np.int64)
        g = (rng.standard_normal((50, D)) * (0.05 if step % 2 else 0.5)).astype(np.float32)
        ev.pending_grads.append(dr.IndexedSlices(T(g), T(ids)))
        opt.apply_gradients([ev], global_step=step)
        oev.apply_adagrad_decay(oacc, opw, lr, dstep, rate, init, g, ids, step + 1)
    keys = np.arange(120, dtype=np.int64)
    np.testing.assert_array_equal(ev.sparse_read(T(keys)).cpu().numpy(), oev.gather(keys),
    )
    np.testing.assert_array_equal(ev.slot("AdagradDecay", init).sparse_read(T(keys)).cpu().numpy(),
                               oacc.gather(keys))
    pw = ev.slot("AdagradDecay_1", 0.0).sparse_read(T(keys)).cpu().numpy()
    np.testing.assert_array_equal(pw, opw.gather(keys))
    assert pw[:, 0].max() >= 2.0            # rows decayed more than once


def test_adagrad_decay_needs_global_step(dr):
    ev = dr.EmbeddingVariable("ad_nogs", 4, 0.5)
    opt = dr.AdagradDecayOptimizer(0.1)
    ev.pending_grads.append(dr.IndexedSlices(T(np.ones((1, 4), np.float32)), T([3])))
    with pytest.raises(ValueError):
        opt.apply_gradients([ev])
    with pytest.raises(ValueError):
        dr.AdagradDecayOptimizer(0.1, accumulator_decay_step=0)


@pytest.mark.parametrize("name", ["adam_async", "rmsprop", "adagrad_decay"])
def test_by_address_grads_equal_value_grads(dr, name):
    """The lookup's row-grouped backward hands gradients by address; the
    apply through them equals the apply of the materialised values."""
    rng = np.random.default_rng(17)
    B, D = 256, 16
    keys = T(rng.integers(0, 500, B).astype(np.int64))
    ind = T(np.stack([np.arange(B), np.zeros(B, np.int64)], 1))
    up = T(rng.standard_normal((B, D)).astype(np.float32))
    outs = []
    for by_addr in (True, False):
        ev = dr.EmbeddingVariable("ba_%s_%d" % (name, by_addr), D, 0.1)
        mk = {"adam_async": lambda: dr.AdamAsyncOptimizer(0.01),
              "rmsprop": lambda: dr.AdamAsyncOptimizer(0.01, apply_sparse_rmsprop=True),
              "adagrad_decay": lambda: dr.AdagradDecayOptimizer(
                  0.1, accumulator_decay_step=1, accumulator_decay_rate=0.5)}[name]
        opt = mk()
        for step in range(3):
            out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(ind, keys, (B, 1)),
                                             combiner="sum")
            out.backward(up)
            if not by_addr:
                for sl in ev.pending_grads:
                    sl.values = sl.values.clone()     # materialise, drop the addresses
            opt.apply_gradients([ev], global_step=step)
        torch.cuda.synchronize()
        outs.append(ev.sparse_read(T(np.arange(500, dtype=np.int64))).cpu().numpy())
    np.testing.assert_array_equal(outs[0], outs[1])


def test_registered_ops_match_optimizers(dr, orc):
    """torch.ops.deeprec.kv_resource_sparse_apply_{adam_async,adagrad_decay}
    (the registered op layer) leave the EVs where the oracle does."""
    import deeprec_amd.torch_ops  # noqa: F401
    rng = np.random.default_rng(23)
    D = 8
    ids = rng.choice(100, 40, replace=False).astype(np.int64)
    g = (rng.standard_normal((40, D)) * 0.3).astype(np.float32)
    ev = dr.EmbeddingVariable("op_aa", D, 0.2)
    m, v = ev.slot("m", 0.0), ev.slot("v", 0.0)
    oev = orc.EV(D, 0.2)
    om, ov = oev.create_slot(1, 0.0), oev.create_slot(2, 0.0)
    bp = torch.tensor([0.9, 0.999], dtype=torch.float32, device=DEV)
    torch.ops.deeprec.kv_resource_sparse_apply_adam_async(
        ev.resource, m.resource, v.resource, bp, 0.01, 0.9, 0.999, 1e-8, T(g), T(ids), 3)
    oev.apply_adam_async(om, ov, 0.9, 0.999, 0.01, 0.9, 0.999, 1e-8, g, ids, gs=3)
    # the op advanced its beta power resources (N > 0)
    assert bp.cpu().tolist() == [float(np.float32(0.9) * np.float32(0.9)),
                                 float(np.float32(0.999) * np.float32(0.999))]
    np.testing.assert_array_equal(ev.sparse_read(T(ids)).cpu().numpy(), oev.gather(ids))
    ev2 = dr.EmbeddingVariable("op_ad", D, 0.2)
    acc, pw = ev2.slot("acc", 0.1), ev2.slot("pw", 0.0)
    oev2 = orc.EV(D, 0.2)
    oacc, opw = oev2.create_slot(1, 0.1), oev2.create_slot(2, 0.0)
    torch.ops.deeprec.kv_resource_sparse_apply_adagrad_decay(
        ev2.resource, acc.resource, pw.resource, 0.5, 2, 0.9, 0.1, 5, T(g), T(ids))
    oev2.apply_adagrad_decay(oacc, opw, 0.5, 2, 0.9, 0.1, g, ids, 5)
    np.testing.assert_array_equal(ev2.sparse_read(T(ids)).cpu().numpy(), oev2.gather(ids))
    np.testing.assert_array_equal(pw.sparse_read(T(ids)).cpu().numpy(), opw.gather(ids))


def test_adam_async_empty_gradient_keeps_powers(dr):
    """N == 0: the op does nothing, beta powers included (training_ali_ops.cc
    :1482 wraps the update and the power advance in `if (N > 0)`)."""
    ev = dr.EmbeddingVariable("aa_empty", 4, 0.5)
    opt = dr.AdamAsyncOptimizer(0.01)
    ev.pending_grads.append(dr.IndexedSlices(T(np.zeros((0, 4), np.float32)),
                                             T(np.zeros(0, np.int64))))
    opt.apply_gradients([ev], global_step=0)
    p = opt._power(ev)
    assert p[0] == float(np.float32(0.9)) and p[1] == float(np.float32(0.999))
    assert ev.sparse_read(T([1])).cpu().numpy().tolist() == [[0.5] * 4]
    # a dense table with an empty gradient keeps its powers too
    tab = dr.DenseTable(T(np.ones((5, 4), np.float32)))
    tab.pending_grads.append(dr.IndexedSlices(T(np.zeros((0, 4), np.float32)),
                                              T(np.zeros(0, np.int64))))
    opt.apply_gradients([tab], global_step=0)
    p = opt._power(tab)
    assert p[0] == float(np.float32(0.9)) and p[1] == float(np.float32(0.999))


def test_adam_async_device_count_guards_powers(dr, orc):
    """A fixed-capacity slice whose DEVICE count (num_valid, as the sharded
    and row-grouped backwards queue them) is 0 is the op's N == 0: no row
    moves and the beta powers stay (training_ali_ops.cc:1482).  A count of 2
    of 4 applies exactly the first two rows and advances the powers once --
    with no host read of the count (the apply can be graph-captured)."""
    D = 8
    ev = dr.EmbeddingVariable("aa_devcnt", D, 0.5)
    oev = orc.EV(D, 0.5)
    om, ov = oev.create_slot(1, 0.0), oev.create_slot(2, 0.0)
    opt = dr.AdamAsyncOptimizer(0.01)
    ids = np.array([3, 7, 11, 19], np.int64)
    g = (np.random.default_rng(5).standard_normal((4, D)) * 0.3).astype(np.float32)
    ev.pending_grads.append(dr.IndexedSlices(T(g), T(ids), num_valid=T([0], torch.int64),
                                             unique=True))
    opt.apply_gradients([ev], global_step=0)
    p = opt._power(ev)
    assert p[0] == float(np.float32(0.9)) and p[1] == float(np.float32(0.999))
    np.testing.assert_array_equal(ev.sparse_read(T(ids)).cpu().numpy(), np.full((4, D), 0.5,
                                                                               np.float32))
    ev2 = dr.EmbeddingVariable("aa_devcnt2", D, 0.5)
    opt2 = dr.AdamAsyncOptimizer(0.01)
    ev2.pending_grads.append(dr.IndexedSlices(T(g), T(ids), num_valid=T([2], torch.int64),
                                              unique=True))
    opt2._slots(ev2)                  # slot EVs allocate: created before the capture
    opt2._power_t(ev2)
    torch.cuda.synchronize()
    g_cap = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_cap):
        opt2.apply_gradients([ev2], global_step=0)
    g_cap.replay()
    torch.cuda.synchronize()
    oev.apply_adam_async(om, ov, 0.9, 0.999, 0.01, 0.9, 0.999, 1e-8, g[:2], ids[:2], gs=0)
    np.testing.assert_array_equal(ev2.sparse_read(T(ids[:2])).cpu().numpy(), oev.gather(ids[:2]))
    p = opt2._power(ev2)
    assert p[0] == float(np.float32(0.9) * np.float32(0.9))
    assert p[1] == float(np.float32(0.999) * np.float32(0.999))


def test_dense_adam_async_fp32_coefficients(dr):
    """Dense-table AdamAsync computes T(1) - beta in fp32 (1.0f - 0.9f =
    0.100000024f), as the op does; pinned against an fp32 numpy restatement
    of the element formula (bit-exact)."""
    R, D = 6, 4
    rng = np.random.default_rng(41)
    w0 = rng.standard_normal((R, D)).astype(np.float32)
    tab = dr.DenseTable(T(w0.copy()))
    opt = dr.AdamAsyncOptimizer(0.05)
    f = np.float32
    w, m, v = w0.copy(), np.zeros((R, D), f), np.zeros((R, D), f)
    b1p, b2p = f(0.9), f(0.999)
    for step in range(3):
        idx = np.array([0, 2, 5], np.int64)
        g = rng.standard_normal((3, D)).astype(f)
        tab.pending_grads.append(dr.IndexedSlices(T(g), T(idx)))
        opt.apply_gradients([tab], global_step=step)
        alpha = f(f(0.05) * np.sqrt(f(1) - b2p)) / (f(1) - b1p)
        m[idx] = m[idx] * f(0.9) + g * (f(1) - f(0.9))
        v[idx] = v[idx] * f(0.999) + (g * g) * (f(1) - f(0.999))
        w[idx] = w[idx] - (m[idx] * alpha) / (np.sqrt(v[idx]) + f(1e-8))
        b1p, b2p = b1p * f(0.9), b2p * f(0.999)
    np.testing.assert_allclose(tab.weight.cpu().numpy(), w, rtol=2e-7, atol=0)


def test_dense_table_adagrad_decay_and_adam_async(dr):
    """Dense tables (SparseApplyAdagradDecay, training_ali_ops.cc:495-670,
    one decay count per row; SparseApplyAdamAsync) against float64 numpy
    restatements of the same updates on the indexed rows."""
    rng = np.random.default_rng(31)
    R, D = 20, 6
    w0 = rng.standard_normal((R, D)).astype(np.float32)
    # AdagradDecay, decay_step 2: rows decay on global_step + 1 = 2, 4, ...
    tab = dr.DenseTable(T(w0.copy()))
    opt = dr.AdagradDecayOptimizer(0.2, initial_accumulator_value=0.1,
                                   accumulator_decay_step=2, accumulator_decay_rate=0.5)
    w, acc, pw = w0.astype(np.float64), np.full((R, D), 0.1), np.zeros(R, np.int64)
    for step in range(4):
        idx = np.sort(rng.choice(R, 8, replace=False)).astype(np.int64)
        g = rng.standard_normal((8, D)).astype(np.float32)
        tab.pending_grads.append(dr.IndexedSlices(T(g), T(idx)))
        opt.apply_gradients([tab], global_step=step)
        gs = step + 1
        for j, r in enumerate(idx):
            if gs // 2 > pw[r]:
                acc[r] = np.maximum(acc[r] * 0.5, 0.1)
                pw[r] += 1
            acc[r] = acc[r] + g[j].astype(np.float64) ** 2
            w[r] = w[r] - 0.2 * g[j] / np.sqrt(acc[r])
    np.testing.assert_allclose(tab.weight.cpu().numpy(), w, rtol=1e-5, atol=1e-6)
    # AdamAsync on a dense table
    tab2 = dr.DenseTable(T(w0.copy()))
    opt2 = dr.AdamAsyncOptimizer(0.05)
    w, m, v = w0.astype(np.float64), np.zeros((R, D)), np.zeros((R, D))
    b1p, b2p = 0.9, 0.999
    for step in range(3):
        idx = np.sort(rng.choice(R, 8, replace=False)).astype(np.int64)
        g = rng.standard_normal((8, D)).astype(np.float32).astype(np.float64)
        tab2.pending_grads.append(dr.IndexedSlices(T(g.astype(np.float32)), T(idx)))
        opt2.apply_gradients([tab2], global_step=step)
        alpha = 0.05 * np.sqrt(1 - b2p) / (1 - b1p)
        m[idx] = m[idx] * 0.9 + g * 0.1
        v[idx] = v[idx] * 0.999 + g * g * 0.001
        w[idx] = w[idx] - alpha * m[idx] / (np.sqrt(v[idx]) + 1e-8)
        b1p, b2p = b1p * 0.9, b2p * 0.999
    np.testing.assert_allclose(tab2.weight.cpu().numpy(), w, rtol=1e-4, atol=1e-5)
