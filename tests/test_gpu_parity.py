"""GPU parity: the HIP engine through its C ABI vs the CPU restatement (oracle/)
and the reference's golden vectors.  Integer/index work must be bit-exact;
fp32 pooling replays the reference association order and is checked
bit-exact as well (the north_star bound is 1e-5 relative); optimizer updates
with rsqrt/sqrt are checked at 1e-5 relative.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RTOL = 1e-5


def load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    deeprec_amd.set_validate(True)
    assert torch.cuda.is_available()
    return deeprec_amd


@pytest.fixture(scope="module")
def ops(dr):
    from deeprec_amd import ops
    return ops


DEV = "cuda:0"


def T(x, dtype=None):
    return torch.as_tensor(np.asarray(x), device=DEV, dtype=dtype)


def H(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------------------
def test_native_library_is_loaded(dr):
    from deeprec_amd import _lib
    assert _lib.lib().dr_abi_version() == 2
    maps = open("/proc/self/maps").read()
    assert "libdeeprec_amd.so" in maps


@pytest.mark.parametrize("case", ["sqrtn", "mean", "sum", "sqrtn_maxnorm200"])
def test_fused_local_forward_golden(ops, orc, case):
    g = load("fused_local")
    c = g["forward"][case]
    comb = c.get("combiner", case)
    table = np.asarray(g["table"], np.float32).reshape(g["bucket"], g["dim"])
    ind = np.asarray(g["sp_indices"], np.int64).reshape(-1, 2)
    out, vo = ops.fused_embedding_local_sparse_look_up(T(g["sp_values"]), T(ind), (g["batch"], 8),
                                                       T(table), comb, c["max_norm"])
    np.testing.assert_allclose(H(out).ravel(), c["expected"], atol=g["tolerance"], rtol=0)
    assert H(vo).tolist() == g["offsets_expected"]
    ref, _ = orc.fused_local_lookup(table, g["sp_values"], ind[:, 0], g["batch"], comb,
                                    c["max_norm"])
    if c["max_norm"] < 0:
        np.testing.assert_array_equal(H(out), ref)
    else:
        np.testing.assert_allclose(H(out), ref, rtol=RTOL)


@pytest.mark.parametrize("case", ["sqrtn", "mean", "sum", "mean_maxnorm100"])
def test_fused_local_grad_golden(ops, orc, case):
    g = load("fused_local")
    c = g["grad"][case]
    comb = c.get("combiner", case)
    table = np.asarray(g["table"], np.float32).reshape(g["bucket"], g["dim"])
    top = np.asarray(g["top_grad"], np.float32).reshape(g["batch"], g["dim"])
    out = ops.fused_embedding_local_sparse_look_up_grad(T(top), T(table), T(g["sp_values"]),
                                                        T(g["offsets_expected"], torch.int32),
                                                        comb, c["max_norm"])
    np.testing.assert_allclose(H(out).ravel(), c["expected"], atol=g["tolerance"], rtol=0)
    ref = orc.fused_local_lookup_grad(top, table, g["sp_values"], g["offsets_expected"], comb,
                                      c["max_norm"])
    np.testing.assert_allclose(H(out), ref, rtol=RTOL, atol=1e-7)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_segment_formula_kat(ops, orc, comb):
    g = load("segment_formula")
    rows, D, n = g["rows"], g["dim"], g["n"]
    data = np.repeat(np.arange(rows, dtype=np.float32)[:, None], D, 1)
    i = np.arange(n)
    idx, seg = (2 * i).astype(np.int32), (i // 2).astype(np.int32)
    fn = {"sum": ops.sparse_segment_sum, "mean": ops.sparse_segment_mean,
          "sqrtn": ops.sparse_segment_sqrt_n}[comb]
    out = H(fn(T(data), T(idx), T(seg)))
    np.testing.assert_array_equal(out, orc.sparse_segment_reduce(data, idx, seg, comb))


@pytest.mark.parametrize("D", [1, 3, 8, 18, 64, 128])
@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_segment_reduce_random_bitexact(ops, orc, D, comb):
    rng = np.random.default_rng(D * 7 + len(comb))
    R = 500
    data = rng.standard_normal((R, D)).astype(np.float32) * 10
    lens = rng.integers(0, 30, 64)
    lens[:12] = np.arange(12)           # every num % 8 branch incl. 0 (gap) and 1
    seg = np.repeat(np.arange(64), lens).astype(np.int32)
    idx = rng.integers(0, R, seg.shape[0]).astype(np.int32)
    fn = {"sum": ops.sparse_segment_sum, "mean": ops.sparse_segment_mean,
          "sqrtn": ops.sparse_segment_sqrt_n}[comb]
    out = H(fn(T(data), T(idx), T(seg), num_segments=70))
    ref = orc.sparse_segment_reduce(data, idx, seg, comb, num_segments=70)
    np.testing.assert_array_equal(out, ref)


def test_segment_reduce_errors_latched(dr, ops):
    data = T(np.ones((4, 2), np.float32))
    with pytest.raises(dr.DeepRecError):
        ops.sparse_segment_sum(data, T([0, 9], torch.int32), T([0, 1], torch.int32))
    with pytest.raises(dr.DeepRecError):
        ops.sparse_segment_sum(data, T([0, 1], torch.int32), T([1, 0], torch.int32),
                               num_segments=2)


@pytest.mark.parametrize("n,lo,hi", [(0, 0, 1), (1, 0, 1), (1000, 0, 10), (200000, -5, 100000),
                                     (300000, 0, 1 << 40), (500000, -3, 4), (400000, 0, 1000)])
def test_unique_bitexact(ops, orc, n, lo, hi):
    rng = np.random.default_rng(n)
    x = rng.integers(lo, hi, n).astype(np.int64)
    if n > 10:
        x[5] = -1                      # all-ones keys are ordinary keys
        x[7] = -1
    y, idx, cnt = ops.unique_with_counts(T(x))
    ry, ridx, rcnt = orc.unique(x, with_counts=True)
    np.testing.assert_array_equal(H(y), ry)
    np.testing.assert_array_equal(H(idx), ridx)
    np.testing.assert_array_equal(H(cnt), rcnt)


def test_unique_grouped_bitexact(ops, orc):
    rng = np.random.default_rng(77)
    sizes = [0, 1, 500, 3000, 17, 40000]
    parts = [rng.integers(-2, 50 + 7 * s, s).astype(np.int64) for s in sizes]
    koff = np.concatenate([[0], np.cumsum(sizes)]).tolist()
    y, idx, cnt, U = ops.unique_grouped(T(np.concatenate(parts)), koff, with_counts=True)
    y, idx, cnt, U = H(y), H(idx), H(cnt), H(U)
    for t, x in enumerate(parts):
        ry, ridx, rcnt = orc.unique(x, with_counts=True)
        assert U[t] == ry.shape[0]
        a = koff[t]
        np.testing.assert_array_equal(y[a:a + U[t]], ry)
        np.testing.assert_array_equal(idx[a:koff[t + 1]], ridx)
        np.testing.assert_array_equal(cnt[a:a + U[t]], rcnt)


@pytest.mark.parametrize("probes", [2048, 1])
def test_unique_skewed_and_overflow_bitexact(dr, ops, orc, probes):
    """LDS-staged Unique on skewed inputs (a padding id holding half of a
    feature, long runs, a 1.3M-key feature that fills 1024 buckets) and, with
    the LDS hash walk cut to one probe, through every bucket's global overflow
    region: outputs stay bit-identical to the oracle's serial Unique."""
    rng = np.random.default_rng(probes)
    pad = rng.integers(0, 400000, 200000).astype(np.int64)
    pad[rng.random(200000) < 0.5] = 0                       # DIN-style padded histories
    runs = np.repeat(rng.integers(-5, 5000, 3000), rng.integers(1, 90, 3000)).astype(np.int64)
    big = rng.integers(0, 1 << 40, 1300000).astype(np.int64)
    parts = [pad, runs, big, np.full(7000, -1, np.int64)]
    from deeprec_amd import _lib
    lib = _lib.lib()
    lib.dr_unique_set_lds_probes(probes)
    try:
        for x in parts:
            y, idx, cnt = ops.unique_with_counts(T(x))
            ry, ridx, rcnt = orc.unique(x, with_counts=True)
            np.testing.assert_array_equal(H(y), ry)
            np.testing.assert_array_equal(H(idx), ridx)
            np.testing.assert_array_equal(H(cnt), rcnt)
        koff = np.concatenate([[0], np.cumsum([p.shape[0] for p in parts])]).tolist()
        y, idx, cnt, U = ops.unique_grouped(T(np.concatenate(parts)), koff, with_counts=True)
        y, idx, cnt, U = H(y), H(idx), H(cnt), H(U)
        for t, x in enumerate(parts):
            ry, ridx, rcnt = orc.unique(x, with_counts=True)
            a = koff[t]
            assert U[t] == ry.shape[0]
            np.testing.assert_array_equal(y[a:a + U[t]], ry)
            np.testing.assert_array_equal(idx[a:koff[t + 1]], ridx)
            np.testing.assert_array_equal(cnt[a:a + U[t]], rcnt)
    finally:
        lib.dr_unique_set_lds_probes(2048)


def test_route_by_owner(ops):
    rng = np.random.default_rng(78)
    sizes = [1000, 0, 2500, 300]
    parts = [rng.integers(0, 10 ** 6, s).astype(np.int64) for s in sizes]
    koff = np.concatenate([[0], np.cumsum(sizes)]).tolist()
    y, idx, cnt, U = ops.unique_grouped(T(np.concatenate(parts)), koff)
    for world in (1, 2, 8):
        keys, tags, perm, counts = ops.route_by_owner(y, koff, U, world)
        counts = H(counts)
        exp_k, exp_t = [], []
        Uh, yh = H(U), H(y)
        for p in range(world):
            for t in range(len(sizes)):
                u = yh[koff[t]:koff[t] + Uh[t]]
                sel = u[u % world == p]
                assert counts[p, t] == sel.shape[0]
                exp_k.append(sel)
                exp_t.append(np.full(sel.shape[0], t))
        m = int(counts.sum())
        np.testing.assert_array_equal(H(keys)[:m], np.concatenate(exp_k))
        np.testing.assert_array_equal(H(tags)[:m], np.concatenate(exp_t))
        np.testing.assert_array_equal(yh[H(perm)[:m]], np.concatenate(exp_k))


@pytest.mark.parametrize("grad", [True, False])
def test_multi_feature_grouped_lookup(dr, orc, grad):
    """grad=False exercises the forward-only direct resolve (no Unique):
    outputs, key counts and exported keys must equal the unique path's."""
    rng = np.random.default_rng(79)
    B, D, F = 300, 32, 5
    evs, oevs, sps, raw = [], [], [], []
    for f in range(F):
        evs.append(dr.EmbeddingVariable("mf%d_%d" % (f, grad), D, 0.1 * (f + 1)))
        oevs.append(orc.EV(D, 0.1 * (f + 1)))
        keys = np.arange(100 * f, 100 * f + 80, dtype=np.int64)
        vals = rng.standard_normal((80, D)).astype(np.float32)
        evs[-1].insert(T(keys), T(vals))
        oevs[-1].insert(keys, vals)
        ind, v = _random_sparse(rng, B, 4, 100 * f + 160)
        sps.append(dr.SparseTensor(T(ind), T(v), (B, 4)))
        raw.append((ind, v))
    with torch.set_grad_enabled(grad):
        out = H(dr.embedding_lookup_sparse_multi(evs, sps, combiner="mean"))
    for f in range(F):
        ref = orc.embedding_lookup_sparse(oevs[f], raw[f][0], raw[f][1], B, combiner="mean")
        np.testing.assert_array_equal(out[:, f * D:(f + 1) * D], ref)
        assert int(evs[f].total_count()[0]) == oevs[f].size()
        k, v = evs[f].export()[:2]
        ok, ov = oevs[f].export()[:2]
        np.testing.assert_array_equal(H(k), ok)
        np.testing.assert_array_equal(H(v), ov)


@pytest.mark.parametrize("kernel", ["1", "2", "0"])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("D", [8, 128])
def test_onehot_forward_lookup(dr, orc, fused, D, kernel):
    """Forward-only one-hot lookup of filter-free EVs: the fused probe+copy
    kernel (dr_ev_lookup_onehot: DR_LOOKUP_KERNEL 1 line probes, the default;
    2 the pipelined persistent kernel; 0 the slot walk) and the resolve ->
    pool pipeline must all equal the oracle's unique -> gather -> pool,
    including misses (inserted with the default row), duplicate new keys in
    one batch, key -1, and a slot EV column whose rows exist but whose column
    was never touched."""
    import os
    from deeprec_amd import embedding_ops as eo
    if not fused and kernel != "1":
        pytest.skip("the kernel switch only selects the fused lookup")
    rng = np.random.default_rng(83 + D)
    B, F = 777, 3
    saved = eo._FUSED_ONEHOT
    eo._FUSED_ONEHOT = fused
    os.environ["DR_LOOKUP_KERNEL"] = kernel
    try:
        evs, oevs = [], []
        for f in range(F):
            evs.append(dr.EmbeddingVariable("oh%d_%d_%d_%s" % (f, D, fused, kernel), D, 0.5 - f,
                                            capacity=300))
            oevs.append(orc.EV(D, 0.5 - f))
            keys = np.arange(0, 400, 2, dtype=np.int64) + f
            vals = rng.standard_normal((keys.shape[0], D)).astype(np.float32)
            evs[-1].insert(T(keys), T(vals))
            oevs[-1].insert(keys, vals)
        for step in range(3):
            ids = rng.integers(-1, 700, (F, B)).astype(np.int64)  # ~half new, dups, -1
            flat = T(ids.reshape(-1))
            ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
            sps = [dr.SparseTensor(T(ind), flat[f * B:(f + 1) * B], (B, 1)) for f in range(F)]
            with torch.no_grad():
                out = H(dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum"))
            for f in range(F):
                ref = orc.embedding_lookup_sparse(oevs[f], ind, ids[f], B, combiner="sum")
                np.testing.assert_array_equal(out[:, f * D:(f + 1) * D], ref)
        for f in range(F):
            assert int(evs[f].total_count()[0]) == oevs[f].size()
            k, v = evs[f].export()[:2]
            ok, ov = oevs[f].export()[:2]
            np.testing.assert_array_equal(H(k), ok)
            np.testing.assert_array_equal(H(v), ov)
    finally:
        eo._FUSED_ONEHOT = saved
        del os.environ["DR_LOOKUP_KERNEL"]


def test_onehot_fused_abi_orders_and_slot_column(dr):
    """dr_ev_lookup_onehot directly: SEQ order turns -0.0 into +0.0 (fused
    op semantics), ALI keeps it; a slot EV (column 1) of existing keys is
    initialised on first touch by the miss path."""
    import ctypes as C
    from deeprec_amd._lib import ORDER_ALI, ORDER_SEQ, check, lib, ptr, stream_handle, workspace
    D, B = 4, 5
    ev = dr.EmbeddingVariable("ohabi", D, 0.0, capacity=64)
    ev.insert(T(np.array([1, 2], np.int64)), T(np.array([[-0.0] * D, [3.0] * D], np.float32)))
    sl = ev.slot("acc", 0.25)
    keys = T(np.array([1, 2, 2, 9, 1], np.int64))
    for col_ev, order, want in ((ev, ORDER_ALI, None), (ev, ORDER_SEQ, None), (sl, ORDER_ALI, 0.25)):
        out = torch.full((B, D), 7.0, device=DEV)
        h = (C.c_void_p * 1)(col_ev.handle.value)
        wsb = lib().dr_ev_lookup_onehot_workspace_size(1, B)
        ws = workspace(wsb, DEV)
        check(lib().dr_ev_lookup_onehot(h, 1, ptr(keys), B, ptr(out), D, order, ptr(ws), wsb,
                                        stream_handle()))
        o = H(out)
        if want is not None:
            assert (o == want).all()
            continue
        np.testing.assert_array_equal(o[1], [3.0] * D)
        np.testing.assert_array_equal(o[3], [0.0] * D)  # new key 9: EV default
        neg = np.signbit(o[0])
        assert neg.all() if order == ORDER_ALI else (~neg).all()


@pytest.mark.parametrize("n,kmax,bit_lo,bit_hi", [
    (100003, 1 << 20, 0, 20), (1, 5, 0, 8), (4095, 1 << 12, 0, 12), (4096, 7, 0, 3),
    (4097, 1 << 40, 0, 40), (2000000, 1 << 21, 0, 21), (300000, 3, 0, 2),
    (50000, 1 << 40, 9, 34), (300000, 1 << 62, 0, 62)])
def test_sort_pairs_stable(ops, n, kmax, bit_lo, bit_hi):
    """Stable LSD sort on bits [bit_lo, bit_hi): ragged last tile, one key,
    exactly one tile, few distinct keys (runs spanning many tiles), and a
    bit window that ignores the low and high bits (ties keep input order)."""
    rng = np.random.default_rng(n)
    keys = rng.integers(0, kmax, n).astype(np.int64)
    vals = np.arange(n, dtype=np.int32)
    ko, vo = ops.sort_pairs(T(keys), T(vals), bit_hi, bit_lo)
    order = np.argsort((keys >> bit_lo) & ((1 << (bit_hi - bit_lo)) - 1), kind="stable")
    np.testing.assert_array_equal(H(ko), keys[order])
    np.testing.assert_array_equal(H(vo), vals[order])


@pytest.mark.parametrize("n,D,S", [(20000, 24, 700), (5000, 128, 40), (3000, 3, 2500)])
def test_unsorted_segment_sum_bitexact(ops, orc, n, D, S):
    rng = np.random.default_rng(11)
    data = (rng.standard_normal((n, D)) * 100).astype(np.float32)
    seg = rng.integers(-3, S, n).astype(np.int32)
    out = H(ops.unsorted_segment_sum(T(data), T(seg), S))
    np.testing.assert_array_equal(out, orc.unsorted_segment_sum(data, seg, S))


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_segment_grad_bitexact(ops, orc, comb):
    rng = np.random.default_rng(5)
    B, D, U = 300, 16, 120
    lens = rng.integers(1, 12, B)
    seg = np.repeat(np.arange(B), lens).astype(np.int32)
    idx = rng.integers(0, U, seg.shape[0]).astype(np.int32)
    grad = rng.standard_normal((B, D)).astype(np.float32)
    fn = {"sum": ops.sparse_segment_sum_grad, "mean": ops.sparse_segment_mean_grad,
          "sqrtn": ops.sparse_segment_sqrt_n_grad}[comb]
    out = H(fn(T(grad), T(idx), T(seg), U))
    np.testing.assert_array_equal(out, orc.sparse_segment_reduce_grad(grad, idx, seg, U, comb))


def test_gather_and_oob(dr, ops):
    t = np.arange(40, dtype=np.float32).reshape(10, 4)
    out = H(ops.gather(T(t), T([3, 0, 9])))
    np.testing.assert_array_equal(out, t[[3, 0, 9]])
    with pytest.raises(dr.DeepRecError):
        ops.gather(T(t), T([10]))


# ---------------------------------------------------------------------------
# EmbeddingVariable
# ---------------------------------------------------------------------------
def test_ev_export_kat(dr, orc):
    k = load("ev")["export"]
    ev = dr.EmbeddingVariable("exp", k["dim"], k["init"],
                              ev_option=dr.EmbeddingVariableOption(
                                  filter_option=dr.CounterFilter(k["filter_freq"]),
                                  evict_option=dr.GlobalStepEvict(k["steps_to_live"])))
    from deeprec_amd import ops
    for _ in range(k["runs"]):
        u, idx, cnt = ops.unique_with_counts(T(k["lookup"]))
        ev.sparse_read(u, counts=cnt)
    keys, vals, vers, frqs = ev.export()
    assert H(keys).tolist() == k["keys"]
    assert H(vals).tolist() == k["values"]
    assert H(vers).tolist() == k["versions"]
    assert H(frqs).tolist() == k["freqs"]


def test_ev_shape_kat(dr):
    k = load("ev")["shape"]
    ev = dr.EmbeddingVariable("shape", k["dim"], 1.0)
    ev.sparse_read(T(k["lookup"]))
    assert ev.total_count().tolist() == k["expected"]


def test_ev_counter_filter_timeline(dr, ops):
    k = load("ev")["counter_filter_gd"]
    ev = dr.EmbeddingVariable("cf", k["dim"], 1.0,
                              ev_option=dr.EmbeddingVariableOption(
                                  filter_option=dr.CounterFilter(k["filter_freq"])))
    opt = dr.GradientDescentOptimizer(k["lr"])
    seen = []
    for step in range(4):
        u, idx, cnt = ops.unique_with_counts(T([k["key"]]))
        seen.append(H(ev.sparse_read(u, counts=cnt)))
        ev.pending_grads.append(dr.IndexedSlices(
            T(np.full((1, k["dim"]), k["loss_scale"], np.float32)), u))
        opt.apply_gradients([ev], global_step=step)
    assert all((s == 1.0).all() for s in seen[:3])
    assert (seen[3] != 1.0).all()


def test_ev_gather_matches_oracle(dr, orc):
    rng = np.random.default_rng(9)
    D = 16
    ev = dr.EmbeddingVariable("g", D, 0.5, capacity=64)      # forces growth
    oev = orc.EV(D, 0.5)
    for step in range(5):
        keys = np.unique(rng.integers(-10, 400, 150)).astype(np.int64)
        rng.shuffle(keys)
        dflt = rng.standard_normal((keys.shape[0], D)).astype(np.float32)
        out = H(ev.sparse_read(T(keys), ev_init_value=T(dflt)))
        ref = oev.gather(keys, dflt)
        np.testing.assert_array_equal(out, ref)
    assert int(ev.total_count()[0]) == oev.size()
    k1, v1, _, _ = ev.export()
    k2, v2, _, _ = oev.export()
    np.testing.assert_array_equal(H(k1), k2)
    np.testing.assert_array_equal(H(v1), v2)


@pytest.mark.parametrize("D", [3, 128])
def test_ev_gather_wide_and_odd_dims(dr, orc, D):
    # dwordx4 copy-out (D % 4 == 0) and the scalar one; EV default row and
    # per-key defaults
    rng = np.random.default_rng(19)
    ev = dr.EmbeddingVariable("gw%d" % D, D, 0.25, capacity=256)
    oev = orc.EV(D, 0.25)
    for step in range(3):
        keys = np.unique(rng.integers(0, 3000, 700)).astype(np.int64)
        rng.shuffle(keys)
        if step == 1:
            dflt = rng.standard_normal((keys.shape[0], D)).astype(np.float32)
            out = H(ev.sparse_read(T(keys), ev_init_value=T(dflt)))
            ref = oev.gather(keys, dflt)
        else:
            out = H(ev.sparse_read(T(keys)))
            ref = oev.gather(keys, np.full((keys.shape[0], D), 0.25, np.float32))
        np.testing.assert_array_equal(out, ref)


def test_ev_insert_import_semantics(dr, orc):
    ev = dr.EmbeddingVariable("imp", 2, 0.0, steps_to_live=5,
                              ev_option=dr.EmbeddingVariableOption(
                                  filter_option=dr.CounterFilter(2)))
    keys = np.arange(20, dtype=np.int64)
    vals = np.repeat(keys[:, None], 2, 1).astype(np.float32)
    ev.import_partitioned(T(keys), T(vals), T(keys * 10), T(np.ones(20, np.int64)), 1, 4)
    k, v, ver, fr = ev.export()
    assert H(k).tolist() == [x for x in range(20) if x % 4 == 1]
    assert (H(fr) == 2).all()
    assert H(ver).tolist() == [x * 10 for x in H(k)]
    # existing rows are kept by insert (Import semantics)
    ev.insert(T(np.array([1], np.int64)), T(np.array([[7.0, 7.0]], np.float32)))
    k, v, _, _ = ev.export()
    assert H(v)[0].tolist() == [1.0, 1.0]


@pytest.mark.parametrize("opt", ["sgd", "adagrad", "adam"])
def test_ev_equals_dense_5step(dr, orc, opt):
    k = load("ev")["ev_equals_dense"]
    D, ids, lr = k["dim"], np.asarray(k["ids"], np.int64), np.float32(k["lr"])
    ev = dr.EmbeddingVariable("eq_" + opt, D, 1.0)
    oev = orc.EV(D, 1.0)
    if opt == "sgd":
        o = dr.GradientDescentOptimizer(lr)
    elif opt == "adagrad":
        o = dr.AdagradOptimizer(lr, k["adagrad_initial_accumulator"])
        oacc = oev.create_slot(1, k["adagrad_initial_accumulator"])
    else:
        a = k["adam"]
        o = dr.AdamOptimizer(lr, a["beta1"], a["beta2"], a["epsilon"])
        om, ov = oev.create_slot(1, 0.0), oev.create_slot(2, 0.0)
    g = np.full((len(ids), D), k["loss_scale"], np.float32)
    for step in range(k["steps"]):
        r = H(ev.sparse_read(T(ids)))
        np.testing.assert_allclose(r, oev.gather(ids), rtol=RTOL)
        ev.pending_grads.append(dr.IndexedSlices(T(g), T(ids)))
        o.apply_gradients([ev], global_step=step)
        if opt == "sgd":
            oev.apply_sgd(lr, g, ids, step)
        elif opt == "adagrad":
            oev.apply_adagrad(oacc, lr, g, ids, step)
        else:
            b1p = np.float32(a["beta1"]) ** (step + 1)
            b2p = np.float32(a["beta2"]) ** (step + 1)
            oev.apply_adam(om, ov, b1p, b2p, lr, a["beta1"], a["beta2"], a["epsilon"], g, ids,
                           step)
    final = H(ev.sparse_read(T(ids)))
    if opt == "sgd":
        np.testing.assert_array_equal(final, oev.gather(ids))
    else:
        np.testing.assert_allclose(final, oev.gather(ids), rtol=RTOL)


def test_ev_bloom_filter_sequential(dr, orc):
    f = dr.CBFFilter(filter_freq=3, max_element_size=1000, false_positive_probability=0.01,
                     counter_type=16)
    ev = dr.EmbeddingVariable("bloom", 4, 0.5, ev_option=dr.EmbeddingVariableOption(
        filter_option=f))
    oev = orc.EV(4, 0.5, filter_freq=3, max_element_size=1000, false_positive_probability=0.01,
                 counter_bits=16)
    for rep in range(5):
        for key in range(12):
            a = H(ev.sparse_read(T([key])))
            b = oev.gather(np.array([key], np.int64))
            np.testing.assert_array_equal(a, b)
    assert int(ev.total_count()[0]) == oev.size()
    _, _, _, f1 = ev.export()
    _, _, _, f2 = oev.export()
    np.testing.assert_array_equal(H(f1), f2)


# ---------------------------------------------------------------------------
# embedding_lookup_sparse composition
# ---------------------------------------------------------------------------
def _random_sparse(rng, B, max_h, vocab, allow_empty=False):
    lens = rng.integers(0 if allow_empty else 1, max_h + 1, B)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(l) for l in lens]) if lens.sum() else np.zeros(0, np.int64)
    ind = np.stack([rows, cols], 1).astype(np.int64)
    vals = rng.integers(0, vocab, rows.shape[0]).astype(np.int64)
    return ind, vals


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
@pytest.mark.parametrize("D", [8, 64, 128])
def test_ev_lookup_sparse_bitexact(dr, orc, comb, D):
    rng = np.random.default_rng(D + 3)
    B = 257
    ev = dr.EmbeddingVariable("els_%s_%d" % (comb, D), D, 0.25)
    oev = orc.EV(D, 0.25)
    # pre-populate part of the key space with distinct rows
    keys = np.arange(0, 300, dtype=np.int64)
    vals = rng.standard_normal((300, D)).astype(np.float32)
    ev.insert(T(keys), T(vals))
    oev.insert(keys, vals)
    ind, v = _random_sparse(rng, B, 20, 600)
    out = H(dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 20)),
                                       combiner=comb))
    ref = orc.embedding_lookup_sparse(oev, ind, v, B, combiner=comb)
    np.testing.assert_array_equal(out, ref)
    assert int(ev.total_count()[0]) == oev.size()


@pytest.mark.parametrize("B", [1, 7, 8, 1003])
def test_onehot_and_mostly_onehot_pooling(dr, orc, B):
    """Pool kernel split: all-singleton chunks go to the lean copy kernel
    (DR_POOL_ONEHOT when the SparseTensor is [B, 1] with nnz == B), mixed
    chunks to the general kernel -- both bit-exact to the oracle."""
    rng = np.random.default_rng(B + 11)
    D, R = 64, 4000
    table = rng.standard_normal((R, D)).astype(np.float32)
    table[5] = -0.0                      # SEQ order must turn -0.0 into +0.0
    # one-hot [B, 1]
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1).astype(np.int64)
    v = rng.integers(0, R, B).astype(np.int64)
    v[0] = 5
    for comb in ("sum", "mean", "sqrtn"):
        out = H(dr.embedding_lookup_sparse(T(table), dr.SparseTensor(T(ind), T(v), (B, 1)),
                                           combiner=comb))
        np.testing.assert_array_equal(out, orc.embedding_lookup_sparse(table, ind, v, B,
                                                                       combiner=comb))
    # mostly one-hot: ~5% of bags hold 2-3 ids, some chunks fast, some general
    lens = np.where(rng.random(B) < 0.05, rng.integers(2, 4, B), 1)
    rows = np.repeat(np.arange(B), lens)
    cols = np.concatenate([np.arange(l) for l in lens])
    ind2 = np.stack([rows, cols], 1).astype(np.int64)
    v2 = rng.integers(0, R, rows.shape[0]).astype(np.int64)
    for comb in ("sum", "mean", "sqrtn"):
        out = H(dr.embedding_lookup_sparse(T(table), dr.SparseTensor(T(ind2), T(v2), (B, 3)),
                                           combiner=comb))
        np.testing.assert_array_equal(out, orc.embedding_lookup_sparse(table, ind2, v2, B,
                                                                       combiner=comb))
    # grouped EV features, one-hot
    evs, oevs, sps, raw = [], [], [], []
    for f in range(3):
        evs.append(dr.EmbeddingVariable("oh%d_%d" % (B, f), D, 0.5))
        oevs.append(orc.EV(D, 0.5))
        keys = np.arange(0, 50, dtype=np.int64)
        vals = rng.standard_normal((50, D)).astype(np.float32)
        evs[-1].insert(T(keys), T(vals))
        oevs[-1].insert(keys, vals)
        vf = rng.integers(0, 100, B).astype(np.int64)
        sps.append(dr.SparseTensor(T(ind), T(vf), (B, 1)))
        raw.append(vf)
    out = H(dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum"))
    for f in range(3):
        ref = orc.embedding_lookup_sparse(oevs[f], ind, raw[f], B, combiner="sum")
        np.testing.assert_array_equal(out[:, f * D:(f + 1) * D], ref)


def test_many_feature_forward_matches_oracle(dr, orc):
    """11 one-hot filter-free EV features without grad (direct resolve, one
    grouped pool launch); outputs and EV contents must equal the oracle
    (insert-on-miss included)."""
    rng = np.random.default_rng(123)
    B, D, F = 700, 32, 11
    ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
    evs, oevs, sps, vals = [], [], [], []
    for f in range(F):
        evs.append(dr.EmbeddingVariable("pipe%d" % f, D, 0.25 + f))
        oevs.append(orc.EV(D, 0.25 + f))
        keys = np.arange(0, 300, dtype=np.int64)
        rows = rng.standard_normal((300, D)).astype(np.float32)
        evs[-1].insert(T(keys), T(rows))
        oevs[-1].insert(keys, rows)
        v = rng.integers(0, 600, B).astype(np.int64)
        vals.append(v)
        sps.append(dr.SparseTensor(T(ind), T(v), (B, 1)))
    with torch.no_grad():
        out = H(dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum"))
    for f in range(F):
        ref = orc.embedding_lookup_sparse(oevs[f], ind, vals[f], B, combiner="sum")
        np.testing.assert_array_equal(out[:, f * D:(f + 1) * D], ref)
        assert int(evs[f].total_count()[0]) == oevs[f].size()


def test_pool_onehot_flag_rejects_weights(dr, ops):
    from deeprec_amd import _lib
    t = torch.zeros((4, 8), device=DEV)
    ids = torch.arange(4, device=DEV)
    w = torch.ones(4, device=DEV)
    out = torch.empty((4, 8), device=DEV)
    d = _lib.DrPoolDesc()
    d.pool, d.pool_rows, d.ids, d.weights = t.data_ptr(), 4, ids.data_ptr(), w.data_ptr()
    d.out, d.out_stride, d.combiner, d.max_norm = out.data_ptr(), 8, 0, -1.0
    with pytest.raises(_lib.InvalidArgumentError):
        ops.pool_grouped([d], 4, 8, onehot=True)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_dense_lookup_sparse_bitexact(dr, orc, comb):
    rng = np.random.default_rng(17)
    B, D, R = 1000, 32, 5000
    table = rng.standard_normal((R, D)).astype(np.float32)
    ind, v = _random_sparse(rng, B, 15, R)
    out = H(dr.embedding_lookup_sparse(T(table), dr.SparseTensor(T(ind), T(v), (B, 15)),
                                       combiner=comb))
    np.testing.assert_array_equal(out, orc.embedding_lookup_sparse(table, ind, v, B,
                                                                   combiner=comb))


def test_weighted_and_max_norm_lookup(dr, orc):
    rng = np.random.default_rng(21)
    B, D, R = 200, 16, 800
    table = rng.standard_normal((R, D)).astype(np.float32)
    ind, v = _random_sparse(rng, B, 6, R)
    w = rng.uniform(0.1, 2.0, v.shape[0]).astype(np.float32)
    sp = dr.SparseTensor(T(ind), T(v), (B, 6))
    for comb in ("sum", "mean", "sqrtn"):
        out = H(dr.embedding_lookup_sparse(T(table), sp, dr.SparseTensor(T(ind), T(w), (B, 6)),
                                           combiner=comb))
        ref = orc.embedding_lookup_sparse(table, ind, v, B, weights=w, combiner=comb)
        np.testing.assert_allclose(out, ref, rtol=RTOL, atol=1e-6)
        out = H(dr.embedding_lookup_sparse(T(table), sp, combiner=comb, max_norm=1.5))
        ref = orc.embedding_lookup_sparse(table, ind, v, B, combiner=comb, max_norm=1.5)
        np.testing.assert_allclose(out, ref, rtol=RTOL, atol=1e-6)


def test_safe_lookup_prune_and_empty_rows(dr, orc):
    rng = np.random.default_rng(23)
    B, D = 100, 8
    ev = dr.EmbeddingVariable("safe", D, 0.5)
    oev = orc.EV(D, 0.5)
    ind, v = _random_sparse(rng, B, 5, 50, allow_empty=True)
    v[::7] = -3                                  # pruned ids
    sp = dr.SparseTensor(T(ind), T(v), (B, 5))
    for default_id in (None, 4):
        out = H(dr.safe_embedding_lookup_sparse(ev, sp, combiner="mean", default_id=default_id))
        ref = orc.safe_embedding_lookup_sparse(oev, ind, v, (B, 5), combiner="mean",
                                               default_id=default_id)
        np.testing.assert_array_equal(out, ref)
    assert int(ev.total_count()[0]) == oev.size()


def test_lookup_backward_matches_segment_grad(dr, orc):
    rng = np.random.default_rng(29)
    B, D = 64, 8
    for comb in ("sum", "mean", "sqrtn"):
        ev = dr.EmbeddingVariable("bw_" + comb, D, 0.1)
        ind, v = _random_sparse(rng, B, 7, 40)
        out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(T(ind), T(v), (B, 7)),
                                         combiner=comb)
        g = rng.standard_normal((B, D)).astype(np.float32)
        out.backward(T(g))
        sl = ev.pending_grads.pop()
        U = int(sl.num_valid.item())
        uids, idx = orc.unique(v)
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        ref = orc.sparse_segment_reduce_grad(g, idx, ind[:, 0].astype(np.int32), U, comb)
        np.testing.assert_array_equal(H(sl.values[:U]), ref)


@pytest.mark.parametrize("onehot", [True, False])
@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_grouped_backward_matches_segment_grad(dr, orc, onehot, comb):
    """Grouped features (one dr_unique_grouped) -> one dr_pool_grad_grouped:
    each feature's IndexedSlices equal the reference SparseSegment*Grad."""
    rng = np.random.default_rng(31 + int(onehot))
    B, D, F = 300, 32, 4
    evs, sps, raw = [], [], []
    for f in range(F):
        evs.append(dr.EmbeddingVariable("gbw_%d_%s_%d" % (int(onehot), comb, f), D, 0.1))
        if onehot:
            ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
            v = rng.integers(0, 120, B).astype(np.int64)
            shape = (B, 1)
        else:
            ind, v = _random_sparse(rng, B, 5, 120, allow_empty=True)
            shape = (B, 5)
        sps.append(dr.SparseTensor(T(ind), T(v), shape))
        raw.append((ind, v))
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner=comb)
    g = rng.standard_normal((B, F * D)).astype(np.float32)
    out.backward(T(g))
    for f in range(F):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        uids, idx = orc.unique(raw[f][1])
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        ref = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g[:, f * D:(f + 1) * D]), idx,
                                             raw[f][0][:, 0].astype(np.int32), U, comb)
        np.testing.assert_array_equal(H(sl.values[:U]), ref)


@pytest.mark.parametrize("comb", ["sum", "mean"])
@pytest.mark.parametrize("D", [18, 32])
def test_grouped_backward_long_runs(dr, orc, comb, D):
    """Hot ids on the Unique path (dr_pool_grad_grouped; it also serves the
    sharded backward): runs of 257, 5000, 21846 (a Criteo-TB feature of
    cardinality 3 at B = 65536) and 65536 positions, besides 256 / 768 / 200.
    Every run, whatever its length, is ONE serial chain in ascending position
    order -- bit-equal to the reference's UnsortedSegmentSum /
    SparseSegmentReductionGrad loops (segment_reduction_ops.cc:391-404)."""
    rng = np.random.default_rng(37)
    runs = {0: 5000, 1: 256, 2: 257, 3: 768, 4: 200, 5: 21846, 6: 65536}
    v = np.concatenate([np.full(n, k, np.int64) for k, n in runs.items()] +
                       [rng.integers(7, 400, 3000).astype(np.int64)])
    rng.shuffle(v)
    B = v.size
    evs, sps = [], []
    for f in range(2):
        evs.append(dr.EmbeddingVariable("lrun_%s_%d_%d" % (comb, D, f), D, 0.1))
        ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
        sps.append(dr.SparseTensor(T(ind), T(v), (B, 1)))
    out = dr.embedding_lookup_sparse_multi(evs, sps, combiner=comb)
    g = rng.standard_normal((B, 2 * D)).astype(np.float32)
    out.backward(T(g))
    uids, idx = orc.unique(v)
    seg = np.arange(B, dtype=np.int32)
    for f in range(2):
        sl = evs[f].pending_grads.pop()
        U = int(sl.num_valid.item())
        assert H(sl.indices[:U]).tolist() == uids.tolist()
        ref = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g[:, f * D:(f + 1) * D]), idx,
                                             seg, U, comb)
        np.testing.assert_array_equal(H(sl.values[:U]), ref)
    dr.status_check()


@pytest.mark.parametrize("comb", ["mean", "sqrtn"])
def test_grouped_backward_long_runs_multihot(dr, orc, comb):
    """Multi-hot bags (the per-term 1/cnt or 1/sqrt(cnt) bag scale) with a
    hot id in 30000 bags and a weighted feature: long runs bit-exact too."""
    rng = np.random.default_rng(43)
    B, H_, D = 40000, 4, 16
    ind, v = _random_sparse(rng, B, H_, 300, allow_empty=False)
    v = v.copy()
    hot = rng.random(v.size) < 0.3
    v[hot] = 7                                  # one id over ~30 % of the positions
    ev = dr.EmbeddingVariable("lrun_mh_%s" % comb, D, 0.1)
    sp = dr.SparseTensor(T(ind), T(v), (B, H_))
    out = dr.embedding_lookup_sparse(ev, sp, combiner=comb)
    g = rng.standard_normal((B, D)).astype(np.float32)
    out.backward(T(g))
    sl = ev.pending_grads.pop()
    U = int(sl.num_valid.item())
    uids, idx = orc.unique(v)
    assert int(np.bincount(idx).max()) > 10000
    assert H(sl.indices[:U]).tolist() == uids.tolist()
    ref = orc.sparse_segment_reduce_grad(g, idx, ind[:, 0].astype(np.int32), U, comb)
    np.testing.assert_array_equal(H(sl.values[:U]), ref)
    dr.status_check()


def test_optimizers_with_repeated_indices(dr, orc):
    """SGD hands raw repeated indices to the KV kernel, which walks them in
    order (gradient_descent.py:71-76); Adagrad sums them first
    (_deduplicate_indexed_slices, optimizer.py:68-83)."""
    rng = np.random.default_rng(3)
    D = 40
    keys = np.array([5, 9, 5, 5, 2, 9, 100, 5] * 20, np.int64)   # ranks up to 80
    g = rng.standard_normal((keys.shape[0], D)).astype(np.float32)
    # SGD: sequential application
    ev = dr.EmbeddingVariable("dup_sgd", D, 0.5)
    oev = orc.EV(D, 0.5)
    ev.pending_grads.append(dr.IndexedSlices(T(g), T(keys)))
    dr.GradientDescentOptimizer(0.1).apply_gradients([ev], global_step=0)
    oev.apply_sgd(np.float32(0.1), g, keys, 0)
    k, v = ev.export()[:2]
    ok, ov = oev.export()[:2]
    np.testing.assert_array_equal(H(k), ok)
    np.testing.assert_array_equal(H(v), ov)
    # Adagrad: dedup (unique + unsorted_segment_sum) then one update per key
    ev2 = dr.EmbeddingVariable("dup_ada", D, 0.5)
    oev2 = orc.EV(D, 0.5)
    oacc = oev2.create_slot(1, 0.1)
    ev2.pending_grads.append(dr.IndexedSlices(T(g), T(keys)))
    dr.AdagradOptimizer(0.1, 0.1).apply_gradients([ev2], global_step=0)
    u, pos = orc.unique(keys)
    gs = orc.unsorted_segment_sum(g, pos, u.shape[0])
    oev2.apply_adagrad(oacc, np.float32(0.1), gs, u, 0)
    k, v = ev2.export()[:2]
    ok, ov = oev2.export()[:2]
    np.testing.assert_array_equal(H(k), ok)
    np.testing.assert_array_equal(H(v), ov)


def test_grouped_train_step_matches_oracle(dr, orc):
    """fwd -> grouped bwd -> KV SGD / Adagrad apply over 3 steps equals the
    oracle EV updated with the reference formulas."""
    rng = np.random.default_rng(77)
    B, D, F = 256, 64, 3
    for opt_name in ("sgd", "adagrad"):
        evs, oevs, oacc = [], [], []
        for f in range(F):
            evs.append(dr.EmbeddingVariable("gts_%s_%d" % (opt_name, f), D, 0.05))
            oevs.append(orc.EV(D, 0.05))
            if opt_name == "adagrad":
                oacc.append(oevs[-1].create_slot(1, 0.1))
        opt = dr.GradientDescentOptimizer(0.3) if opt_name == "sgd" else dr.AdagradOptimizer(0.3)
        for step in range(3):
            ind = np.stack([np.arange(B), np.zeros(B, np.int64)], 1)
            vals = [rng.integers(0, 200, B).astype(np.int64) for _ in range(F)]
            sps = [dr.SparseTensor(T(ind), T(v), (B, 1)) for v in vals]
            out = dr.embedding_lookup_sparse_multi(evs, sps, combiner="sum")
            g = rng.standard_normal((B, F * D)).astype(np.float32)
            for f in range(F):
                ref = orc.embedding_lookup_sparse(oevs[f], ind, vals[f], B, combiner="sum")
                np.testing.assert_array_equal(H(out)[:, f * D:(f + 1) * D], ref)
            out.backward(T(g))
            opt.apply_gradients(evs)
            for f in range(F):
                uids, idx = orc.unique(vals[f])
                gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g[:, f * D:(f + 1) * D]),
                                                    idx, np.arange(B, dtype=np.int32),
                                                    uids.shape[0], "sum")
                if opt_name == "sgd":
                    oevs[f].apply_sgd(0.3, gu, uids)
                else:
                    oevs[f].apply_adagrad(oacc[f], 0.3, gu, uids)
        for f in range(F):
            k, v = evs[f].export()[:2]
            ok, ov = oevs[f].export()[:2]
            np.testing.assert_array_equal(H(k), ok)
            np.testing.assert_array_equal(H(v), ov)


# ---------------------------------------------------------------------------
# interactions / exchange helpers
# ---------------------------------------------------------------------------
def test_fm2(ops, orc):
    rng = np.random.default_rng(31)
    e = rng.standard_normal((300, 26, 64)).astype(np.float32)
    out = H(ops.fm_second_order(T(e)))
    ref = orc.fm2(e)
    scale = 0.5 * (np.abs(e).sum(1) ** 2 + (e * e).sum(1))
    assert (np.abs(out - ref) <= 1e-5 * scale + 1e-6).all()


@pytest.mark.parametrize("F,D", [(5, 64), (26, 64), (40, 8), (3, 6)])
def test_fm2_grad(ops, orc, F, D):
    # register-resident kernel (F <= 8 / 32) and the scalar fallback (F > 32, D % 4)
    rng = np.random.default_rng(33)
    e = rng.standard_normal((97, F, D)).astype(np.float32)
    g = rng.standard_normal((97, D)).astype(np.float32)
    out = H(ops.fm_second_order_grad(T(e), T(g)))
    ref = (e.astype(np.float64).sum(1, keepdims=True) - e) * g[:, None, :]
    scale = np.abs(e).sum(1, keepdims=True) * np.abs(g)[:, None, :]
    assert (np.abs(out - ref) <= 1e-5 * scale + 1e-6).all()


@pytest.mark.parametrize("B,F,D", [(50, 27, 128), (9, 5, 16), (7, 2, 8), (5, 30, 64),
                                   (6, 27, 12), (33, 17, 32), (21, 16, 64), (11, 32, 128),
                                   (13, 27, 16), (4, 24, 96)])
def test_dot_interaction(ops, orc, B, F, D):
    # f32 MFMA kernel: F <= 32, D in {16, 32, 64, 128} (one or three 16x16
    # blocks: F = 16 / 17 / 32 are the edges); LDS-tiled kernel: nb(nb+1)/2
    # <= 32 tiles, D % 8 == 0 (D = 96); others: per-pair kernel
    rng = np.random.default_rng(37)
    x = rng.standard_normal((B, F, D)).astype(np.float32)
    out = H(ops.dot_interaction(T(x)))
    ref = orc.dot_interaction(x)
    scale = np.abs(x).sum(2).max() ** 2 / F
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5 * scale)


def test_crossnet_bf16(ops, orc):
    rng = np.random.default_rng(41)
    B, d = 200, 200
    bf = lambda a: torch.as_tensor(a, device=DEV).to(torch.bfloat16)
    x0 = bf(rng.standard_normal((B, d)).astype(np.float32))
    xl = bf(rng.standard_normal((B, d)).astype(np.float32))
    W = bf((rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32))
    b = torch.as_tensor(rng.standard_normal(d).astype(np.float32), device=DEV)
    out = ops.crossnet_layer(x0, xl, W, b).float()
    ref = orc.crossnet_layer(H(x0.float()), H(xl.float()), H(W.float()), H(b))
    err = np.abs(H(out) - ref)
    assert err.max() <= 2e-2 * np.abs(ref).max() + 1e-2


def test_partition_by_owner(ops):
    rng = np.random.default_rng(43)
    keys = rng.integers(0, 10 ** 9, 50000).astype(np.int64)
    for world in (1, 2, 4, 8):
        ko, perm, counts = ops.partition_by_owner(T(keys), world)
        owner = keys % world
        order = np.argsort(owner, kind="stable")
        np.testing.assert_array_equal(H(perm), order)
        np.testing.assert_array_equal(H(ko), keys[order])
        np.testing.assert_array_equal(H(counts), np.bincount(owner, minlength=world))
