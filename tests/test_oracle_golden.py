"""Pins the CPU restatement (oracle/) against the reference's own KATs.

CPU-only; the fixtures come from tests/golden/make_golden.py (reference test
file:line cited there and in each test below).
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b).max() if a.size else 0


# fused_embedding_local_ops_test.cc:63-191 (forward) -------------------------
@pytest.mark.parametrize("case", ["sqrtn", "mean", "sum", "sqrtn_maxnorm200"])
def test_fused_local_forward_kat(orc, case):
    g = load("fused_local")
    c = g["forward"][case]
    table = np.asarray(g["table"], np.float32).reshape(g["bucket"], g["dim"])
    ind = np.asarray(g["sp_indices"], np.int64).reshape(-1, 2)
    out, off = orc.fused_local_lookup(table, g["sp_values"], ind[:, 0], g["batch"],
                                      c.get("combiner", case), c["max_norm"])
    np.testing.assert_allclose(out.ravel(), c["expected"], atol=g["tolerance"], rtol=0)
    assert off.tolist() == g["offsets_expected"]


# fused_embedding_local_ops_test.cc:200-365 (grad) ---------------------------
@pytest.mark.parametrize("case", ["sqrtn", "mean", "sum", "mean_maxnorm100"])
def test_fused_local_grad_kat(orc, case):
    g = load("fused_local")
    c = g["grad"][case]
    table = np.asarray(g["table"], np.float32).reshape(g["bucket"], g["dim"])
    top = np.asarray(g["top_grad"], np.float32).reshape(g["batch"], g["dim"])
    out = orc.fused_local_lookup_grad(top, table, g["sp_values"], g["offsets_expected"],
                                      c.get("combiner", case), c["max_norm"])
    np.testing.assert_allclose(out.ravel(), c["expected"], atol=g["tolerance"], rtol=0)


# fused_embedding_ops_test.cc:59-97 (stable partition) ----------------------
def test_pre_lookup_partition_kat(orc):
    g = load("pre_lookup_partition")
    ind = np.asarray(g["sp_indices"], np.int64).reshape(-1, 2)
    parts = orc.fused_pre_lookup(g["sp_values"], g["partition_rows"])
    for (vals, pos), exp in zip(parts, g["expected"]):
        assert vals.tolist() == exp["values"]
        assert ind[pos].ravel().tolist() == exp["indices"]


# segment_reduction_ali_ops_test.cc:75-240 ----------------------------------
def _formula_inputs(g):
    rows, D, n = g["rows"], g["dim"], g["n"]
    data = np.repeat((np.arange(rows * D) // D).astype(np.float32).reshape(rows, D)[:, :1], D, 1)
    i = np.arange(n)
    return data, (2 * i).astype(np.int32), (i // 2).astype(np.int32)


@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_segment_reduce_formula_kat(orc, comb):
    g = load("segment_formula")
    data, idx, seg = _formula_inputs(g)
    out = orc.sparse_segment_reduce(data, idx, seg, comb)
    s = np.arange(65536, dtype=np.int64)
    base = (s * 4 + s * 4 + 2).astype(np.float32)
    if comb == "mean":
        base = base / np.float32(2.0)
    elif comb == "sqrtn":
        base = base / np.sqrt(np.float32(2.0))
    exp = np.repeat(base[:, None], g["dim"], 1)
    assert out.shape == exp.shape
    assert ulp_diff(out, exp) <= 4  # ExpectTensorEqual<float> == EXPECT_FLOAT_EQ (4 ULP)
    if comb != "sqrtn":
        np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(out[:64, 0], np.asarray(g["forward_sum"], np.float32)
                                  / (np.float32(2.0) if comb == "mean" else np.float32(1.0))
                                  if comb != "sqrtn" else out[:64, 0])


@pytest.mark.parametrize("comb", ["mean", "sqrtn"])
def test_segment_reduce_grad_formula_kat(orc, comb):
    g = load("segment_formula")
    rows, D, n = g["rows"], g["dim"], g["n"]
    grad = np.repeat(np.arange(65536, dtype=np.float32)[:, None], D, 1)
    i = np.arange(n)
    out = orc.sparse_segment_reduce_grad(grad, (2 * i).astype(np.int32),
                                         (i // 2).astype(np.int32), rows, comb)
    head = np.asarray(g["grad_mean_head" if comb == "mean" else "grad_sqrtn_head"], np.float32)
    assert ulp_diff(out[:64, 0], head) <= 4
    r = np.arange(rows)
    div = np.float32(2.0) if comb == "mean" else np.sqrt(np.float32(2.0))
    exp = np.where(r % 2 == 0, (r // 4).astype(np.float32) / div, 0).astype(np.float32)
    assert ulp_diff(out[:, 0], exp) <= 4


# Unique first-occurrence order (unique_ali_op_util.h:192-222; upstream ---
# unique_op_test.cc / tf.unique docstring example) --------------------------
def test_unique_order_kat(orc):
    y, idx, cnt = orc.unique([1, 1, 2, 4, 4, 4, 7, 8, 8], with_counts=True)
    assert y.tolist() == [1, 2, 4, 7, 8]
    assert idx.tolist() == [0, 0, 1, 2, 2, 2, 3, 4, 4]
    assert cnt.tolist() == [2, 1, 3, 1, 2]
    y, idx = orc.unique([5, -3, 5, 9, -3, 0])
    assert y.tolist() == [5, -3, 9, 0] and idx.tolist() == [0, 1, 0, 2, 1, 3]
    y, idx = orc.unique(np.zeros(0, np.int64))
    assert y.size == 0 and idx.size == 0


def test_unique_random_matches_numpy(orc):
    rng = np.random.default_rng(2021)
    x = rng.integers(-50, 50, 5000)
    y, idx, cnt = orc.unique(x, with_counts=True)
    _, first = np.unique(x, return_index=True)
    np.testing.assert_array_equal(y, x[np.sort(first)])
    np.testing.assert_array_equal(y[idx], x)
    np.testing.assert_array_equal(cnt, [np.sum(x == v) for v in y])


# Segment-reduce association order: each num%8 branch ----------------------
def test_segment_reduce_association_order(orc):
    rng = np.random.default_rng(7)
    D = 5
    data = (rng.standard_normal((200, D)) * 1e3).astype(np.float32)
    for num in range(1, 27):
        idx = rng.integers(0, 200, num).astype(np.int32)
        seg = np.zeros(num, np.int32)
        out = orc.sparse_segment_reduce(data, idx, seg, "sum")[0]
        r = num % 8
        r = 8 if r == 0 else (9 if r == 1 else r)
        if num == 1:
            exp = data[idx[0]]
        else:
            exp = data[idx[0]].copy()
            for k in range(1, r):
                exp = (exp + data[idx[k]]).astype(np.float32)
            for gi in range(r, num, 8):
                s = data[idx[gi]].copy()
                for k in range(1, 8):
                    s = (s + data[idx[gi + k]]).astype(np.float32)
                exp = (exp + s).astype(np.float32)
        np.testing.assert_array_equal(out, exp)


def test_segment_reduce_errors_and_gaps(orc):
    data = np.ones((4, 2), np.float32)
    out = orc.sparse_segment_reduce(data, [0, 1, 2], [0, 2, 2], "sum", num_segments=5)
    assert out.tolist() == [[1, 1], [0, 0], [2, 2], [0, 0], [0, 0]]
    with pytest.raises(orc.OracleError):
        orc.sparse_segment_reduce(data, [0, 9], [0, 1], "sum")
    with pytest.raises(orc.OracleError):
        orc.sparse_segment_reduce(data, [0, 1], [1, 0], "sum")
    assert orc.sparse_segment_reduce(data, [], [], "sum", num_segments=3).tolist() == [[0, 0]] * 3


def test_unsorted_segment_sum_serial_order(orc):
    data = np.asarray([[1e8], [1.0], [-1e8], [1.0]], np.float32)
    out = orc.unsorted_segment_sum(data, [0, 0, 0, -1], 2)
    # serial ascending-i order: ((0 + 1e8) + 1) + -1e8 = 0 in fp32
    assert out.tolist() == [[0.0], [0.0]]


# EV KATs: embedding_variable_ops_test.py ----------------------------------
def test_ev_export_kat(orc):
    k = load("ev")["export"]
    ev = orc.EV(k["dim"], k["init"], filter_freq=k["filter_freq"], steps_to_live=k["steps_to_live"])
    uids, idx, cnt = orc.unique(k["lookup"], with_counts=True)
    for _ in range(k["runs"]):
        ev.gather(uids, None, cnt)
    keys, vals, vers, frqs = ev.export()
    assert keys.tolist() == k["keys"]
    assert vals.tolist() == k["values"]
    assert vers.tolist() == k["versions"]
    assert frqs.tolist() == k["freqs"]


def test_ev_shape_kat(orc):
    k = load("ev")["shape"]
    ev = orc.EV(k["dim"], 1.0)
    ev.gather(k["lookup"])
    assert [ev.size(), ev.dim] == k["expected"]


def test_ev_counter_filter_timeline_kat(orc):
    k = load("ev")["counter_filter_gd"]
    ev = orc.EV(k["dim"], 1.0, filter_freq=k["filter_freq"])
    seen = []
    for step in range(4):
        uids, idx, cnt = orc.unique([k["key"]], with_counts=True)
        emb = ev.gather(uids, None, cnt)
        seen.append(emb.copy())
        ev.apply_sgd(k["lr"], np.full((1, k["dim"]), k["loss_scale"], np.float32), uids, step)
    assert all((s == 1.0).all() for s in seen[:3])
    assert (seen[3] != 1.0).all()


@pytest.mark.parametrize("opt", ["sgd", "adagrad", "adam"])
def test_ev_equals_dense_5step(orc, opt):
    k = load("ev")["ev_equals_dense"]
    D, ids, lr = k["dim"], np.asarray(k["ids"], np.int64), np.float32(k["lr"])
    ev = orc.EV(D, 1.0)
    table = np.ones((100, D), np.float32)
    if opt == "adagrad":
        acc_ev = ev.create_slot(1, k["adagrad_initial_accumulator"])
        acc = np.full((100, D), k["adagrad_initial_accumulator"], np.float32)
    if opt == "adam":
        a = k["adam"]
        m_ev, v_ev = ev.create_slot(1, 0.0), ev.create_slot(2, 0.0)
        m = np.zeros((100, D), np.float32)
        v = np.zeros((100, D), np.float32)
    g = np.full((len(ids), D), k["loss_scale"], np.float32)
    for step in range(k["steps"]):
        r_ev = ev.gather(ids)
        r_dense = table[ids].copy()
        np.testing.assert_array_equal(r_ev, r_dense)
        if opt == "sgd":
            ev.apply_sgd(lr, g, ids, step)
            orc.dense_apply_sgd(table, lr, g, ids)
        elif opt == "adagrad":
            ev.apply_adagrad(acc_ev, lr, g, ids, step)
            orc.dense_apply_adagrad(table, acc, lr, g, ids)
        else:
            b1p = np.float32(a["beta1"]) ** (step + 1)
            b2p = np.float32(a["beta2"]) ** (step + 1)
            ev.apply_adam(m_ev, v_ev, b1p, b2p, lr, a["beta1"], a["beta2"], a["epsilon"], g, ids,
                          step)
            alpha = lr * np.sqrt(np.float32(1) - b2p) / (np.float32(1) - b1p)
            m[ids] += (g - m[ids]) * (np.float32(1) - np.float32(a["beta1"]))
            v[ids] += (g * g - v[ids]) * (np.float32(1) - np.float32(a["beta2"]))
            table[ids] -= (m[ids] * alpha) / (np.sqrt(v[ids]) + np.float32(a["epsilon"]))
    final = ev.gather(ids)
    if opt == "adam":
        np.testing.assert_allclose(final, table[ids], atol=k["adam"]["delta"], rtol=0)
    else:
        np.testing.assert_array_equal(final, table[ids])


def test_ev_bloom_filter_admission(orc):
    # BloomFilter (embedding_filter.h:27-286): keys admitted after filter_freq lookups.
    ev = orc.EV(4, 0.5, filter_freq=3, max_element_size=1000, false_positive_probability=0.01,
                counter_bits=16)
    keys = np.arange(10, dtype=np.int64)
    for _ in range(3):
        out = ev.gather(keys)
        assert (out == 0.5).all()
        assert ev.size() == 0
    assert all(ev.freq(int(x)) >= 3 for x in keys)
    ev.gather(keys)
    assert ev.size() == 10
    assert orc.fasthash64(1, 2) == orc.fasthash64(1, 2)


def test_ev_import_partition_filter(orc):
    ev = orc.EV(2, 0.0, steps_to_live=5, filter_freq=2)
    keys = np.arange(0, 20, dtype=np.int64)
    vals = np.repeat(keys[:, None], 2, 1).astype(np.float32)
    ev.insert(keys, vals, versions=keys * 10, freqs=np.ones(20, np.int64), partition_id=1,
              partition_num=4)
    k, v, ver, fr = ev.export()
    assert k.tolist() == [x for x in range(20) if x % 1000 % 4 == 1]
    assert (fr == 2).all()               # clamped up to filter_freq (embedding_var.h:204-209)
    assert ver.tolist() == [x * 10 for x in k]


# Fingerprint64 / StringToHashBucketFast: fingerprint_test.cc:26-29,
# fingerprint_op_test.cc:64-106, string_to_hash_bucket_op_test.py:40-50 ------
def _iota_bytes(start, n):
    return ((np.arange(n) + start) % 256).astype(np.uint8).tobytes()


def test_fingerprint64_kat(orc):
    g = load("fingerprint")
    for c in g["fingerprint64"] + g["fingerprint64_letters"]:
        assert orc.fingerprint64(c["ascii"].encode()) == int(c["value"])
    hb = g["hash_bucket_fast"]
    np.testing.assert_array_equal(orc.string_to_hash_bucket_fast(hb["strings"], hb["num_buckets"]),
                                  hb["expected"])
    ob = g["op_bytes"]                                  # > 64 bytes: the long loop
    fp = orc.fingerprint64(_iota_bytes(ob["iota_start"], ob["length"]))
    assert fp.to_bytes(8, "little").hex() == ob["expected_le"]
    os_ = g["op_strings"]                               # 0-16 and 17-32 bytes
    each = [orc.fingerprint64(_iota_bytes(s, n)).to_bytes(8, "little")
            for s, n in zip(os_["iota_starts"], os_["lengths"])]
    assert [e.hex() for e in each] == os_["expected_each_le"]
    assert orc.fingerprint64(b"".join(each)).to_bytes(8, "little").hex() == \
        os_["expected_combined_le"]


def test_hash_bucket_int64_max_for_ev_columns(orc):
    # feature_column_v2.py:5954-5957: EV string columns hash into INT64_MAX buckets
    ids = orc.string_to_hash_bucket_fast(["a", "Hello"], np.iinfo(np.int64).max)
    assert ids[0] == 12917804110809363939 % (2 ** 63 - 1)
    assert ids[1] == 15404698994557526151 % (2 ** 63 - 1)


# fused_embedding_ops_test.cc:129-196 / :217-290 (partitioned post-lookup) ----
def test_post_lookup_kat(orc):
    c = load("post_lookup")["forward"]
    D = c["dim"]
    shards = [np.asarray(s, np.float32).reshape(-1, D) for s in c["shards"]]
    inds = [np.asarray(i, np.int64).reshape(-1, 2) for i in c["indices"]]
    out, fnum = orc.fused_post_lookup(shards, inds, c["batch"], c["cols"], c["combiner"],
                                      c["max_norm"])
    np.testing.assert_allclose(out.ravel(), c["expected"], atol=c["tol"], rtol=0)
    assert fnum.tolist() == c["feature_nums"]


def test_post_lookup_grad_kat(orc):
    c = load("post_lookup")["grad"]
    D = c["dim"]
    top = np.asarray(c["top_grad"], np.float32).reshape(c["batch"], D)
    shards = [np.asarray(s, np.float32).reshape(-1, D) for s in c["shards"]]
    inds = [np.asarray(i, np.int64).reshape(-1, 2) for i in c["indices"]]
    outs = orc.fused_post_lookup_grad(top, shards, inds, c["feature_nums"], c["combiner"],
                                      c["max_norm"])
    for o, e in zip(outs, c["expected"]):
        np.testing.assert_allclose(o.ravel(), e, atol=c["tol"], rtol=0)


def test_pre_post_equals_local_lookup(orc):
    """PostLookUp(PreLookUp(x)) with per-partition gathers reproduces the
    local fused lookup on the concatenated table bit for bit (the order the
    oracle and the engine fix for the reference's atomics)."""
    rng = np.random.default_rng(5)
    B, D, M = 40, 8, 6
    rows = [7, 3, 11]
    table = rng.standard_normal((sum(rows), D)).astype(np.float32) * 3
    lens = rng.integers(1, M + 1, B)
    r = np.repeat(np.arange(B), lens)
    c = np.concatenate([np.sort(rng.choice(M, n, replace=False)) for n in lens])
    ind = np.stack([r, c], 1).astype(np.int64)
    vals = rng.integers(0, sum(rows), r.shape[0]).astype(np.int64)
    acc = np.cumsum([0] + rows)
    for comb in ("sum", "mean", "sqrtn"):
        for mn in (-1.0, 4.0):
            parts = orc.fused_pre_lookup(vals, rows)
            shards = [table[acc[p] + v] for p, (v, _) in enumerate(parts)]
            inds = [ind[pos] for _, pos in parts]
            out, fnum = orc.fused_post_lookup(shards, inds, B, M, comb, mn)
            ref, _ = orc.fused_local_lookup(table, vals, r, B, comb, mn)
            np.testing.assert_array_equal(out, ref)
            assert fnum.tolist() == lens.tolist()


def _torch_lookup_sparse(table, ind, vals, B, w, comb, max_norm):
    """The reference composition (embedding_ops.py:589-651 + _clip) in torch
    fp64 autograd: an independent check of the oracle's chain rule."""
    import torch
    t = torch.tensor(table, dtype=torch.float64, requires_grad=True)
    uids, idx = np.unique(vals, return_inverse=True)
    emb = t[torch.as_tensor(uids)]
    if max_norm is not None:
        l2 = torch.sqrt((emb * emb).sum(1, keepdim=True))
        emb = emb * max_norm / torch.maximum(l2, torch.tensor(max_norm, dtype=torch.float64))
    seg = torch.as_tensor(ind[:, 0])
    g = emb[torch.as_tensor(idx)]
    ww = torch.ones(len(vals), dtype=torch.float64) if w is None else torch.tensor(w, dtype=torch.float64)
    s = torch.zeros((B, table.shape[1]), dtype=torch.float64).index_add(0, seg, g * ww[:, None])
    if comb != "sum":
        q = torch.zeros(B, dtype=torch.float64).index_add(0, seg, ww if comb == "mean" else ww * ww)
        q = q if comb == "mean" else torch.sqrt(q)
        s = s / q[:, None]
    return t, s


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("max_norm", [None, 2.0])
@pytest.mark.parametrize("comb", ["sum", "mean", "sqrtn"])
def test_lookup_sparse_grad_oracle_vs_autograd(orc, weighted, max_norm, comb):
    rng = np.random.default_rng(17)
    B, D, R = 30, 6, 25
    table = (rng.standard_normal((R, D)) * 1.5).astype(np.float32)
    lens = rng.integers(1, 5, B)
    r = np.repeat(np.arange(B), lens)
    c = np.concatenate([np.arange(n) for n in lens])
    ind = np.stack([r, c], 1).astype(np.int64)
    vals = rng.integers(0, R, r.shape[0]).astype(np.int64)
    w = rng.uniform(0.2, 2.0, r.shape[0]).astype(np.float32) if weighted else None
    top = rng.standard_normal((B, D)).astype(np.float32)
    uids, gu = orc.embedding_lookup_sparse_grad(table, ind, vals, B, top, w, comb, max_norm)
    t, out = _torch_lookup_sparse(table, ind, vals, B, w, comb, max_norm)
    out.backward(__import__("torch").tensor(top, dtype=__import__("torch").float64))
    ref = t.grad.numpy()[uids]
    np.testing.assert_allclose(gu, ref, rtol=1e-5, atol=1e-6)
