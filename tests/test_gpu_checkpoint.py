"""EV save / restore in DeepRec's checkpoint layout with the GPU engine.

Save: dr_ev_export + the 1000-way key % 1000 split on the device must give
the oracle's DumpEmbeddingValues arrays (kv_variable_ops.h:148-265) for the
same snapshot, bit for bit.  Restore (EVRestoreDynamically,
kv_variable_ops.h:459-673) into partition_num shards must equal the oracle EV
importing every saved entry through EmbeddingVar::Import's partition filter
(embedding_var.h:187-219).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _make_ev(dr, name, dim, n, seed, **kw):
    rng = np.random.default_rng(seed)
    keys = np.unique(rng.integers(-50, 200000, n)).astype(np.int64)
    rng.shuffle(keys)
    vals = rng.standard_normal((keys.shape[0], dim)).astype(np.float32)
    ev = dr.EmbeddingVariable(name, dim, 0.5, device=DEV, **kw)
    vers = rng.integers(0, 100, keys.shape[0]).astype(np.int64)
    ev.insert(torch.as_tensor(keys, device=DEV), torch.as_tensor(vals, device=DEV),
              torch.as_tensor(vers, device=DEV))
    return ev


@pytest.mark.parametrize("steps_to_live", [0, 7])
def test_save_layout_matches_oracle_dump(tmp_path, steps_to_live):
    import deeprec_amd as dr
    from deeprec_amd import checkpoint as ck
    from oracle import oracle as orc
    ev = _make_ev(dr, "ck_save_%d" % steps_to_live, 16, 3000, 1, steps_to_live=steps_to_live)
    keys, vals, vers, frqs = [x.cpu().numpy() for x in ev.export()]
    pre = str(tmp_path / "model.ckpt-1")
    ck.save(pre, {"emb/part_0": ev})
    r = ck.BundleReader(pre)
    offs, k, v, ve, fr = orc.dump_embedding_values(keys, vals, vers, frqs)
    np.testing.assert_array_equal(r.lookup("emb/part_0-partition_offset"), offs)
    np.testing.assert_array_equal(r.lookup("emb/part_0-keys"), k)
    np.testing.assert_array_equal(r.lookup("emb/part_0-values"), v)
    np.testing.assert_array_equal(r.lookup("emb/part_0-versions"), ve)
    np.testing.assert_array_equal(r.lookup("emb/part_0-freqs"), fr)
    assert (r.lookup("emb/part_0-keys") >= 0).all()
    assert r.dtype_and_shape("emb/part_0-versions")[1] == ((k.shape[0],) if steps_to_live else (0,))


@pytest.mark.parametrize("partition_num", [1, 3])
def test_restore_repartitions_like_import(tmp_path, partition_num):
    import deeprec_amd as dr
    from deeprec_amd import checkpoint as ck
    from oracle import oracle as orc
    # two saved parts (a job that ran with 2 partitions)
    evs = [_make_ev(dr, "ck_src_%d_%d" % (partition_num, p), 8, 2000, 10 + p, steps_to_live=3)
           for p in range(2)]
    pre = str(tmp_path / "m")
    ck.save(pre, {"scope/emb/part_%d/x" % p: evs[p] for p in range(2)})
    r = ck.BundleReader(pre)
    allk = np.concatenate([r.lookup("scope/emb/part_%d/x-keys" % p) for p in range(2)])
    allv = np.concatenate([r.lookup("scope/emb/part_%d/x-values" % p) for p in range(2)])
    allve = np.concatenate([r.lookup("scope/emb/part_%d/x-versions" % p) for p in range(2)])
    for pid in range(partition_num):
        ev = dr.EmbeddingVariable("ck_dst_%d_%d" % (partition_num, pid), 8, 0.5, device=DEV,
                                  steps_to_live=3)
        ck.restore_embedding_variable(ev, r, "scope/emb/part_%d/x" % pid, pid, partition_num)
        ref = orc.EV(8, 0.5, steps_to_live=3)
        ref.insert(allk, allv, allve, None, pid, partition_num)
        rk, rv, rve, _ = ref.export()
        k, v, ve, _ = [x.cpu().numpy() for x in ev.export()]
        o, ro = np.argsort(k), np.argsort(rk)
        np.testing.assert_array_equal(k[o], rk[ro])
        np.testing.assert_array_equal(v[o], rv[ro])
        np.testing.assert_array_equal(ve[o], rve[ro])
        assert np.all(k % 1000 % partition_num == pid)


def test_restore_without_partition_and_counter_filter(tmp_path):
    import deeprec_amd as dr
    from deeprec_amd import checkpoint as ck
    opt = dr.EmbeddingVariableOption(filter_option=dr.CounterFilter(filter_freq=3))
    ev = dr.EmbeddingVariable("ck_cf", 4, 0.25, ev_option=opt, device=DEV)
    ids = torch.as_tensor(np.array([5, 5, 5, 9, 9, 11, 5, 9, 9], np.int64), device=DEV)
    for i in range(ids.numel()):
        ev.sparse_read(ids[i:i + 1])
    keys, vals, _, frqs = [x.cpu().numpy() for x in ev.export()]
    pre = str(tmp_path / "f")
    ck.save(pre, {"emb": ev})
    r = ck.BundleReader(pre)
    assert r.dtype_and_shape("emb-freqs")[1] == (keys.shape[0],)
    ev2 = dr.EmbeddingVariable("ck_cf2", 4, 0.25, ev_option=opt, device=DEV)
    ck.restore(pre, {"emb": ev2})
    k2, v2, _, f2 = [x.cpu().numpy() for x in ev2.export()]
    o, o2 = np.argsort(keys), np.argsort(k2)
    np.testing.assert_array_equal(keys[o], k2[o2])
    np.testing.assert_array_equal(vals[o], v2[o2])
    # Import clamps freqs up to filter_freq (embedding_var.h:204-209)
    np.testing.assert_array_equal(np.maximum(frqs[o], 3), f2[o2])


def test_restore_missing_values_is_not_found(tmp_path):
    """A new-form part with -keys but no -values fails with NotFound (the
    reference's LookupHeader status; EVRestoreDynamically treats it as
    fatal) instead of leaving the EV half restored."""
    import deeprec_amd as dr
    from deeprec_amd import checkpoint as ck
    pre = str(tmp_path / "m")
    w = ck.BundleWriter(pre)
    w.add("emb/part_0/x-keys", np.array([1, 2], np.int64))
    w.add("emb/part_0/x-partition_offset", np.zeros(1001, np.int32))
    w.finish()
    ev = dr.EmbeddingVariable("ck_missing", 4, 0.5, device=DEV)
    with pytest.raises(dr.DeepRecError) as e:
        ck.restore_embedding_variable(ev, ck.BundleReader(pre), "emb/part_0/x", 0, 1)
    assert e.value.code == 5
    assert int(ev.total_count()[0]) == 0
