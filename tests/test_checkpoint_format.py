"""TensorBundle format and DeepRec's EV checkpoint layout, on CPU.

* The writer reproduces two checkpoints from the reference's own testdata
  byte for byte (tests/golden/ckpt/: python/feature_column/testdata/
  embedding.ckpt, contrib/framework/testdata/bundle_checkpoint), and the
  reader returns the values the reference's tests expect
  (feature_column_v2_test.py:7948-7953).
* The oracle's DumpEmbeddingValues layout (kv_variable_ops.h:148-265) gives
  the tensor names / shapes the reference's EV save tests check
  (core/kernels/embedding_variable_ops_test.cc:195-330).
"""
import os
import tempfile

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ckpt")


@pytest.fixture(scope="module")
def ck():
    from deeprec_amd import checkpoint
    return checkpoint


@pytest.mark.parametrize("name", ["embedding.ckpt", "bundle_checkpoint"])
def test_writer_is_byte_exact_with_reference_testdata(ck, name, tmp_path):
    pre = os.path.join(GOLD, name)
    r = ck.BundleReader(pre)
    w = ck.BundleWriter(str(tmp_path / "x"))
    for k in sorted(r.keys(), key=lambda k: r.entries[k]["offset"]):
        w.add(k, r.lookup(k))
    w.finish()
    for suf in (".index", ".data-00000-of-00001"):
        assert open(str(tmp_path / "x") + suf, "rb").read() == open(pre + suf, "rb").read()


def test_reader_values_match_reference_test(ck):
    r = ck.BundleReader(os.path.join(GOLD, "embedding.ckpt"))
    assert r.keys() == ["my_embedding"]
    np.testing.assert_array_equal(r.lookup("my_embedding"), [[1., 2.], [3., 5.], [7., 11.]])
    r2 = ck.BundleReader(os.path.join(GOLD, "bundle_checkpoint"))
    assert r2.dtype_and_shape("some_scope/embeddings") == (np.dtype(np.float32), (5, 16))
    assert r2.dtype_and_shape("some_scope/indices") == (np.dtype(np.int64), (5,))


def test_multi_block_index_round_trip(ck, tmp_path):
    rng = np.random.default_rng(3)
    arrays = {}
    w = ck.BundleWriter(str(tmp_path / "m"), block_size=256)    # many blocks
    for i in range(300):
        name = "scope_%03d/var_%d" % (i % 37, i)
        a = rng.standard_normal((i % 5, 3)).astype(np.float32) if i % 2 else \
            rng.integers(-9, 9, i % 7).astype(np.int64)
        arrays[name] = a
        w.add(name, a)
    w.finish()
    r = ck.BundleReader(str(tmp_path / "m"))
    assert r.keys() == sorted(arrays)
    for k, a in arrays.items():
        np.testing.assert_array_equal(r.lookup(k), a)
        assert r.lookup(k).dtype == a.dtype


def test_corruption_is_detected(ck, tmp_path):
    w = ck.BundleWriter(str(tmp_path / "c"))
    w.add("v", np.arange(10, dtype=np.float32))
    w.finish()
    p = str(tmp_path / "c") + ".data-00000-of-00001"
    b = bytearray(open(p, "rb").read())
    b[5] ^= 1
    open(p, "wb").write(bytes(b))
    import deeprec_amd
    with pytest.raises(deeprec_amd.DeepRecError):
        ck.BundleReader(str(tmp_path / "c")).lookup("v")


def test_duplicate_key_rejected(ck, tmp_path):
    import deeprec_amd
    w = ck.BundleWriter(str(tmp_path / "d"))
    w.add("a", np.zeros(1, np.int64))
    with pytest.raises(deeprec_amd.InvalidArgumentError):
        w.add("a", np.zeros(1, np.int64))


def test_ev_dump_layout_kats(orc, ck, tmp_path):
    # TestEmptyEV (embedding_variable_ops_test.cc:195-259): five tensors, empty
    offs, k, v, ve, fr = orc.dump_embedding_values(np.zeros(0, np.int64),
                                                   np.zeros((0, 8), np.float32),
                                                   np.zeros(0, np.int64), np.zeros(0, np.int64))
    w = ck.BundleWriter(str(tmp_path / "e"))
    ck.write_ev_tensors(w, "var/part_0", offs, k, v, ve, fr)
    w.finish()
    r = ck.BundleReader(str(tmp_path / "e"))
    assert r.keys() == ["var/part_0-freqs", "var/part_0-keys", "var/part_0-partition_offset",
                        "var/part_0-values", "var/part_0-versions"]
    assert r.dtype_and_shape("var/part_0-values")[1] == (0, 8)
    assert r.dtype_and_shape("var/part_0-partition_offset") == (np.dtype(np.int32), (1001,))
    # TestEVExportSmall (:261-330): keys 0..4, value 9 with column i = 5,
    # steps_to_live 5 -> versions saved, no filter -> freqs empty
    ev = orc.EV(8, 9.0, steps_to_live=5)
    vals = np.full((5, 8), 9.0, np.float32)
    vals[np.arange(5), np.arange(5)] = 5.0
    ev.insert(np.arange(5), vals)
    keys, vv, vers, _ = ev.export()
    offs, k, v, ve, fr = orc.dump_embedding_values(keys, vv, vers, np.zeros(0, np.int64))
    w = ck.BundleWriter(str(tmp_path / "s"))
    ck.write_ev_tensors(w, "var/part_0", offs, k, v, ve, fr)
    w.finish()
    r = ck.BundleReader(str(tmp_path / "s"))
    np.testing.assert_array_equal(r.lookup("var/part_0-keys"), np.arange(5))
    np.testing.assert_array_equal(r.lookup("var/part_0-values"), vals)
    assert r.dtype_and_shape("var/part_0-versions")[1] == (5,)
    assert r.dtype_and_shape("var/part_0-freqs")[1] == (0,)
    po = r.lookup("var/part_0-partition_offset")
    np.testing.assert_array_equal(po[:7], [0, 1, 2, 3, 4, 5, 5])
    assert po[-1] == 5


def test_ev_dump_partitions_by_key_mod_1000(orc):
    keys = np.array([2001, -3, 5, 1005, 999, 2005, 1, -1000], np.int64)
    vals = np.arange(8 * 2, dtype=np.float32).reshape(8, 2)
    offs, k, v, _, _ = orc.dump_embedding_values(keys, vals, np.zeros(0), np.zeros(0))
    np.testing.assert_array_equal(k, [2001, 1, 5, 1005, 2005, 999])   # negatives dropped
    assert offs[1] == 0 and offs[2] == 2 and offs[5] == 2 and offs[6] == 5 and offs[1000] == 6
    np.testing.assert_array_equal(v[0], vals[0])
