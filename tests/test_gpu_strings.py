"""String -> id on the GPU (dr_fingerprint64 / dr_string_to_hash_bucket_fast)
against the reference's golden fingerprints and the oracle's restatement
(bit-exact: integer work)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fingerprint.json")


def _iota(start, n):
    return ((np.arange(n) + start) % 256).astype(np.uint8).tobytes()


def _u64(t):
    return [int(x) & 0xFFFFFFFFFFFFFFFF for x in t.cpu().numpy().tolist()]


def test_fingerprint_goldens():
    from deeprec_amd import string_ops as so
    g = json.load(open(GOLD))
    cases = g["fingerprint64"] + g["fingerprint64_letters"]
    got = _u64(so.fingerprint64([c["ascii"] for c in cases]))
    assert got == [int(c["value"]) for c in cases]
    hb = g["hash_bucket_fast"]
    out = so.string_to_hash_bucket_fast(hb["strings"], hb["num_buckets"]).cpu().tolist()
    assert out == hb["expected"]
    ob = g["op_bytes"]
    fp = _u64(so.fingerprint64([_iota(ob["iota_start"], ob["length"])]))[0]
    assert fp.to_bytes(8, "little").hex() == ob["expected_le"]
    os_ = g["op_strings"]
    each = _u64(so.fingerprint64([_iota(s, n) for s, n in zip(os_["iota_starts"],
                                                              os_["lengths"])]))
    assert [e.to_bytes(8, "little").hex() for e in each] == os_["expected_each_le"]
    comb = b"".join(e.to_bytes(8, "little") for e in each)
    assert _u64(so.fingerprint64([comb]))[0].to_bytes(8, "little").hex() == \
        os_["expected_combined_le"]


@pytest.mark.parametrize("maxlen", [16, 70, 300])
def test_hash_bucket_random_matches_oracle(maxlen):
    from oracle import oracle as orc
    from deeprec_amd import string_ops as so
    rng = np.random.default_rng(maxlen)
    n = 5000
    lens = rng.integers(0, maxlen + 1, n)
    lens[:130] = np.arange(130) % (maxlen + 1)        # every length class incl. 0
    strings = [rng.integers(0, 256, int(k)).astype(np.uint8).tobytes() for k in lens]
    for nb in (10, 1000003, np.iinfo(np.int64).max):
        got = so.string_to_hash_bucket_fast(strings, nb).cpu().numpy()
        np.testing.assert_array_equal(got, orc.string_to_hash_bucket_fast(strings, nb))
    fp = _u64(so.fingerprint64(strings))
    assert fp == [orc.fingerprint64(s) for s in strings]


def test_strings_at_unaligned_buffer_end():
    """A string ending on the last byte of an odd-sized device buffer."""
    from oracle import oracle as orc
    from deeprec_amd import string_ops as so
    raw = bytes(range(1, 52))                           # 51 bytes
    data = torch.as_tensor(np.frombuffer(raw, np.uint8).copy(), device="cuda")
    offs = torch.as_tensor([0, 3, 20, 51, 51], dtype=torch.int64, device="cuda")
    st = so.StringTensor(data, offs)
    got = _u64(so.fingerprint64(st))
    want = [orc.fingerprint64(raw[a:b]) for a, b in ((0, 3), (3, 20), (20, 51), (51, 51))]
    assert got == want


def test_ev_string_column_ids_feed_lookup():
    """EV string column: ids = Fingerprint64 % INT64_MAX, then the lookup."""
    import deeprec_amd as dr
    from oracle import oracle as orc
    from deeprec_amd import string_ops as so
    words = ["user_%d" % (i % 37) for i in range(200)]
    ids = so.ev_string_ids(words)
    ref_ids = orc.string_to_hash_bucket_fast(words, np.iinfo(np.int64).max)
    np.testing.assert_array_equal(ids.cpu().numpy(), ref_ids)
    ev = dr.EmbeddingVariable("strcol", 8, 0.5)
    ind = torch.stack([torch.arange(200, device="cuda"), torch.zeros(200, dtype=torch.int64,
                                                                     device="cuda")], 1)
    out = dr.embedding_lookup_sparse(ev, dr.SparseTensor(ind, ids, (200, 1)), combiner="sum")
    oev = orc.EV(8, 0.5)
    ref = orc.embedding_lookup_sparse(oev, ind.cpu().numpy(), ref_ids, 200, combiner="sum")
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref)


def test_bad_offsets_latch_invalid_argument():
    import deeprec_amd as dr
    from deeprec_amd import string_ops as so
    data = torch.zeros(8, dtype=torch.uint8, device="cuda")
    offs = torch.as_tensor([0, 5, 2], dtype=torch.int64, device="cuda")
    with pytest.raises(dr.InvalidArgumentError):   # at the op (validate mode) or the check
        so.fingerprint64(so.StringTensor(data, offs))
        dr.status_check()
