"""The oracle's parallel Unique (ParallelComputeV1, unique_ali_op_util.h:
226-445, UniqueAliOp's default above kPartitionLimit) returns exactly the
serial first-occurrence Unique (SerialComputeV1, :192-222) -- keys and
indices -- for every pool size, including the section / task splits the
Partitioner makes uneven, empty and one-element inputs, all-equal keys and
keys repeated across every section.  Also the pooled cpu_baseline pipeline
against the per-stage oracle."""
import numpy as np
import pytest

from oracle import oracle as orc


@pytest.fixture(scope="module", params=[1, 2, 3, 5, 8])
def pool(request):
    p = orc.Pool(request.param)
    yield p
    p.close()


@pytest.mark.parametrize("n", [0, 1, 7, 14335, 14336, 20001, 65536])
@pytest.mark.parametrize("hi", [1, 3, 1000, 1 << 40])
def test_parallel_unique_equals_serial(pool, n, hi):
    rng = np.random.default_rng(n * 31 + pool.threads)
    x = rng.integers(0, hi, n).astype(np.int64)
    y0, i0 = orc.unique(x)
    y1, i1 = orc.unique_parallel(x, pool)
    assert np.array_equal(y0, y1)
    assert np.array_equal(i0, i1)


def test_parallel_unique_keys_spanning_sections(pool):
    # every section holds every key: all later maps defer to map 0
    x = np.tile(np.arange(997, dtype=np.int64)[::-1], 40)
    y0, i0 = orc.unique(x)
    y1, i1 = orc.unique_parallel(x, pool)
    assert np.array_equal(y0, y1) and np.array_equal(i0, i1)
    assert y1.shape[0] == 997


@pytest.mark.parametrize("serial", [0, 1])
def test_pooled_pipeline_matches_stages(pool, serial):
    D, R, B = 8, 5000, 20000
    rng = np.random.default_rng(7)
    ev = orc.EV(D, 0.0)
    keys = np.arange(R, dtype=np.int64)
    vals = rng.standard_normal((R, D), dtype=np.float32)
    ev.insert(keys, vals)
    ids = rng.integers(0, R + 100, B).astype(np.int64)   # some keys absent: default 0
    seg = np.arange(B + 1, dtype=np.int32)
    out = np.empty((B, D), np.float32)
    rc = orc.lib().orc_pipeline_ev_lookup_sparse_pool(pool._h, ev._h, orc._p(ids), B, orc._p(seg),
                                                      B, 0, serial, orc._p(out))
    assert rc == 0
    want = np.where((ids < R)[:, None], vals[np.minimum(ids, R - 1)], 0.0).astype(np.float32)
    assert np.array_equal(out, want)
