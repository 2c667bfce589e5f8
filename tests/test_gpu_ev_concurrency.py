"""GPU: the reference's multi-thread EmbeddingVar invariants
(core/kernels/embedding_variable_ops_test.cc), restated for the device EV.

TestMultiInsertion (:554-590): THREADNUM threads LookupOrCreate keys 0..4 of
one EV at once -> Size() == 5, the snapshot holds 5 keys, and every row is
the initial value (9.0).  TestInsertAndLookup (:920-965): threads insert
disjoint random key sets concurrently, then every key looks up its own value
(InsertAndLookup, :892-918) and Size() counts them all.

Here each host thread issues on its own HIP stream (torch's current stream
is per thread), so the kernels of different threads run concurrently on the
device: the CAS insert is the only arbitration, as the lockless map's CAS is
in the reference.
"""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
THREADNUM = 16


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    assert torch.cuda.is_available()
    return deeprec_amd


def _in_threads(fn, n):
    errs = []

    def run(i):
        try:
            s = torch.cuda.Stream(device=DEV)
            with torch.cuda.stream(s):
                fn(i)
            s.synchronize()
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    if errs:
        raise errs[0]
    torch.cuda.synchronize()


def test_multi_insertion_lookup_or_create(dr):
    D = 128
    for rep in range(3):
        ev = dr.EmbeddingVariable("mtins_%d" % rep, D, 9.0)
        keys = torch.arange(5, dtype=torch.int64, device=DEV)
        outs = [None] * THREADNUM

        def work(i):
            for _ in range(5):
                outs[i] = ev.sparse_read(keys)

        _in_threads(work, THREADNUM)
        dr.status_check()
        assert ev.total_count().tolist() == [5, D]
        k, v = ev.export()[:2]
        assert sorted(k.cpu().tolist()) == [0, 1, 2, 3, 4]
        assert bool((v == 9.0).all())
        for o in outs:
            assert bool((o == 9.0).all())


def test_insert_and_lookup_disjoint_threads(dr):
    D = 16
    rng = np.random.default_rng(7)
    loops = 1000 * THREADNUM // 16 * 16
    keys = rng.choice(1 << 40, size=loops, replace=False).astype(np.int64)
    vals = (keys[:, None] % 9973).astype(np.float32) + np.arange(D, dtype=np.float32)[None, :]
    ev = dr.EmbeddingVariable("mtlookup", D, 0.0, capacity=1024)   # grows while threads insert
    per = loops // THREADNUM
    got = [None] * THREADNUM

    def work(i):
        k = torch.as_tensor(keys[i * per:(i + 1) * per], device=DEV)
        ev.insert(k, torch.as_tensor(vals[i * per:(i + 1) * per], device=DEV))
        got[i] = ev.sparse_read(k).cpu().numpy()

    _in_threads(work, THREADNUM)
    dr.status_check()
    assert ev.total_count().tolist() == [loops, D]
    for i in range(THREADNUM):
        np.testing.assert_array_equal(got[i], vals[i * per:(i + 1) * per])
    # and all of them from the default stream afterwards
    np.testing.assert_array_equal(ev.sparse_read(torch.as_tensor(keys, device=DEV)).cpu().numpy(),
                                  vals)


def test_overlapping_lookup_or_create_while_growing(dr):
    """16 threads LookupOrCreate overlapping key sets (each key drawn by ~4
    threads, in different orders) on an EV that starts with room for 256
    keys: every key gets exactly one row (Size = distinct keys, export = the
    distinct keys).  Then 16 threads Import overlapping sets into a second
    growing EV, every writer with the same value f(key) -- Import keeps the
    first row it finds (LookupOrCreateEmb, embedding_var.h:187-219), so
    whichever insert wins, every key reads f(key) from every thread."""
    D = 32
    rng = np.random.default_rng(11)
    universe = rng.choice(1 << 50, size=8000, replace=False).astype(np.int64)
    picks = [rng.permutation(universe)[:2000] for _ in range(THREADNUM)]
    ev = dr.EmbeddingVariable("mtover", D, 0.5, capacity=256)

    def work(i):
        k = torch.as_tensor(picks[i], device=DEV)
        for chunk in torch.split(k, 500):
            out = ev.sparse_read(chunk)
            assert bool((out == 0.5).all())

    _in_threads(work, THREADNUM)
    dr.status_check()
    distinct = np.unique(np.concatenate(picks))
    assert ev.total_count().tolist() == [distinct.size, D]
    k = ev.export()[0].cpu().numpy()
    np.testing.assert_array_equal(np.sort(k), distinct)

    def f(keys):
        return (keys[:, None] % 997).astype(np.float32) + np.arange(D, dtype=np.float32)[None, :]

    ev2 = dr.EmbeddingVariable("mtover2", D, 0.5, capacity=256)

    def imp(i):
        for chunk in np.array_split(picks[i], 4):
            ev2.insert(torch.as_tensor(chunk, device=DEV), torch.as_tensor(f(chunk), device=DEV))

    _in_threads(imp, THREADNUM)
    dr.status_check()
    assert ev2.total_count().tolist() == [distinct.size, D]
    got = [None] * THREADNUM

    def read(i):
        got[i] = ev2.sparse_read(torch.as_tensor(picks[i], device=DEV)).cpu().numpy()

    _in_threads(read, THREADNUM)
    for i in range(THREADNUM):
        np.testing.assert_array_equal(got[i], f(picks[i]))
    assert ev2.total_count().tolist() == [distinct.size, D]


def test_disjoint_threads_fill_to_growth_limit(dr):
    """Capacity accounting across streams (the mirror of the device row count
    is taken on one stream; adds reserved on other streams may not have run
    yet): 16 threads, one stream each, LookupOrCreate disjoint keys in many
    small calls, every call bringing the EV to or just past its growth limit,
    so that a count that forgot another stream's pending adds would skip a
    growth and latch RESOURCE_EXHAUSTED (the key served the default forever).
    Every key must get its own row and the status word must stay clean."""
    D = 16
    rng = np.random.default_rng(23)
    per, calls = 96, 24
    keys = rng.choice(1 << 45, size=THREADNUM * per * calls, replace=False).astype(np.int64)
    for rep in range(2):
        ev = dr.EmbeddingVariable("mtfill_%d" % rep, D, 0.25, capacity=512)

        def work(i):
            mine = keys[i * per * calls:(i + 1) * per * calls]
            for c in range(calls):
                k = torch.as_tensor(mine[c * per:(c + 1) * per], device=DEV)
                out = ev.sparse_read(k)
                assert out.shape == (per, D)

        _in_threads(work, THREADNUM)
        dr.status_check()
        assert ev.total_count().tolist() == [keys.size, D]
        k = ev.export()[0].cpu().numpy()
        np.testing.assert_array_equal(np.sort(k), np.sort(keys))
        got = ev.sparse_read(torch.as_tensor(keys, device=DEV)).cpu().numpy()
        assert bool((got == 0.25).all())
        dr.status_check()


@pytest.mark.parametrize("threads,reps", [(5, 1)])
def test_feature_filter_parallel(dr, threads, reps):
    """TestFeatureFilterParallel (:1012-1037): EmbeddingConfig(steps_to_live 5,
    filter_freq 7); 5 threads each LookupOrCreate key 20 once -> its
    frequency counts every one of them (5), and the key, still below the
    threshold, reads the default row.  (Past the threshold the reference
    stops counting -- CounterFilter::LookupOrCreate, embedding_filter.h:
    295-305 -- so more concurrent lookups than filter_freq leave a racy count
    there: not pinned.)"""
    ev = dr.EmbeddingVariable(
        "mtfilter_%d" % threads, 10, 10.0, steps_to_live=5,
        ev_option=dr.EmbeddingVariableOption(filter_option=dr.CounterFilter(7)))
    outs = [None] * threads

    def work(i):
        for _ in range(reps):
            outs[i] = ev.sparse_read(torch.tensor([20], dtype=torch.int64, device=DEV))

    _in_threads(work, threads)
    dr.status_check()
    fr, _, _ = ev.key_meta(np.array([20], np.int64))
    assert int(fr[0]) == threads * reps
    for o in outs:
        assert bool((o == 10.0).all())
