"""The RCCL transport of the sharded C entries (dr_comm_init with an
ncclUniqueId: sharded.Comm.rccl) executed at world 1 on one GPU --
ncclCommInitRank with one rank, the self block of every all-to-all copied
inside an ncclGroupStart / ncclGroupEnd pair -- driving NativeShardedLookup
(dr_sharded_forward / dr_sharded_backward; SOK's all2all_input_dispatcher.cu
/ all2all_output_dispatcher.cu protocol).  Forward bit-equal to
embedding_lookup_sparse_multi over a full copy of the tables; backward
IndexedSlices bit-equal to the oracle's Unique + SparseSegmentSumGrad."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

T, D, B, KEYSPACE = 3, 32, 4096, 20000


@pytest.fixture(scope="module")
def dr():
    import deeprec_amd
    deeprec_amd.load()
    deeprec_amd.set_validate(True)
    assert torch.cuda.is_available()
    return deeprec_amd


def _vals(t, keys):
    k = np.asarray(keys, np.float64)[:, None]
    return np.sin(0.011 * k + 0.5 * t + 0.03 * np.arange(D)[None, :]).astype(np.float32)


def test_rccl_comm_world1_forward_backward(dr, orc):
    from deeprec_amd.embedding_ops import SparseTensor, embedding_lookup_sparse_multi
    from deeprec_amd.sharded import Comm, NativeShardedLookup
    dev = torch.device("cuda", 0)
    half = np.arange(0, KEYSPACE // 2, dtype=np.int64)

    def evset(tag):
        evs = []
        for t in range(T):
            ev = dr.EmbeddingVariable("rccl_%s_%d" % (tag, t), D, 0.125, capacity=KEYSPACE)
            ev.insert(torch.as_tensor(half, device=dev), torch.as_tensor(_vals(t, half), device=dev))
            evs.append(ev)
        return evs

    shard, full = evset("sh"), evset("fu")
    comm = Comm.rccl(0, 1)
    eng = NativeShardedLookup(comm, shard, dev)
    rng = np.random.default_rng(7)
    ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64, device=dev)], 1)
    for step in range(3):
        ids = rng.integers(0, KEYSPACE, (T, B)).astype(np.int64)
        ids[:, :300] = 11 + step             # a run longer than one 256-position chunk
        it = torch.as_tensor(ids, device=dev)
        ref = embedding_lookup_sparse_multi(full, [SparseTensor(ind, it[t], (B, 1))
                                                   for t in range(T)], combiner="sum")
        out = eng.forward(it, combiner="sum", need_grad=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref.detach().cpu().numpy())
        g = rng.standard_normal((B, T * D)).astype(np.float32)
        slices = eng.backward(torch.as_tensor(g, device=dev))
        for t in range(T):
            k, v = slices[t]
            u, idx = orc.unique(ids[t])
            gu = orc.sparse_segment_reduce_grad(np.ascontiguousarray(g[:, t * D:(t + 1) * D]), idx,
                                                np.arange(B, dtype=np.int32), u.size, "sum")
            np.testing.assert_array_equal(k.cpu().numpy(), u)
            np.testing.assert_array_equal(v.cpu().numpy(), gu)
        for e in shard:
            e.pending_grads.clear()
        for e in full:
            e.pending_grads.clear()
    st = eng.stats()
    assert st["sent_keys"] > 0
    dr.status_check()
    eng.close()
    comm.close()
