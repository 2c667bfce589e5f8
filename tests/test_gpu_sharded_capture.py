"""The host-read-free sharded engine kinds (dr_sharded_create_ex: XGMI peer
writes, fixed-capacity all-to-all) through the C ABI on an RCCL dr_comm at
world 1, captured into a hipGraph: the forward (with gradient) and the
backward of a step captured once, replayed on new ids copied into the
captured input, bit-equal to the same engine run eagerly, and the forward
bit-equal to the single-GPU lookup (embedding_lookup_sparse_multi).  The
variable-size RCCL kind reads its split sizes on the host and cannot be
captured; its N > 1 / callback paths are tests/test_gpu_sharded_c.py.
Reference: sparse_operation_kit/kit_cc_impl/embedding/dispatcher/
all2all_input_dispatcher.cu:241-286 (the host sync SOK pays, removed here)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

T, D, B, KEYS = 4, 32, 512, 6000


def _tables(dr, dev, tag):
    evs = []
    for t in range(T):
        ev = dr.EmbeddingVariable("cap_%s%d" % (tag, t), D, 0.25, capacity=KEYS + 8 * B,
                                  device=dev)
        k = np.arange(0, KEYS // 2, dtype=np.int64)
        v = np.cos(0.01 * k[:, None] + 0.3 * t + 0.07 * np.arange(D)[None, :]).astype(np.float32)
        ev.insert(torch.as_tensor(k, device=dev), torch.as_tensor(v, device=dev))
        evs.append(ev)
    return evs


@pytest.mark.parametrize("kind", ["xgmi", "fixed"])
def test_sharded_kind_captures_at_world_1(kind):
    import deeprec_amd as dr
    from deeprec_amd.embedding_ops import SparseTensor, embedding_lookup_sparse_multi
    from deeprec_amd.sharded import Comm, NativeShardedLookup
    dev = torch.device("cuda:0")
    dr.load()
    comm = Comm.rccl(0, 1)
    evs = _tables(dr, dev, kind)
    ref_evs = _tables(dr, dev, kind + "r")
    eng = NativeShardedLookup(comm, evs, dev, kind=kind, batch=B, max_ids=B)
    rng = np.random.default_rng(7)
    batches = [torch.as_tensor(rng.integers(0, KEYS, (T, B)), device=dev) for _ in range(3)]
    grads = [torch.as_tensor(rng.standard_normal((B, T * D)).astype(np.float32), device=dev)
             for _ in range(3)]
    ind = torch.stack([torch.arange(B, device=dev), torch.zeros(B, dtype=torch.int64,
                                                                device=dev)], 1)
    # every key of every batch exists before the capture (a captured resolve
    # must not grow a table); eager results of each batch
    eager = []
    for ids, g in zip(batches, grads):
        out = eng.forward(ids, need_grad=True).clone()
        sl = eng.backward(g)
        n = [int(x[2].item()) for x in sl]
        eager.append((out, [(x[0][:k].clone(), x[1][:k].clone()) for x, k in zip(sl, n)]))
        ref = embedding_lookup_sparse_multi(ref_evs, [SparseTensor(ind, ids[t], (B, 1))
                                                      for t in range(T)], combiner="sum")
        assert torch.equal(out, ref.detach()), "eager %s engine != single-GPU lookup" % kind
    for e in evs + ref_evs:
        e.pending_grads.clear()
    torch.cuda.synchronize()
    static_ids = batches[0].clone()
    static_g = grads[0].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm the engine's buffers on the capture's stream kind
        eng.forward(static_ids, need_grad=True)
        eng.backward(static_g)
    torch.cuda.current_stream().wait_stream(s)
    for e in evs:
        e.pending_grads.clear()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gout = eng.forward(static_ids, need_grad=True)
        gsl = eng.backward(static_g)
    for e in evs:
        e.pending_grads.clear()
    for r in (1, 2, 0, 1):
        static_ids.copy_(batches[r])
        static_g.copy_(grads[r])
        graph.replay()
        torch.cuda.synchronize()
        out, sl = eager[r]
        assert torch.equal(gout, out), "replay of batch %d: forward differs" % r
        for t in range(T):
            n = int(gsl[t][2].item())
            assert n == sl[t][0].numel(), (r, t)
            assert torch.equal(gsl[t][0][:n], sl[t][0]), (r, t)
            assert torch.equal(gsl[t][1][:n].view(torch.int32), sl[t][1].view(torch.int32)), (r, t)
    dr.status_check(dev)
    eng.close()
    comm.close()
