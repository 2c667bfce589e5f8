"""The torch.library registration of the op surface (torch.ops.deeprec.*):
every op is registered with the reference op's arguments, and its fake
(meta) implementation gives the output shapes, so graphs using the ops can
be traced without running them.  CPU only (meta tensors); the GPU tests
(test_gpu_torch_ops.py) run the ops."""
import pytest
import torch


@pytest.fixture(scope="module")
def tops():
    from deeprec_amd import torch_ops
    return torch_ops


def test_every_op_is_registered(tops):
    assert len(tops.OPS) >= 20
    for name in tops.OPS:
        sch = str(getattr(torch.ops.deeprec, name).default._schema)
        assert sch.startswith("deeprec::" + name + "(")


def test_reference_argument_names(tops):
    s = str(torch.ops.deeprec.kv_resource_sparse_apply_adam.default._schema)
    for a in ("beta1_power", "beta2_power", "lr", "beta1", "beta2", "epsilon", "grad", "indices"):
        assert a in s
    s = str(torch.ops.deeprec.fused_embedding_sparse_post_look_up.default._schema)
    for a in ("emb_shards", "partitioned_indices", "sp_dense_shape", "combiner", "max_norm"):
        assert a in s


def test_stateful_ops_declare_mutation(tops):
    """Ops that change an EV list its resource tensor as mutated (schema
    `Tensor(a!)`), so functionalization / torch.compile can neither drop nor
    reorder them; pure ops mutate nothing."""
    stateful = {"kv_resource_gather": ["resource"], "kv_resource_insert": ["resource"],
                "kv_embedding_lookup_sparse": ["resource"],
                "kv_resource_sparse_apply_gradient_descent": ["var"],
                "kv_resource_sparse_apply_adagrad": ["var", "accum"],
                "kv_resource_sparse_apply_adam": ["var", "m", "v"],
                "kv_resource_sparse_apply_ftrl": ["var", "accum", "linear"],
                "kv_resource_sparse_apply_adam_async": ["var", "m", "v", "beta_powers"],
                "kv_resource_sparse_apply_adagrad_decay": ["var", "accum", "accum_decay_power"]}
    for name in tops.OPS:
        sch = getattr(torch.ops.deeprec, name).default._schema
        mutated = [a.name for a in sch.arguments if a.alias_info is not None
                   and a.alias_info.is_write]
        assert mutated == stateful.get(name, []), (name, mutated)


def test_fake_shapes_on_meta(tops):
    m = dict(device="meta")
    x = torch.empty(10, dtype=torch.int64, **m)
    y, idx, cnt, u = torch.ops.deeprec.unique_with_counts(x)
    assert y.shape == (10,) and idx.dtype == torch.int32 and u.shape == (1,)
    data = torch.empty((7, 4), **m)
    out = torch.ops.deeprec.sparse_segment_reduce(data, torch.empty(5, dtype=torch.int32, **m),
                                                  torch.empty(5, dtype=torch.int32, **m), 3, "sum")
    assert out.shape == (3, 4)
    t = torch.empty((100, 8), **m)
    e = torch.ops.deeprec.embedding_lookup_sparse(t, torch.empty((20, 2), dtype=torch.int64, **m),
                                                  torch.empty(20, dtype=torch.int64, **m), 6)
    assert e.shape == (6, 8)
    res = torch.zeros(1, dtype=torch.int64)
    g = torch.ops.deeprec.kv_resource_gather(res, torch.empty((3, 5), dtype=torch.int64, **m), 16)
    assert g.shape == (3, 5, 16)
    e = torch.ops.deeprec.kv_embedding_lookup_sparse(
        res, torch.empty((20, 2), dtype=torch.int64, **m), torch.empty(20, dtype=torch.int64, **m),
        6, 32)
    assert e.shape == (6, 32)
    u, gr, nu = torch.ops.deeprec.kv_embedding_lookup_sparse_grad(
        torch.empty((20, 2), dtype=torch.int64, **m), torch.empty(20, dtype=torch.int64, **m), 6,
        torch.empty((6, 32), **m))
    assert u.shape == (20,) and gr.shape == (20, 32) and nu.shape == (1,)
    d = torch.ops.deeprec.dot_interaction(torch.empty((4, 27, 16), **m))
    assert d.shape == (4, 351)
