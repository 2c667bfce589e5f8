"""The engine's op surface registered as PyTorch custom operators
(torch.library), namespace `deeprec`: torch.ops.deeprec.<op>.

This is the realisable form of north_star's "host code registers custom ops"
(SURVEY.md section 8(b)): TensorFlow is not importable here, so the ops that
DeepRec registers with REGISTER_OP are registered with PyTorch's dispatcher
instead -- same names (snake_case), same argument meaning -- and each calls
the HIP engine through the C ABI (ops.py / include/deeprec_amd.h).  Every op
has a fake (meta) implementation so that graphs can be traced / exported
(torch.export, make_fx), and the differentiable ones carry their
reference gradients via torch.library.register_autograd.

EmbeddingVariables are resources in the reference (a `resource` handle
input); here they are passed as their resource tensor
(EmbeddingVariable.resource, a host int64[1] holding the library handle),
listed in mutates_args by every op that changes the EV.  Data-dependent output sizes (Unique,
PreLookUp) are returned at their static upper bound plus a device count, as
dr_unique does, so no op synchronises the host.

Reference op definitions: core/ops/kv_variable_ops.cc:222-492,
core/ops/training_ali_ops.cc:94-510, core/ops/fused_embedding_ops.cc:12-198,
core/ops/math_ops.cc (SparseSegment*), core/ops/array_ops.cc:1640,1669
(Unique[WithCounts]).
"""
from typing import List, Optional, Tuple

import ctypes as C

import torch
from torch import Tensor
from torch.library import custom_op

from . import _lib, ops
from ._lib import check, lib, ptr, stream_handle, workspace

_NS = "deeprec"
_COMB = ("sum", "mean", "sqrtn")


def _h(handle):
    return C.c_void_p(int(handle))


# ---------------------------------------------------------------------------
# Unique / UniqueWithCounts (core/ops/array_ops.cc:1640,1669)
# ---------------------------------------------------------------------------
@custom_op(_NS + "::unique_with_counts", mutates_args=(), device_types="cuda")
def unique_with_counts(x: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """(y [n], idx [n] int32, count [n] int32, num_unique [1] int64): y /
    count valid up to num_unique, first-occurrence order."""
    y, idx, cnt, u = ops.unique_device(x, with_counts=True)
    return y, idx, cnt, u


@unique_with_counts.register_fake
def _(x):
    n = x.numel()
    kt = torch.int32 if x.dtype == torch.int32 else torch.int64
    return (x.new_empty(n, dtype=kt), x.new_empty(n, dtype=torch.int32),
            x.new_empty(n, dtype=torch.int32), x.new_empty(1, dtype=torch.int64))


# ---------------------------------------------------------------------------
# Segment reductions (math_ops.cc SparseSegment{Sum,Mean,SqrtN}, grads
# math_grad.py:321-368) and UnsortedSegmentSum
# ---------------------------------------------------------------------------
@custom_op(_NS + "::sparse_segment_reduce", mutates_args=(), device_types="cuda")
def sparse_segment_reduce(data: Tensor, indices: Tensor, segment_ids: Tensor, num_segments: int,
                          combiner: str) -> Tensor:
    return ops._segment_reduce(data, indices, segment_ids, num_segments, combiner)


@sparse_segment_reduce.register_fake
def _(data, indices, segment_ids, num_segments, combiner):
    return data.new_empty((num_segments,) + tuple(data.shape[1:]), dtype=torch.float32)


@custom_op(_NS + "::sparse_segment_reduce_grad", mutates_args=(), device_types="cuda")
def sparse_segment_reduce_grad(grad: Tensor, indices: Tensor, segment_ids: Tensor,
                               output_dim0: int, combiner: str) -> Tensor:
    return ops._segment_grad(grad, indices, segment_ids, output_dim0, combiner)


@sparse_segment_reduce_grad.register_fake
def _(grad, indices, segment_ids, output_dim0, combiner):
    return grad.new_empty((output_dim0,) + tuple(grad.shape[1:]), dtype=torch.float32)


def _ssr_setup(ctx, inputs, output):
    data, indices, segment_ids, _, combiner = inputs
    ctx.save_for_backward(indices, segment_ids)
    ctx.combiner = combiner
    ctx.dim0 = data.shape[0]


def _ssr_backward(ctx, g):
    indices, segment_ids = ctx.saved_tensors
    gd = torch.ops.deeprec.sparse_segment_reduce_grad(g.contiguous(), indices, segment_ids,
                                                      ctx.dim0, ctx.combiner)
    return gd, None, None, None, None


sparse_segment_reduce.register_autograd(_ssr_backward, setup_context=_ssr_setup)


@custom_op(_NS + "::unsorted_segment_sum", mutates_args=(), device_types="cuda")
def unsorted_segment_sum(data: Tensor, segment_ids: Tensor, num_segments: int) -> Tensor:
    return ops.unsorted_segment_sum(data, segment_ids, num_segments)


@unsorted_segment_sum.register_fake
def _(data, segment_ids, num_segments):
    return data.new_empty((num_segments,) + tuple(data.shape[1:]), dtype=torch.float32)


def _uss_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[1])


def _uss_backward(ctx, g):
    (seg,) = ctx.saved_tensors
    # the grad of UnsortedSegmentSum is a gather of g by segment (0 for seg < 0)
    s = seg.to(torch.int64)
    valid = s >= 0
    rows = torch.ops.deeprec.resource_gather(g.contiguous(), torch.where(valid, s, 0))
    return rows * valid.reshape((-1,) + (1,) * (rows.dim() - 1)), None, None


unsorted_segment_sum.register_autograd(_uss_backward, setup_context=_uss_setup)


# ---------------------------------------------------------------------------
# Dense-table gather (ResourceGather / GatherV2)
# ---------------------------------------------------------------------------
@custom_op(_NS + "::resource_gather", mutates_args=(), device_types="cuda")
def resource_gather(params: Tensor, indices: Tensor) -> Tensor:
    return ops.gather(params, indices)


@resource_gather.register_fake
def _(params, indices):
    return params.new_empty(tuple(indices.shape) + (params.shape[1],), dtype=torch.float32)


def _rg_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[1])
    ctx.rows = inputs[0].shape[0]


def _rg_backward(ctx, g):
    (indices,) = ctx.saved_tensors
    D = g.shape[-1]
    dense = torch.ops.deeprec.unsorted_segment_sum(g.reshape(-1, D).contiguous(),
                                                   indices.reshape(-1).to(torch.int32), ctx.rows)
    return dense, None


resource_gather.register_autograd(_rg_backward, setup_context=_rg_setup)


# ---------------------------------------------------------------------------
# EmbeddingVariable ops (core/ops/kv_variable_ops.cc, training_ali_ops.cc).
#
# An EV enters an op as its RESOURCE tensor (EmbeddingVariable.resource: a
# host int64[1] holding the library handle -- TF's DT_RESOURCE scalar lives
# in host memory too).  Every op that changes the EV -- the insert-on-miss
# gather, insert, the sparse applies -- lists that tensor in mutates_args, so
# functionalization / torch.compile keep such ops, in program order, against
# every other op on the same EV (a None-returning op with no mutated input
# could be dead-code eliminated or reordered).  The tensor's value is never
# changed; it is the dependency token of the resource.
# ---------------------------------------------------------------------------
def _hr(resource):
    """c_void_p EV handle held by a resource tensor."""
    if resource.device.type != "cpu" or resource.dtype != torch.int64 or resource.numel() != 1:
        raise ValueError("an EV resource is a host int64[1] tensor (EmbeddingVariable.resource)")
    return C.c_void_p(int(resource.item()))


@custom_op(_NS + "::kv_resource_gather", mutates_args=("resource",), device_types="cuda")
def kv_resource_gather(resource: Tensor, indices: Tensor, dim: int,
                       default_value: Optional[Tensor] = None,
                       counts: Optional[Tensor] = None) -> Tensor:
    """KvResourceGather[V1] (kv_variable_ops.cc:314-449): rows of `indices`,
    insert-on-miss with default_value ([n, dim] or None = the EV default);
    counts (V1) feed the admission filter."""
    ids = indices.reshape(-1).to(torch.int64).contiguous()
    n = ids.numel()
    out = torch.empty((n, dim), dtype=torch.float32, device=ids.device)
    if n:
        dflt = None if default_value is None else default_value.to(torch.float32).contiguous()
        cnt = None if counts is None else counts.reshape(-1).to(torch.int32).contiguous()
        wsb = lib().dr_ev_gather_workspace_size(n)
        ws = workspace(wsb, ids.device)
        check(lib().dr_ev_gather(_hr(resource), ptr(ids), n, ptr(dflt), ptr(cnt), ptr(out),
                                 ptr(ws), wsb, stream_handle(ids.device)))
        ops._post(ids.device)
    return out.reshape(tuple(indices.shape) + (dim,))


@kv_resource_gather.register_fake
def _(resource, indices, dim, default_value=None, counts=None):
    return indices.new_empty(tuple(indices.shape) + (dim,), dtype=torch.float32)


@custom_op(_NS + "::kv_resource_insert", mutates_args=("resource",), device_types="cuda")
def kv_resource_insert(resource: Tensor, keys: Tensor, values: Tensor,
                       versions: Optional[Tensor] = None, freqs: Optional[Tensor] = None,
                       partition_id: int = 0, partition_num: int = 0) -> None:
    """KvResourceInsert / KvResourceImportV2 (Import semantics, optional
    key % 1000 % partition_num == partition_id filter)."""
    k = keys.reshape(-1).to(torch.int64).contiguous()
    v = values.to(torch.float32).contiguous()
    ver = None if versions is None else versions.to(torch.int64).contiguous()
    fr = None if freqs is None else freqs.to(torch.int64).contiguous()
    check(lib().dr_ev_insert(_hr(resource), ptr(k), k.numel(), ptr(v), ptr(ver), ptr(fr),
                             int(partition_id), int(partition_num), stream_handle(k.device)))
    ops._post(k.device)


def _apply_common(grad, indices):
    g = grad.to(torch.float32).contiguous()
    k = indices.reshape(-1).to(torch.int64).contiguous()
    return g, k, k.numel(), stream_handle(k.device)


def _one(x):
    return (C.c_void_p * 1)(x)


@custom_op(_NS + "::kv_resource_sparse_apply_gradient_descent", mutates_args=("var",),
           device_types="cuda")
def kv_resource_sparse_apply_gradient_descent(var: Tensor, alpha: float, grad: Tensor,
                                              indices: Tensor, global_step: int = -1,
                                              num_valid: Optional[Tensor] = None) -> None:
    """KvResourceSparseApplyGradientDescent (training_ali_ops.cc:1597-1678).
    num_valid: optional DEVICE int64[1] count of the valid leading rows (the
    IndexedSlices of a Unique with a data-dependent size)."""
    g, k, n, st = _apply_common(grad, indices)
    check(lib().dr_ev_apply_sgd(_hr(var), alpha, ptr(g), ptr(k), n, ptr(num_valid), global_step,
                                st))
    ops._post(k.device)


@custom_op(_NS + "::kv_resource_sparse_apply_adagrad", mutates_args=("var", "accum"),
           device_types="cuda")
def kv_resource_sparse_apply_adagrad(var: Tensor, accum: Tensor, lr: float, grad: Tensor,
                                     indices: Tensor, global_step: int = -1,
                                     num_valid: Optional[Tensor] = None) -> None:
    """KvResourceSparseApplyAdagrad (training_ali_ops.cc:61-145)."""
    g, k, n, st = _apply_common(grad, indices)
    check(lib().dr_ev_apply_adagrad(_hr(var), _hr(accum), lr, ptr(g), ptr(k), n, ptr(num_valid),
                                    global_step, st))
    ops._post(k.device)


@custom_op(_NS + "::kv_resource_sparse_apply_adam", mutates_args=("var", "m", "v"),
           device_types="cuda")
def kv_resource_sparse_apply_adam(var: Tensor, m: Tensor, v: Tensor, beta1_power: float,
                                  beta2_power: float, lr: float, beta1: float, beta2: float,
                                  epsilon: float, grad: Tensor, indices: Tensor,
                                  global_step: int = -1,
                                  num_valid: Optional[Tensor] = None) -> None:
    """KvResourceSparseApplyAdam (training_ali_ops.cc:848-975)."""
    g, k, n, st = _apply_common(grad, indices)
    check(lib().dr_ev_apply_adam(_hr(var), _hr(m), _hr(v), beta1_power, beta2_power, lr, beta1,
                                 beta2, epsilon, ptr(g), ptr(k), n, ptr(num_valid), global_step,
                                 st))
    ops._post(k.device)


@custom_op(_NS + "::kv_resource_sparse_apply_ftrl", mutates_args=("var", "accum", "linear"),
           device_types="cuda")
def kv_resource_sparse_apply_ftrl(var: Tensor, accum: Tensor, linear: Tensor, grad: Tensor,
                                  indices: Tensor, lr: float, l1: float, l2: float,
                                  lr_power: float, l2_shrinkage: float = 0.0,
                                  global_step: int = -1) -> None:
    """KvResourceSparseApplyFtrl[V2] (training_ali_ops.cc:167-331)."""
    g, k, n, st = _apply_common(grad, indices)
    check(lib().dr_ev_apply_ftrl(_hr(var), _hr(accum), _hr(linear), lr, l1, l2, lr_power,
                                 l2_shrinkage, ptr(g), ptr(k), n, None, global_step, st))
    ops._post(k.device)


@custom_op(_NS + "::kv_resource_sparse_apply_adam_async",
           mutates_args=("var", "m", "v", "beta_powers"), device_types="cuda")
def kv_resource_sparse_apply_adam_async(var: Tensor, m: Tensor, v: Tensor, beta_powers: Tensor,
                                        lr: float, beta1: float, beta2: float, epsilon: float,
                                        grad: Tensor, indices: Tensor, global_step: int = -1,
                                        apply_sparse_rmsprop: bool = False,
                                        num_valid: Optional[Tensor] = None) -> None:
    """KvResourceSparseApplyAdamAsync (training_ali_ops.cc:1404-1575).
    beta_powers: DEVICE float32[2] {beta1_power, beta2_power} -- the
    reference's beta power resources (:1523-1526) -- read for alpha and
    advanced by the op itself when N > 0 (:1482, :1558-1559)."""
    g, k, n, st = _apply_common(grad, indices)
    if not apply_sparse_rmsprop and (beta_powers.dtype != torch.float32
                                     or beta_powers.numel() != 2 or not beta_powers.is_cuda):
        raise ValueError("beta_powers must be a device float32[2]")
    check(lib().dr_ev_apply_adam_async_grouped(
        1 if apply_sparse_rmsprop else 0, 0, _one(_hr(var)), _one(_hr(m)), _one(_hr(v)), 1,
        _one(g.data_ptr()), _one(k.data_ptr()), (C.c_int64 * 1)(n), _one(ptr(num_valid)),
        _one(beta_powers.data_ptr()), lr, beta1, beta2, epsilon, global_step, st))
    ops._post(k.device)


@custom_op(_NS + "::kv_resource_sparse_apply_adagrad_decay",
           mutates_args=("var", "accum", "accum_decay_power"), device_types="cuda")
def kv_resource_sparse_apply_adagrad_decay(var: Tensor, accum: Tensor, accum_decay_power: Tensor,
                                           lr: float, decay_step: int, decay_rate: float,
                                           decay_baseline: float, global_step: int,
                                           grad: Tensor, indices: Tensor) -> None:
    """KvResourceSparseApplyAdagradDecay (training_ali_ops.cc:703-823)."""
    g, k, n, st = _apply_common(grad, indices)
    check(lib().dr_ev_apply_adagrad_decay_grouped(
        _one(_hr(var)), _one(_hr(accum)), _one(_hr(accum_decay_power)), 1, _one(g.data_ptr()), 0,
        _one(k.data_ptr()), (C.c_int64 * 1)(n), _one(None), lr, decay_step, decay_rate,
        decay_baseline, global_step, st))
    ops._post(k.device)


class _EvRef(object):
    """(handle, dim) view of a resource for ops.embedding_lookup_sparse_c."""

    def __init__(self, resource, dim):
        self.handle, self.dim = _hr(resource), dim


@custom_op(_NS + "::kv_embedding_lookup_sparse", mutates_args=("resource",),
           device_types="cuda")
def kv_embedding_lookup_sparse(resource: Tensor, sp_indices: Tensor, sp_values: Tensor,
                               batch: int, dim: int, sp_weights: Optional[Tensor] = None,
                               combiner: str = "mean", max_norm: float = -1.0,
                               safe: bool = False, default_id: int = -1,
                               prune: bool = True) -> Tensor:
    """embedding_lookup_sparse / safe_embedding_lookup_sparse on an EV
    (python/ops/embedding_ops.py:480-675, :1209-1344; the gather is
    EmbeddingVariable.sparse_read -> KvResourceGather, kv_variable_ops.py:
    644-664): the whole composition in ONE C call (dr_embedding_lookup_
    sparse), insert-on-miss on the EV.  The north_star hot path as one
    traceable op; its gradient is kv_embedding_lookup_sparse_grad."""
    if combiner not in _COMB:
        raise ValueError("combiner must be one of 'mean', 'sqrtn' or 'sum'")
    return ops.embedding_lookup_sparse_c(_EvRef(resource, dim), sp_indices, sp_values, batch,
                                         sp_weights, combiner,
                                         None if max_norm < 0 else max_norm, safe,
                                         None if default_id < 0 else default_id, prune)


@kv_embedding_lookup_sparse.register_fake
def _(resource, sp_indices, sp_values, batch, dim, sp_weights=None, combiner="mean",
      max_norm=-1.0, safe=False, default_id=-1, prune=True):
    return sp_values.new_empty((batch, dim), dtype=torch.float32)


@custom_op(_NS + "::kv_embedding_lookup_sparse_grad", mutates_args=(), device_types="cuda")
def kv_embedding_lookup_sparse_grad(sp_indices: Tensor, sp_values: Tensor, batch: int,
                                    top_grad: Tensor, sp_weights: Optional[Tensor] = None,
                                    combiner: str = "mean", resource: Optional[Tensor] = None,
                                    max_norm: float = -1.0, safe: bool = False,
                                    default_id: int = -1,
                                    prune: bool = True) -> Tuple[Tensor, Tensor, Tensor]:
    """The gradient of kv_embedding_lookup_sparse w.r.t. the EV as the
    reference's IndexedSlices (embedding_ops.py:592-675, math_grad.py:321-368):
    (unique ids in first-occurrence order, gradient rows, num_unique DEVICE
    int64[1]); the outputs hold nnz rows (nnz + batch when safe), rows past
    num_unique are unused.  Feed to a kv_resource_sparse_apply_* op with
    num_valid = num_unique.

    Takes the forward's safe / default_id / prune / max_norm:
      * safe: the same _prune_invalid_ids [/ _prune_invalid_weights] +
        sparse_fill_empty_rows (:1289-1310), so pruned ids get no gradient and
        the filled default_id (or 0) gets its rows' gradient; with default_id
        None (-1) the forward zeroes the empty rows (tf.where, :1330-1337), so
        their gradient is 0;
      * max_norm: the clip of the gathered unique rows
        (_embedding_lookup_and_transform -> _clip, :94-190) is differentiated
        (clip_by_norm's chain rule) at the EV's current rows -- `resource`
        is then required."""
    from .embedding_ops import (SparseTensor, _Feature, _grad_to_slices, _prune_and_fill)
    if combiner not in _COMB:
        raise ValueError("combiner must be one of 'mean', 'sqrtn' or 'sum'")
    if max_norm >= 0 and resource is None:
        raise ValueError("a max_norm gradient needs the EV resource (the clip's rows)")

    class _P(object):
        pass

    p = _P()
    p.dim = top_grad.shape[1]
    ind = sp_indices.to(torch.int64).contiguous()
    val = sp_values.to(torch.int64).contiguous()
    w = None if sp_weights is None else sp_weights.to(torch.float32).contiguous()
    g = top_grad.to(torch.float32).contiguous()
    n_out = val.numel() + (batch if safe else 0)
    if safe:
        sp, spw, empty = _prune_and_fill(
            SparseTensor(ind, val, (batch, 1)),
            None if w is None else SparseTensor(ind, w, (batch, 1)), combiner,
            None if default_id < 0 else default_id, prune)
        ind, val = sp.indices.contiguous(), sp.values.contiguous()
        w = None if spw is None else spw.values.contiguous()
        if default_id < 0:
            g = torch.where(empty[:, None], torch.zeros_like(g), g)
    f = _Feature(p, val, ind, batch, w, combiner, None)
    sl = _grad_to_slices(f, g, 0, g.shape[1])
    n = val.numel()
    idx = torch.zeros(n_out, dtype=torch.int64, device=g.device)
    vals = torch.zeros((n_out, g.shape[1]), dtype=torch.float32, device=g.device)
    idx[:n] = sl.indices[:n]
    vals[:n] = sl.values[:n]
    if max_norm >= 0 and n > 0:
        h = _hr(resource)
        rows = torch.empty(n, dtype=torch.int64, device=g.device)
        wsb = lib().dr_ev_resolve_workspace_size(n)
        ws = workspace(wsb, g.device)
        st = stream_handle(g.device)
        check(lib().dr_ev_resolve(h, ptr(idx), n, ptr(sl.num_valid), None, None, ptr(rows),
                                  ptr(ws), wsb, st))
        ops._post(g.device)
        sub = vals[:n]
        ops.clip_by_norm_grad(sub, int(lib().dr_ev_pool(h)), rows, max_norm,
                              default_rows=int(lib().dr_ev_default_row(h)), default_stride=0,
                              n_dev=sl.num_valid)
    return idx, vals, sl.num_valid.clone()


@kv_embedding_lookup_sparse_grad.register_fake
def _(sp_indices, sp_values, batch, top_grad, sp_weights=None, combiner="mean", resource=None,
      max_norm=-1.0, safe=False, default_id=-1, prune=True):
    n = sp_values.numel() + (batch if safe else 0)
    return (sp_values.new_empty(n, dtype=torch.int64),
            top_grad.new_empty((n, top_grad.shape[1]), dtype=torch.float32),
            sp_values.new_empty(1, dtype=torch.int64))


# ---------------------------------------------------------------------------
# Fused embedding ops (core/ops/fused_embedding_ops.cc)
# ---------------------------------------------------------------------------
@custom_op(_NS + "::fused_embedding_local_sparse_look_up", mutates_args=(), device_types="cuda")
def fused_embedding_local_sparse_look_up(sp_values: Tensor, sp_indices: Tensor,
                                         sp_dense_shape: List[int], emb_variable: Tensor,
                                         combiner: str, max_norm: float = -1.0
                                         ) -> Tuple[Tensor, Tensor]:
    return ops.fused_embedding_local_sparse_look_up(sp_values, sp_indices, sp_dense_shape,
                                                    emb_variable, combiner, max_norm)


@fused_embedding_local_sparse_look_up.register_fake
def _(sp_values, sp_indices, sp_dense_shape, emb_variable, combiner, max_norm=-1.0):
    B = sp_dense_shape[0]
    return (emb_variable.new_empty((B, emb_variable.shape[1]), dtype=torch.float32),
            emb_variable.new_empty((B,), dtype=torch.int32))


@custom_op(_NS + "::fused_embedding_local_sparse_look_up_grad", mutates_args=(),
           device_types="cuda")
def fused_embedding_local_sparse_look_up_grad(top_grad: Tensor, emb_variable: Tensor,
                                              sp_values: Tensor, sp_values_offset: Tensor,
                                              combiner: str, max_norm: float = -1.0) -> Tensor:
    return ops.fused_embedding_local_sparse_look_up_grad(top_grad, emb_variable, sp_values,
                                                         sp_values_offset, combiner, max_norm)


@fused_embedding_local_sparse_look_up_grad.register_fake
def _(top_grad, emb_variable, sp_values, sp_values_offset, combiner, max_norm=-1.0):
    return top_grad.new_empty((sp_values.numel(), top_grad.shape[1]), dtype=torch.float32)


def _fl_setup(ctx, inputs, output):
    sp_values, _, _, emb, combiner, max_norm = inputs
    ctx.save_for_backward(emb, sp_values, output[1])
    ctx.combiner, ctx.max_norm, ctx.rows = combiner, max_norm, emb.shape[0]


def _fl_backward(ctx, g, _g_off):
    emb, sp_values, vo = ctx.saved_tensors
    gv = torch.ops.deeprec.fused_embedding_local_sparse_look_up_grad(
        g.contiguous(), emb, sp_values, vo, ctx.combiner, ctx.max_norm)
    dense = torch.ops.deeprec.unsorted_segment_sum(gv, sp_values.to(torch.int32), ctx.rows)
    return None, None, None, dense, None, None


fused_embedding_local_sparse_look_up.register_autograd(_fl_backward, setup_context=_fl_setup)


@custom_op(_NS + "::fused_embedding_sparse_post_look_up", mutates_args=(), device_types="cuda")
def fused_embedding_sparse_post_look_up(emb_shards: List[Tensor], partitioned_indices: List[Tensor],
                                        sp_dense_shape: List[int], combiner: str,
                                        max_norm: float = -1.0) -> Tuple[Tensor, Tensor]:
    return ops.fused_embedding_sparse_post_look_up(emb_shards, partitioned_indices,
                                                   sp_dense_shape, None, combiner,
                                                   None if max_norm < 0 else max_norm)


@fused_embedding_sparse_post_look_up.register_fake
def _(emb_shards, partitioned_indices, sp_dense_shape, combiner, max_norm=-1.0):
    B = sp_dense_shape[0]
    e = emb_shards[0]
    return (e.new_empty((B, e.shape[1]), dtype=torch.float32),
            e.new_empty((B,), dtype=torch.int32))


@custom_op(_NS + "::fused_embedding_sparse_post_look_up_grad", mutates_args=(),
           device_types="cuda")
def fused_embedding_sparse_post_look_up_grad(top_grad: Tensor, emb_shards: List[Tensor],
                                             partitioned_indices: List[Tensor],
                                             feature_nums: Tensor, combiner: str,
                                             max_norm: float = -1.0) -> List[Tensor]:
    return ops.fused_embedding_sparse_post_look_up_grad(
        top_grad, emb_shards, partitioned_indices, feature_nums, combiner,
        None if max_norm < 0 else max_norm)


@fused_embedding_sparse_post_look_up_grad.register_fake
def _(top_grad, emb_shards, partitioned_indices, feature_nums, combiner, max_norm=-1.0):
    return [top_grad.new_empty((s.shape[0], top_grad.shape[1]), dtype=torch.float32)
            for s in emb_shards]


def _pl_setup(ctx, inputs, output):
    shards, inds, _, combiner, max_norm = inputs
    ctx.save_for_backward(output[1], *shards, *inds)
    ctx.P, ctx.combiner, ctx.max_norm = len(shards), combiner, max_norm


def _pl_backward(ctx, g, _g_fn):
    saved = ctx.saved_tensors
    fnum, shards, inds = saved[0], list(saved[1:1 + ctx.P]), list(saved[1 + ctx.P:])
    grads = torch.ops.deeprec.fused_embedding_sparse_post_look_up_grad(
        g.contiguous(), shards, inds, fnum, ctx.combiner, ctx.max_norm)
    return list(grads), None, None, None, None


fused_embedding_sparse_post_look_up.register_autograd(_pl_backward, setup_context=_pl_setup)


# ---------------------------------------------------------------------------
# Feature interactions (modelzoo DeepFM FM-2nd, DLRM dot)
# ---------------------------------------------------------------------------
@custom_op(_NS + "::fm_second_order", mutates_args=(), device_types="cuda")
def fm_second_order(emb: Tensor) -> Tensor:
    return ops.fm_second_order(emb)


@fm_second_order.register_fake
def _(emb):
    return emb.new_empty((emb.shape[0], emb.shape[2]), dtype=torch.float32)


@custom_op(_NS + "::fm_second_order_grad", mutates_args=(), device_types="cuda")
def fm_second_order_grad(emb: Tensor, top_grad: Tensor) -> Tensor:
    return ops.fm_second_order_grad(emb, top_grad)


@fm_second_order_grad.register_fake
def _(emb, top_grad):
    return torch.empty_like(emb, dtype=torch.float32)


def _save_first(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])


def _fm_backward(ctx, g):
    return (torch.ops.deeprec.fm_second_order_grad(ctx.saved_tensors[0], g.contiguous()),)


fm_second_order.register_autograd(_fm_backward, setup_context=_save_first)


@custom_op(_NS + "::dot_interaction", mutates_args=(), device_types="cuda")
def dot_interaction(x: Tensor) -> Tensor:
    return ops.dot_interaction(x)


@dot_interaction.register_fake
def _(x):
    F = x.shape[1]
    return x.new_empty((x.shape[0], F * (F - 1) // 2), dtype=torch.float32)


@custom_op(_NS + "::dot_interaction_grad", mutates_args=(), device_types="cuda")
def dot_interaction_grad(x: Tensor, top_grad: Tensor) -> Tensor:
    return ops.dot_interaction_grad(x, top_grad)


@dot_interaction_grad.register_fake
def _(x, top_grad):
    return torch.empty_like(x, dtype=torch.float32)


def _dot_backward(ctx, g):
    return (torch.ops.deeprec.dot_interaction_grad(ctx.saved_tensors[0], g.contiguous()),)


dot_interaction.register_autograd(_dot_backward, setup_context=_save_first)


OPS = ["unique_with_counts", "sparse_segment_reduce", "sparse_segment_reduce_grad",
       "unsorted_segment_sum", "resource_gather", "kv_resource_gather", "kv_resource_insert",
       "kv_resource_sparse_apply_gradient_descent", "kv_resource_sparse_apply_adagrad",
       "kv_resource_sparse_apply_adam", "kv_resource_sparse_apply_ftrl",
       "kv_resource_sparse_apply_adam_async", "kv_resource_sparse_apply_adagrad_decay",
       "fused_embedding_local_sparse_look_up", "fused_embedding_local_sparse_look_up_grad",
       "fused_embedding_sparse_post_look_up", "fused_embedding_sparse_post_look_up_grad",
       "fm_second_order", "fm_second_order_grad", "dot_interaction", "dot_interaction_grad",
       "kv_embedding_lookup_sparse", "kv_embedding_lookup_sparse_grad"]


# ---------------------------------------------------------------------------
# embedding_lookup_sparse over a dense table as one traceable op
# (python/ops/embedding_ops.py:480-675 composition, fused on the GPU:
# unique -> gather -> [clip] -> [* w] -> segment reduce; backward = the
# reference's chain (SparseSegment*Grad / weighted chain, clip_by_norm grad)
# scattered onto the table rows)
# ---------------------------------------------------------------------------
def _els_feature(params, sp_indices, sp_values, batch, sp_weights, combiner, max_norm):
    from .embedding_ops import _Feature
    v = sp_values.to(torch.int64).contiguous()
    w = None if sp_weights is None else sp_weights.to(torch.float32).contiguous()
    return _Feature(params, v, sp_indices.to(torch.int64).contiguous(), batch, w, combiner,
                    None if max_norm < 0 else max_norm)


@custom_op(_NS + "::embedding_lookup_sparse", mutates_args=(), device_types="cuda")
def embedding_lookup_sparse(params: Tensor, sp_indices: Tensor, sp_values: Tensor, batch: int,
                            sp_weights: Optional[Tensor] = None, combiner: str = "mean",
                            max_norm: float = -1.0) -> Tensor:
    from .embedding_ops import _pool_all
    if combiner not in _COMB:
        raise ValueError("combiner must be one of 'mean', 'sqrtn' or 'sum'")
    f = _els_feature(params, sp_indices, sp_values, batch, sp_weights, combiner, max_norm)
    return _pool_all([f], _lib.ORDER_ALI)


@embedding_lookup_sparse.register_fake
def _(params, sp_indices, sp_values, batch, sp_weights=None, combiner="mean", max_norm=-1.0):
    return params.new_empty((batch, params.shape[1]), dtype=torch.float32)


def _els_setup(ctx, inputs, output):
    params, sp_indices, sp_values, batch, sp_weights, combiner, max_norm = inputs
    ctx.save_for_backward(params, sp_indices, sp_values,
                          sp_weights if sp_weights is not None else sp_values.new_empty(0))
    ctx.batch, ctx.combiner, ctx.max_norm = batch, combiner, max_norm
    ctx.weighted = sp_weights is not None


def _els_backward(ctx, g):
    from .embedding_ops import _dense_grad, _grad_to_slices
    params, sp_indices, sp_values, w = ctx.saved_tensors
    f = _els_feature(params, sp_indices, sp_values, ctx.batch, w if ctx.weighted else None,
                     ctx.combiner, ctx.max_norm)
    g = g.contiguous()
    return (_dense_grad(params, _grad_to_slices(f, g, 0, g.shape[1])), None, None, None, None,
            None, None)


embedding_lookup_sparse.register_autograd(_els_backward, setup_context=_els_setup)
OPS.append("embedding_lookup_sparse")
