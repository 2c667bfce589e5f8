"""Functional GPU ops with DeepRec/TF op names, on torch device tensors.

Each op calls the HIP C ABI (include/deeprec_amd.h) on torch's current stream.
Data-dependent errors (OP_REQUIRES in the reference) are latched on the
device; call `status_check()` or enable `set_validate(True)` to have every op
synchronise and raise, which is what the parity tests do.
"""
import ctypes as C
import os

import torch

from . import _lib
from ._lib import COMBINERS, ORDER_ALI, ORDER_SEQ, check, lib, ptr, stream_handle, workspace

_VALIDATE = os.environ.get("DEEPREC_AMD_VALIDATE", "0") == "1"


def set_validate(on):
    global _VALIDATE
    _VALIDATE = bool(on)


def _post(device):
    # (no validation sync while a hipGraph is being captured: the status word
    # is checked after the replay instead)
    if _VALIDATE and not torch.cuda.is_current_stream_capturing():
        _lib.status_check(device)


def status_check(device=None):
    _lib.status_check(device)


def _dev(t):
    if not t.is_cuda:
        raise _lib.DeepRecError(_lib.INVALID_ARGUMENT,
                                "deeprec_amd ops take device tensors (got %s)" % t.device)
    return t.device


def _c(t, dtype):
    return t.to(dtype).contiguous()


def _inner(t):
    """Elements per row of a [n, ...] tensor (also when n == 0)."""
    k = 1
    for x in t.shape[1:]:
        k *= int(x)
    return k


# ---------------------------------------------------------------------------
# Unique (UniqueAliOp, core/kernels/unique_ali_op.cc:46-180)
# ---------------------------------------------------------------------------
def unique_device(x, with_counts=False):
    """First-occurrence unique with NO host sync.

    Returns (y [n], idx [n] int32, counts [n] int32 or None, num_unique int64[1]);
    only y[:num_unique] / counts[:num_unique] are meaningful."""
    dev = _dev(x)
    i32 = x.dtype == torch.int32               # the int32 registration: y stays int32
    x = _c(x.reshape(-1), torch.int32 if i32 else torch.int64)
    n = x.numel()
    y = torch.empty(n, dtype=x.dtype, device=dev)
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev) if with_counts else None
    u = torch.empty(1, dtype=torch.int64, device=dev)
    if i32:
        wsb = lib().dr_unique_i32_workspace_size(n)
        ws = workspace(wsb, dev)
        check(lib().dr_unique_i32(ptr(x), n, ptr(y), ptr(idx), ptr(cnt), ptr(u), ptr(ws), wsb,
                                  stream_handle(dev)))
    else:
        wsb = lib().dr_unique_workspace_size(n)
        ws = workspace(wsb, dev)
        check(lib().dr_unique(ptr(x), n, ptr(y), ptr(idx), ptr(cnt), ptr(u), ptr(ws), wsb,
                              stream_handle(dev)))
    _post(dev)
    return y, idx, cnt, u


def _koff_array(koff):
    import ctypes as C
    return (C.c_int64 * len(koff))(*[int(k) for k in koff])


def unique_grouped(keys, koff, with_counts=False):
    """Grouped first-occurrence unique of T features in one pass.

    keys: concatenated [sum n_t] int64; koff: host offsets (T+1).  Returns
    (uniq, idx, counts or None, num_unique[T] int64 device); feature t's
    uniques are uniq[koff[t] : koff[t] + num_unique[t]], idx is feature-local."""
    dev = _dev(keys)
    k = _c(keys, torch.int64)
    n = k.numel()
    T = len(koff) - 1
    ka = _koff_array(koff)
    y = torch.empty(n, dtype=torch.int64, device=dev)
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev) if with_counts else None
    u = torch.empty(T, dtype=torch.int64, device=dev)
    wsb = lib().dr_unique_grouped_workspace_size(ka, T)
    ws = workspace(wsb, dev)
    check(lib().dr_unique_grouped(ptr(k), ka, T, ptr(y), ptr(idx), ptr(cnt), ptr(u), ptr(ws), wsb,
                                  stream_handle(dev)))
    _post(dev)
    return y, idx, cnt, u


def route_by_owner(uniq, koff, num_unique, world):
    """(owner, feature)-blocked send order of a grouped unique: returns
    (keys_send, tags_send, perm, counts[world, T]) with only the first
    counts.sum() entries meaningful."""
    dev = _dev(uniq)
    n = uniq.numel()
    T = len(koff) - 1
    ka = _koff_array(koff)
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    tags = torch.empty(n, dtype=torch.int32, device=dev)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty((world, T), dtype=torch.int64, device=dev)
    wsb = lib().dr_route_workspace_size(n, world, T)
    ws = workspace(wsb, dev)
    check(lib().dr_route_by_owner(ptr(uniq), ka, T, ptr(num_unique), world, ptr(keys), ptr(tags),
                                  ptr(perm), ptr(counts), ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return keys, tags, perm, counts


def unique(x, out_idx=torch.int32):
    """tf.unique: (y, idx), y in first-occurrence order (syncs for |y|)."""
    y, idx, _, u = unique_device(x)
    k = int(u.item())
    return y[:k], idx.to(out_idx)


def unique_with_counts(x, out_idx=torch.int32):
    y, idx, cnt, u = unique_device(x, with_counts=True)
    k = int(u.item())
    return y[:k], idx.to(out_idx), cnt[:k]


# ---------------------------------------------------------------------------
# Gather / segment reductions
# ---------------------------------------------------------------------------
def gather(params, indices):
    """ResourceGather on a dense [R, D] table (gather_functor.h:36-115)."""
    dev = _dev(params)
    params = _c(params, torch.float32)
    idx = _c(indices.reshape(-1), torch.int64)
    D = params.shape[1]
    out = torch.empty((idx.numel(), D), dtype=torch.float32, device=dev)
    check(lib().dr_gather(ptr(params), params.shape[0], D, ptr(idx), idx.numel(), ptr(out),
                          stream_handle(dev)))
    _post(dev)
    return out.reshape(tuple(indices.shape) + (D,))


def _segment_reduce(data, indices, segment_ids, num_segments, combiner):
    dev = _dev(data)
    data = _c(data, torch.float32)
    data2 = data.reshape(data.shape[0], _inner(data))
    idx = _c(indices, torch.int32)
    seg = _c(segment_ids, torch.int32)
    if num_segments is None:  # output rows = last segment id + 1 (reference CPU)
        num_segments = int(seg[-1].item()) + 1 if seg.numel() else 0
    D = data2.shape[1]
    out = torch.empty((num_segments, D), dtype=torch.float32, device=dev)
    wsb = lib().dr_segment_workspace_size(num_segments)
    ws = workspace(wsb, dev)
    check(lib().dr_sparse_segment_reduce(ptr(data2), data2.shape[0], D, ptr(idx), ptr(seg),
                                         idx.numel(), num_segments, COMBINERS[combiner], ptr(out),
                                         ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return out.reshape((num_segments,) + tuple(data.shape[1:]))


def sparse_segment_sum(data, indices, segment_ids, num_segments=None):
    return _segment_reduce(data, indices, segment_ids, num_segments, "sum")


def sparse_segment_mean(data, indices, segment_ids, num_segments=None):
    return _segment_reduce(data, indices, segment_ids, num_segments, "mean")


def sparse_segment_sqrt_n(data, indices, segment_ids, num_segments=None):
    return _segment_reduce(data, indices, segment_ids, num_segments, "sqrtn")


def _segment_grad(grad, indices, segment_ids, output_dim0, combiner):
    dev = _dev(grad)
    grad = _c(grad, torch.float32)
    g2 = grad.reshape(grad.shape[0], _inner(grad))
    idx = _c(indices, torch.int32)
    seg = _c(segment_ids, torch.int32)
    D = g2.shape[1]
    out = torch.empty((output_dim0, D), dtype=torch.float32, device=dev)
    wsb = lib().dr_segment_grad_workspace_size(idx.numel(), g2.shape[0], output_dim0)
    ws = workspace(wsb, dev)
    check(lib().dr_sparse_segment_reduce_grad(ptr(g2), g2.shape[0], D, ptr(idx), ptr(seg),
                                              idx.numel(), output_dim0, COMBINERS[combiner],
                                              ptr(out), ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return out.reshape((output_dim0,) + tuple(grad.shape[1:]))


def sparse_segment_sum_grad(grad, indices, segment_ids, output_dim0):
    """Grad of SparseSegmentSum = unsorted_segment_sum(gather(grad, seg), idx, dim0)
    (math_grad.py:321-327), deterministic CPU order."""
    return _segment_grad(grad, indices, segment_ids, output_dim0, "sum")


def sparse_segment_mean_grad(grad, indices, segment_ids, output_dim0):
    return _segment_grad(grad, indices, segment_ids, output_dim0, "mean")


def sparse_segment_sqrt_n_grad(grad, indices, segment_ids, output_dim0):
    return _segment_grad(grad, indices, segment_ids, output_dim0, "sqrtn")


def unsorted_segment_sum(data, segment_ids, num_segments):
    """UnsortedSegmentSum (segment_reduction_ops.cc:377-405): serial order, seg<0 skipped."""
    dev = _dev(data)
    data = _c(data, torch.float32)
    d2 = data.reshape(data.shape[0], _inner(data))
    seg = _c(segment_ids, torch.int32)
    D = d2.shape[1]
    out = torch.empty((num_segments, D), dtype=torch.float32, device=dev)
    wsb = lib().dr_unsorted_segment_sum_workspace_size(seg.numel(), num_segments)
    ws = workspace(wsb, dev)
    check(lib().dr_unsorted_segment_sum(ptr(d2), d2.shape[0], D, ptr(seg), num_segments, ptr(out),
                                        ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return out.reshape((num_segments,) + tuple(data.shape[1:]))


def bag_offsets(segment_ids, batch):
    """CSR offsets [batch+1] of sorted segment ids (int32 or int64)."""
    dev = _dev(segment_ids)
    off = torch.empty(batch + 1, dtype=torch.int32, device=dev)
    if segment_ids.dtype == torch.int32:
        s = segment_ids.contiguous()
        check(lib().dr_bag_offsets_i32(ptr(s), s.numel(), batch, ptr(off), stream_handle(dev)))
    else:
        s = _c(segment_ids, torch.int64)
        check(lib().dr_bag_offsets(ptr(s), s.numel(), batch, ptr(off), stream_handle(dev)))
    _post(dev)
    return off


def pool_grouped(descs, batch, dim, order=ORDER_ALI, device=None, onehot=False, bf16=False,
                 out_bf16=False):
    """Launch dr_pool_grouped_ex on a list of _lib.DrPoolDesc (<= 32 tables).
    onehot: every bag b holds exactly nnz b (bag_off not read).  bf16: the
    tables hold bf16 values (DR_POOL_BF16), pooled into fp32 -- or into bf16
    with out_bf16 (DR_POOL_OUT_BF16); strides in elements of their type."""
    arr = (_lib.DrPoolDesc * len(descs))(*descs)
    flags = ((_lib.POOL_ONEHOT if onehot else 0) | (_lib.POOL_BF16 if bf16 else 0)
             | (_lib.POOL_OUT_BF16 if out_bf16 else 0))
    check(lib().dr_pool_grouped_ex(arr, len(descs), batch, dim, order, flags,
                                   stream_handle(device)))
    _post(device)


def sort_pairs(keys, vals, bit_hi, bit_lo=0):
    """Stable LSD radix sort of (uint64 key, int32 value) pairs."""
    dev = _dev(keys)
    k = _c(keys, torch.int64)
    v = _c(vals, torch.int32)
    ko = torch.empty_like(k)
    vo = torch.empty_like(v)
    wsb = lib().dr_sort_pairs_workspace_size(k.numel())
    ws = workspace(wsb, dev)
    check(lib().dr_sort_pairs(ptr(k), ptr(v), ptr(ko), ptr(vo), k.numel(), bit_lo, bit_hi, ptr(ws),
                              wsb, stream_handle(dev)))
    _post(dev)
    return ko, vo


# ---------------------------------------------------------------------------
# embedding_lookup_sparse / safe_embedding_lookup_sparse through the single
# C entry dr_embedding_lookup_sparse (embedding_ops.py:480-675, :1209-1344):
# what a TF custom-op kernel binds.  Forward only.
# ---------------------------------------------------------------------------
def embedding_lookup_sparse_c(params, sp_indices, sp_values, batch, sp_weights=None,
                              combiner="mean", max_norm=None, safe=False, default_id=None,
                              prune=True):
    """params: an EmbeddingVariable (handle / dim attributes) or a dense fp32
    [rows, dim] tensor.  sp_indices [nnz, 2] int64 rows-sorted, sp_values
    [nnz] int64, sp_weights [nnz] fp32 or None.  Returns [batch, dim]."""
    ind = sp_indices.to(torch.int64).contiguous()
    val = sp_values.to(torch.int64).contiguous()
    w = None if sp_weights is None else sp_weights.to(torch.float32).contiguous()
    nnz = val.numel()
    dev = val.device
    if torch.is_tensor(params):
        ev, table = None, params.contiguous()
        rows, dim = table.shape
    else:
        ev, table, rows, dim = params.handle, None, 0, params.dim
    out = torch.empty((batch, dim), dtype=torch.float32, device=dev)
    wsb = lib().dr_embedding_lookup_sparse_workspace_size(nnz, batch)
    ws = workspace(wsb, dev)
    check(lib().dr_embedding_lookup_sparse(
        ev, ptr(table), rows, dim, ptr(ind), ptr(val), ptr(w), nnz, batch, COMBINERS[combiner],
        -1.0 if max_norm is None else float(max_norm), 1 if safe else 0,
        -1 if default_id is None else int(default_id), 1 if prune else 0, ptr(out), dim,
        ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return out


# ---------------------------------------------------------------------------
# Fused embedding ops (core/ops/fused_embedding_ops.cc:12-58)
# ---------------------------------------------------------------------------
def fused_embedding_local_sparse_look_up(sp_values, sp_indices, sp_dense_shape, emb_variable,
                                         combiner="mean", max_norm=-1.0):
    dev = _dev(emb_variable)
    table = _c(emb_variable, torch.float32)
    vals = _c(sp_values, torch.int64)
    ind = _c(sp_indices, torch.int64)
    B = int(sp_dense_shape[0])
    D = table.shape[1]
    out = torch.empty((B, D), dtype=torch.float32, device=dev)
    vo = torch.empty(B, dtype=torch.int32, device=dev)
    wsb = lib().dr_fused_local_workspace_size(B)
    ws = workspace(wsb, dev)
    check(lib().dr_fused_local_lookup(ptr(table), table.shape[0], D, ptr(vals), ptr(ind),
                                      vals.numel(), B, COMBINERS[combiner], float(max_norm),
                                      ptr(out), ptr(vo), ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return out, vo


def fused_embedding_local_sparse_look_up_grad(top_grad, emb_variable, sp_values,
                                              sp_values_offset, combiner="mean", max_norm=-1.0):
    dev = _dev(top_grad)
    tg = _c(top_grad, torch.float32)
    table = _c(emb_variable, torch.float32)
    vals = _c(sp_values, torch.int64)
    vo = _c(sp_values_offset, torch.int32)
    D = tg.shape[1]
    out = torch.empty((vals.numel(), D), dtype=torch.float32, device=dev)
    check(lib().dr_fused_local_lookup_grad(ptr(tg), ptr(table), table.shape[0], D, ptr(vals),
                                           ptr(vo), vals.numel(), tg.shape[0],
                                           COMBINERS[combiner], float(max_norm), ptr(out),
                                           stream_handle(dev)))
    _post(dev)
    return out


def _combiner(combiner):
    if combiner not in COMBINERS:
        raise ValueError("combiner must be one of 'mean', 'sqrtn' or 'sum'")
    return COMBINERS[combiner]


def _max_norm(max_norm):
    return -1.0 if max_norm is None else float(max_norm)


def fused_embedding_sparse_pre_look_up(partition_shapes, sp_values, sp_indices):
    """FusedEmbeddingSparsePreLookUp (core/ops/fused_embedding_ops.cc:60-107,
    fused_embedding_ops_gpus.cu.cc:150-283): ids stably sorted and split by
    the "div" boundaries of partition_shapes[i][0], rebased per partition.
    Returns (partitioned_values, partitioned_indices) lists.  Like the
    reference kernel (:228-238) it reads the partition sizes back to the host
    once to shape its outputs."""
    dev = _dev(sp_values)
    rows = [int(s[0]) for s in partition_shapes]
    P = len(rows)
    if P < 1 or P > _lib.MAX_PARTITIONS:
        raise ValueError("num_partitions must be in [1, %d]" % _lib.MAX_PARTITIONS)
    vals = _c(sp_values.reshape(-1), torch.int64)
    ind = _c(sp_indices, torch.int64)
    n = vals.numel()
    if ind.shape != (n, 2):
        raise _lib.InvalidArgumentError(_lib.INVALID_ARGUMENT, "sp_indices must be [nnz, 2]")
    import ctypes as C
    vout = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    iout = torch.empty((max(n, 1), 2), dtype=torch.int64, device=dev)
    off = torch.empty(P + 1, dtype=torch.int64, device=dev)
    wsb = lib().dr_fused_pre_lookup_workspace_size(n)
    ws = workspace(wsb, dev)
    check(lib().dr_fused_pre_lookup(ptr(vals), ptr(ind), n, (C.c_int64 * P)(*rows), P, ptr(vout),
                                    ptr(iout), ptr(off), ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    o = off.cpu().tolist()
    return ([vout[o[p]:o[p + 1]] for p in range(P)], [iout[o[p]:o[p + 1]] for p in range(P)])


def _shard_arrays(emb_shards, partitioned_indices):
    import ctypes as C
    P = len(emb_shards)
    if P < 1 or P > _lib.MAX_PARTITIONS or len(partitioned_indices) != P:
        raise ValueError("need 1..%d emb_shards with one partitioned_indices each"
                         % _lib.MAX_PARTITIONS)
    shards = [_c(s, torch.float32) for s in emb_shards]
    inds = [_c(i, torch.int64) for i in partitioned_indices]
    for s, i in zip(shards, inds):
        if s.shape[0] != i.shape[0]:
            raise _lib.InvalidArgumentError(
                _lib.INVALID_ARGUMENT, "emb_shard and partitioned_indice dosn't have the same length")
    A = C.c_void_p * P
    sp = A(*[s.data_ptr() if s.numel() else None for s in shards])
    ip = A(*[i.data_ptr() if i.numel() else None for i in inds])
    rows = (C.c_int64 * P)(*[s.shape[0] for s in shards])
    return shards, inds, sp, ip, rows


def fused_embedding_sparse_post_look_up(emb_shards, partitioned_indices, sp_dense_shape,
                                        partitioned_values=None, combiner="mean", max_norm=None):
    """FusedEmbeddingSparsePostLookUp (core/ops/fused_embedding_ops.cc:109-155,
    fused_embedding_ops_gpus.cu.cc:285-384) -> (emb_vectors [B, D],
    feature_nums [B] int32).  Bags are summed in (row, col) order, so the
    result equals the local fused lookup of the same ids bit for bit."""
    dev = _dev(emb_shards[0])
    shards, inds, sp, ip, rows = _shard_arrays(emb_shards, partitioned_indices)
    P = len(shards)
    D = shards[0].shape[1]
    B, cols = int(sp_dense_shape[0]), int(sp_dense_shape[1])
    out = torch.empty((B, D), dtype=torch.float32, device=dev)
    fnum = torch.empty(B, dtype=torch.int32, device=dev)
    N = sum(s.shape[0] for s in shards)
    wsb = lib().dr_fused_post_lookup_workspace_size(N, B)
    ws = workspace(wsb, dev)
    check(lib().dr_fused_post_lookup(sp, ip, rows, P, B, max(cols, 1), D, _combiner(combiner),
                                     _max_norm(max_norm), ptr(out), ptr(fnum), ptr(ws), wsb,
                                     stream_handle(dev)))
    _post(dev)
    return out, fnum


def fused_embedding_sparse_post_look_up_grad(top_grad, emb_shards, partitioned_indices,
                                             feature_nums, combiner="mean", max_norm=None):
    """FusedEmbeddingSparsePostLookUpGrad (core/ops/fused_embedding_ops.cc:157-196,
    fused_embedding_ops_gpus.cu.cc:386-514) -> grad_shards list."""
    import ctypes as C
    dev = _dev(top_grad)
    tg = _c(top_grad, torch.float32)
    shards, inds, sp, ip, rows = _shard_arrays(emb_shards, partitioned_indices)
    P = len(shards)
    D = tg.shape[1]
    outs = [torch.empty((s.shape[0], D), dtype=torch.float32, device=dev) for s in shards]
    fn = _c(feature_nums, torch.int32)
    check(lib().dr_fused_post_lookup_grad(
        ptr(tg), sp, ip, rows, P, tg.shape[0], D, ptr(fn), _combiner(combiner),
        _max_norm(max_norm), (C.c_void_p * P)(*[o.data_ptr() if o.numel() else None
                                               for o in outs]), stream_handle(dev)))
    _post(dev)
    return outs


def bag_weight_scale(weights, bag_off, combiner):
    """Per-bag divisor of a weighted lookup: sum(w) (mean) / sqrt(sum(w^2))."""
    dev = _dev(weights)
    B = bag_off.numel() - 1
    q = torch.empty(max(B, 1), dtype=torch.float32, device=dev)
    check(lib().dr_bag_weight_scale(ptr(weights), ptr(bag_off), B, _combiner(combiner), ptr(q),
                                    stream_handle(dev)))
    _post(dev)
    return q


def clip_by_norm_grad(grad, pool, rows, max_norm, pool_rows=None, default_rows=None,
                      default_stride=0, n_dev=None):
    """In place: grad [n, D] of clip_by_norm(pool[rows], max_norm) -> grad of
    the unclipped rows (clip_ops.py:164-184 chain rule)."""
    dev = _dev(grad)
    n, D = grad.shape
    pr = (1 << 62) if pool_rows is None else int(pool_rows)
    dr_ = default_rows if isinstance(default_rows, int) else ptr(default_rows)
    check(lib().dr_clip_by_norm_grad(pool if isinstance(pool, int) else ptr(pool), pr, ptr(rows),
                                     dr_, int(default_stride), ptr(n_dev), n, D,
                                     float(max_norm), ptr(grad), stream_handle(dev)))
    _post(dev)
    return grad


# ---------------------------------------------------------------------------
# Interactions
# ---------------------------------------------------------------------------
def fm_second_order(emb):
    """0.5 * ((sum_f e)^2 - sum_f e^2) over [B, F, D] (DeepFM train.py:205-209)."""
    dev = _dev(emb)
    e = _c(emb, torch.float32)
    B, F, D = e.shape
    out = torch.empty((B, D), dtype=torch.float32, device=dev)
    check(lib().dr_fm2(ptr(e), B, F, D, ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def fm_second_order_grad(emb, top_grad):
    dev = _dev(emb)
    e = _c(emb, torch.float32)
    g = _c(top_grad, torch.float32)
    B, F, D = e.shape
    out = torch.empty_like(e)
    check(lib().dr_fm2_grad(ptr(e), ptr(g), B, F, D, ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def fm_second_order_bf16_copy(emb):
    """dr_fm2_bf16_copy: (fm [B, D] fp32, bf16 copy of emb as [B, F*D])."""
    dev = _dev(emb)
    emb = _c(emb, torch.float32)
    B, F, D = emb.shape
    out = torch.empty((B, D), dtype=torch.float32, device=dev)
    cp = torch.empty((B, F * D), dtype=torch.bfloat16, device=dev)
    check(lib().dr_fm2_bf16_copy(ptr(emb), B, F, D, ptr(out), ptr(cp), stream_handle(dev)))
    _post(dev)
    return out, cp


def fm_second_order_grad_add_bf16(emb, top_grad, add):
    """dr_fm2_grad_add_bf16: FM gradient + float(add) (add bf16 [B, F*D])."""
    dev = _dev(emb)
    emb = _c(emb, torch.float32)
    g = _c(top_grad, torch.float32)
    B, F, D = emb.shape
    if add.dtype != torch.bfloat16 or add.stride(1) != 1:
        raise ValueError("add must be bf16 with unit column stride")
    out = torch.empty_like(emb)
    check(lib().dr_fm2_grad_add_bf16(ptr(emb), ptr(g), ptr(add), add.stride(0), B, F, D, ptr(out),
                                     stream_handle(dev)))
    _post(dev)
    return out


def dot_interaction(x):
    """DLRM dot_op (DLRM train.py:150-163): strictly-lower triangle of X X^T."""
    dev = _dev(x)
    x = _c(x, torch.float32)
    B, F, D = x.shape
    out = torch.empty((B, F * (F - 1) // 2), dtype=torch.float32, device=dev)
    check(lib().dr_dot_interaction(ptr(x), B, F, D, ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def dot_interaction_grad(x, top_grad):
    """Backward of dot_interaction: [B, F, D] grad of X."""
    dev = _dev(x)
    x = _c(x, torch.float32)
    g = _c(top_grad, torch.float32)
    B, F, D = x.shape
    out = torch.empty_like(x)
    check(lib().dr_dot_interaction_grad(ptr(x), ptr(g), B, F, D, ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def dot_interaction_concat_bf16(x, out_cols):
    """DLRM dot layer + concat + --bf16 cast (modelzoo/DLRM/train.py:211-226):
    x [B, F, D] fp32 with x[:, 0] = dense_inputs -> bf16 [B, out_cols] =
    x[:, 0] | dot_interaction(x) | zero padding (dr_dot_interaction_concat_bf16)."""
    dev = _dev(x)
    x = _c(x, torch.float32)
    B, F, D = x.shape
    out = torch.empty((B, out_cols), dtype=torch.bfloat16, device=dev)
    check(lib().dr_dot_interaction_concat_bf16(ptr(x), B, F, D, ptr(out), out_cols,
                                               stream_handle(dev)))
    _post(dev)
    return out


def dot_interaction_concat_grad_bf16(x, grad):
    """Backward of dot_interaction_concat_bf16 from the bf16 [B, cols] gradient."""
    dev = _dev(x)
    x = _c(x, torch.float32)
    if grad.dtype != torch.bfloat16 or grad.stride(1) != 1:
        raise ValueError("grad must be bf16 with unit column stride")
    B, F, D = x.shape
    out = torch.empty_like(x)
    check(lib().dr_dot_interaction_concat_grad_bf16(ptr(x), ptr(grad), grad.stride(0), B, F, D,
                                                    ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def relu_grad_bf16(g, y):
    """dr_relu_grad_bf16: bf16(g) masked by y > 0 (y the bf16 ReLU output);
    g fp32 [R, C] with unit column stride (any row stride)."""
    dev = _dev(g)
    R, C = y.shape
    if g.dtype != torch.float32 or g.stride(1) != 1 or y.dtype != torch.bfloat16 \
            or y.stride(1) != 1 or tuple(g.shape) != (R, C):
        raise ValueError("relu_grad_bf16 needs fp32 g and bf16 y of one shape, unit column stride")
    out = torch.empty((R, C), dtype=torch.bfloat16, device=dev)
    check(lib().dr_relu_grad_bf16(ptr(g), g.stride(0), ptr(y), y.stride(0), R, C, ptr(out), C,
                                  stream_handle(dev)))
    _post(dev)
    return out


def mlp_head_forward(h, w, bias=None):
    """dr_mlp_head_forward_bf16: the N = 1 output layer on the bf16 tower
    output h [B, K] -> z [B] fp32.  w bf16: the bf16 layer (a bf16-rounded
    logit); w fp32: the fp32 layer on the widened h.  bias a 1-element fp32
    device tensor or None."""
    dev = _dev(h)
    B, K = h.shape
    if h.dtype != torch.bfloat16 or h.stride(1) != 1 or \
            w.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("mlp_head_forward needs bf16 h (unit column stride), bf16 / fp32 w")
    z = torch.empty(B, dtype=torch.float32, device=dev)
    bb = None if bias is None else _c(bias.reshape(1), torch.float32)
    check(lib().dr_mlp_head_forward_bf16(ptr(h), h.stride(0), B, K, ptr(w.contiguous()),
                                         1 if w.dtype == torch.float32 else 0, ptr(bb), ptr(z),
                                         stream_handle(dev)))
    _post(dev)
    return z


def mlp_head_backward(h, w, gz):
    """dr_mlp_head_backward_bf16 -> (grad_h bf16 [B, K] with h's ReLU mask
    applied, dw fp32 [K], db fp32 scalar tensor); w as in mlp_head_forward."""
    dev = _dev(h)
    B, K = h.shape
    gz = _c(gz.reshape(B), torch.float32)
    P = lib().dr_mlp_head_grad_partials(B)
    gh = torch.empty((B, K), dtype=torch.bfloat16, device=dev)
    dwp = torch.empty((max(P, 1), K), dtype=torch.float32, device=dev)
    dbp = torch.empty(max(P, 1), dtype=torch.float32, device=dev)
    check(lib().dr_mlp_head_backward_bf16(ptr(h), h.stride(0), B, K, ptr(w.contiguous()),
                                          1 if w.dtype == torch.float32 else 0, ptr(gz), ptr(gh),
                                          K, ptr(dwp), ptr(dbp), stream_handle(dev)))
    _post(dev)
    return gh, dwp[:P].sum(0), dbp[:P].sum()


def crossnet_layer(x0, xl, weight, bias=None):
    """DCN-v2 cross layer x0 * (xl W^T + b) + xl, bf16 MFMA, fp32 accumulate.

    Feature dims that are not a multiple of 64 are zero-padded (exact); a
    caller that keeps its features padded (modelzoo.DCNv2) pays no copy."""
    dev = _dev(x0)
    B, d = x0.shape
    dp = (d + 63) // 64 * 64

    def pad2(t, rows, cols):
        t = t.to(torch.bfloat16)
        if t.shape[1] == cols and t.shape[0] == rows:
            return t.contiguous()
        o = torch.zeros((rows, cols), dtype=torch.bfloat16, device=dev)
        o[:t.shape[0], :t.shape[1]] = t
        return o

    a0 = pad2(x0, B, dp)
    al = pad2(xl, B, dp)
    w = pad2(weight, dp, dp)
    b = None
    if bias is not None:
        b = torch.zeros(dp, dtype=torch.float32, device=dev)
        b[:d] = bias.float()
    out, _ = crossnet_forward(a0, al, w, b, with_lin=False)
    return out[:, :d]


def crossnet_forward(x0, xl, weight, bias, with_lin=True):
    """dr_crossnet_forward_bf16 on padded operands: x0 / xl [B, d] bf16,
    weight [d, d] bf16 (out, in), bias [d] fp32 or None, d % 64 == 0.
    Returns (out [B, d] bf16, lin = xl W^T + b [B, d] bf16 or None)."""
    dev = _dev(x0)
    B, d = x0.shape
    if d % 64 or x0.dtype != torch.bfloat16 or xl.dtype != torch.bfloat16 \
            or weight.dtype != torch.bfloat16 or tuple(weight.shape) != (d, d):
        raise ValueError("crossnet_forward needs bf16 operands with d % 64 == 0")
    x0, xl, weight = x0.contiguous(), xl.contiguous(), weight.contiguous()
    b = None if bias is None else bias.to(torch.float32).contiguous()
    out = torch.empty((B, d), dtype=torch.bfloat16, device=dev)
    lin = torch.empty((B, d), dtype=torch.bfloat16, device=dev) if with_lin else None
    check(lib().dr_crossnet_forward_bf16(ptr(x0), ptr(xl), ptr(weight), ptr(b), B, d, ptr(out),
                                         ptr(lin), stream_handle(dev)))
    _post(dev)
    return out, lin


ACT_NONE, ACT_RELU, ACT_MASK = 0, 1, 2


def gemm_nt(a, b, bias=None, act=ACT_NONE, out_fp32=False, split_k=1, out=None, mask=None):
    """dr_gemm_nt_bf16[_ex]: act(a b^T + bias) with a [M, K], b [N, K] bf16
    (row strides free, unit column stride), K % 64 == 0, N % 8 == 0; fp32
    accumulate; bf16 (or fp32) [M, N] output.  split_k > 1: K cut into
    chunks summed in chunk order (deterministic).  mask (bf16 [M, N]): the
    result is zeroed where mask <= 0 (act ACT_MASK, a ReLU's backward)."""
    dev = _dev(a)
    M, K = a.shape
    N = b.shape[0]
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or b.shape[1] != K \
            or a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("gemm_nt needs bf16 a [M, K], b [N, K] with unit column stride")
    odt = torch.float32 if out_fp32 else torch.bfloat16
    if out is None:
        out = torch.empty((M, N), dtype=odt, device=dev)
    bb = None if bias is None else bias.to(torch.float32).contiguous()
    wsb = lib().dr_gemm_nt_workspace_size(M, N, split_k)
    ws = workspace(wsb, dev) if wsb else None
    if mask is not None:
        if mask.dtype != torch.bfloat16 or tuple(mask.shape) != (M, N) or mask.stride(1) != 1:
            raise ValueError("mask must be bf16 [M, N] with unit column stride")
        act = ACT_MASK
    check(lib().dr_gemm_nt_bf16_ex(ptr(a), a.stride(0), ptr(b), b.stride(0), M, N, K, ptr(bb), act,
                                   ptr(mask), mask.stride(0) if mask is not None else 0, ptr(out),
                                   out.stride(0), 1 if out_fp32 else 0, split_k, ptr(ws), wsb,
                                   stream_handle(dev)))
    _post(dev)
    return out


def gemm_tn(g, x, split_k=1, colsum=False):
    """dr_gemm_tn_bf16: g^T x in fp32 for g [R, N], x [R, K] bf16 (unit column
    strides, R % 64 == 0): [N, K]; colsum=True also returns g's fp32 column
    sums (the bias gradient): (dw, db)."""
    dev = _dev(g)
    R, N = g.shape
    K = x.shape[1]
    if g.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or x.shape[0] != R \
            or g.stride(1) != 1 or x.stride(1) != 1:
        raise ValueError("gemm_tn needs bf16 g [R, N], x [R, K] with unit column stride")
    out = torch.empty((N, K), dtype=torch.float32, device=dev)
    cs = torch.empty(N, dtype=torch.float32, device=dev) if colsum else None
    wsb = lib().dr_gemm_tn_workspace_size(N, K, split_k, 1 if colsum else 0)
    ws = workspace(wsb, dev) if wsb else None
    check(lib().dr_gemm_tn_bf16(ptr(g), g.stride(0), ptr(x), x.stride(0), R, N, K, ptr(out), K,
                                ptr(cs), split_k, ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return (out, cs) if colsum else out


def transpose_bf16(x, colsum=False):
    """dr_transpose_bf16: [R, C] bf16 (unit column stride) -> contiguous [C, R].
    colsum=True (dr_transpose_bf16_colsum): also the fp32 column sums of x,
    from per-64-row-tile partials summed in tile order; returns (out, sums)."""
    dev = _dev(x)
    R, Cc = x.shape
    if x.dtype != torch.bfloat16 or x.stride(1) != 1:
        raise ValueError("transpose_bf16 needs a bf16 matrix with unit column stride")
    out = torch.empty((Cc, R), dtype=torch.bfloat16, device=dev)
    if not colsum:
        check(lib().dr_transpose_bf16(ptr(x), R, Cc, x.stride(0), ptr(out), R,
                                      stream_handle(dev)))
        _post(dev)
        return out
    part = torch.empty(((R + 63) // 64, Cc), dtype=torch.float32, device=dev)
    check(lib().dr_transpose_bf16_colsum(ptr(x), R, Cc, x.stride(0), ptr(out), R, ptr(part),
                                         stream_handle(dev)))
    _post(dev)
    return out, part.sum(0)


def crossnet_dx(u, wt, g):
    """dr_crossnet_dx_bf16: dx = u W + g for a cross layer's input gradient,
    wt = W^T [d, d] bf16 contiguous; u, g [B, d] bf16, d % 64 == 0.  One
    rounding of the fp32 u W + g (torch.addmm(g, u, W) in bf16)."""
    dev = _dev(u)
    B, d = u.shape
    if d % 64 or tuple(g.shape) != (B, d) or tuple(wt.shape) != (d, d) or any(
            t.dtype != torch.bfloat16 for t in (u, wt, g)):
        raise ValueError("crossnet_dx needs bf16 u, g [B, d] and wt [d, d] with d % 64 == 0")
    u, wt, g = u.contiguous(), wt.contiguous(), g.contiguous()
    dx = torch.empty((B, d), dtype=torch.bfloat16, device=dev)
    check(lib().dr_crossnet_dx_bf16(ptr(u), ptr(wt), ptr(g), B, d, ptr(dx), stream_handle(dev)))
    _post(dev)
    return dx


def crossnet_dw(u, xl):
    """dr_crossnet_dw_bf16: dW = u^T x_l (fp32 [d, d]) for a cross layer's
    weight gradient; u, xl [B, d] bf16, d and B multiples of 64 (None
    otherwise: the caller falls back to a library GEMM)."""
    dev = _dev(u)
    B, d = u.shape
    if d % 64 or B % 64 or tuple(xl.shape) != (B, d) or any(
            t.dtype != torch.bfloat16 for t in (u, xl)):
        return None
    u, xl = u.contiguous(), xl.contiguous()
    dw = torch.empty((d, d), dtype=torch.float32, device=dev)
    wsb = lib().dr_crossnet_dw_workspace_size(B, d)
    ws = workspace(wsb, dev)
    check(lib().dr_crossnet_dw_bf16(ptr(u), ptr(xl), B, d, ptr(dw), ptr(ws), wsb,
                                    stream_handle(dev)))
    _post(dev)
    return dw


def crossnet_backward_elem(g, x0, lin, acc=None):
    """dr_crossnet_backward_elem_bf16: the elementwise part of a cross
    layer's backward in one pass.  g, x0, lin [B, d] bf16; acc [B, d] fp32
    running dx0 (None: start at 0; updated in place).  Returns (u = g * x0
    bf16, acc + g * lin fp32, db = column sums of u fp32)."""
    dev = _dev(g)
    B, d = g.shape
    for t in (g, x0, lin):
        if t.dtype != torch.bfloat16 or tuple(t.shape) != (B, d):
            raise ValueError("crossnet_backward_elem needs bf16 [B, d] operands")
    g, x0, lin = g.contiguous(), x0.contiguous(), lin.contiguous()
    out = torch.empty((B, d), dtype=torch.float32, device=dev) if acc is None else acc
    if acc is not None and (acc.dtype != torch.float32 or not acc.is_contiguous()
                            or tuple(acc.shape) != (B, d)):
        raise ValueError("acc must be a contiguous fp32 [B, d] tensor")
    u = torch.empty((B, d), dtype=torch.bfloat16, device=dev)
    db = torch.empty(d, dtype=torch.float32, device=dev)
    wsb = lib().dr_crossnet_backward_workspace_size(B, d)
    ws = workspace(wsb, dev)
    check(lib().dr_crossnet_backward_elem_bf16(ptr(g), ptr(x0), ptr(lin), ptr(acc), ptr(out),
                                               ptr(u), ptr(db), B, d, ptr(ws), wsb,
                                               stream_handle(dev)))
    _post(dev)
    return u, out, db


# ---------------------------------------------------------------------------
# DIN attention (modelzoo/DIN/script/utils.py:264-309, script/model.py:94-98)
# ---------------------------------------------------------------------------
def din_attention_input(query, facts):
    """din_all = concat([q, f, q - f, q * f], -1): query [B, H], facts
    [B, T, H] -> [B, T, 4H] (utils.py:280-282)."""
    dev = _dev(facts)
    B, T, H = facts.shape
    q, f = _c(query, torch.float32), _c(facts, torch.float32)
    out = torch.empty((B, T, 4 * H), dtype=torch.float32, device=dev)
    check(lib().dr_din_attention_input(ptr(q), ptr(f), B, T, H, ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def din_attention_input_grad(query, facts, top_grad, grad_facts=None):
    """Backward of din_attention_input -> (grad_query [B, H], grad_facts
    [B, T, H]); when grad_facts is given it is accumulated into in place."""
    dev = _dev(facts)
    B, T, H = facts.shape
    q, f, g = _c(query, torch.float32), _c(facts, torch.float32), _c(top_grad, torch.float32)
    gq = torch.empty((B, H), dtype=torch.float32, device=dev)
    acc = grad_facts is not None
    if not acc:
        grad_facts = torch.empty((B, T, H), dtype=torch.float32, device=dev)
    elif not grad_facts.is_contiguous() or grad_facts.dtype != torch.float32:
        raise ValueError("grad_facts must be a contiguous fp32 tensor")
    check(lib().dr_din_attention_input_grad(ptr(q), ptr(f), ptr(g), B, T, H, ptr(gq),
                                            ptr(grad_facts), int(acc), stream_handle(dev)))
    _post(dev)
    return gq, grad_facts


DIN_MLP_HIDDEN = (16, 32, 36, 64)


class DinMlpBuffers(object):
    """The fused DIN attention MLP's buffers (dr_din_mlp_buf) for one step:
    forward state kept for the backward, backward outputs the weight
    gradients are formed from.  cap = batch * seq_len (no host read of the
    valid-position count P).  The per-position buffers (h1t, h2t, da1t, da2t,
    xt, dsc) hold positions [0, P) only: with the hand weight-gradient pass
    their columns p >= P stay unwritten (uninitialised memory) and that pass
    stops at P itself; the library GEMM path asks the backward to zero the
    backward buffers' columns past P (zero_tail = 1).

    fill (test hook, None in use): a value every per-position buffer is
    filled with when allocated, so a test can show the hand pass never reads
    past P (NaN there must not reach a gradient)."""

    fill = None

    def __init__(self, B, T, H, n1, n2, dev):
        cap = B * T
        i32, f32 = torch.int32, torch.float32
        e = lambda shape, dt=f32: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
        self.pos, self.cnt, self.off = e(cap, i32), e(B, i32), e(B + 1, i32)
        self.w1p, self.w2t, self.cq = e((n1, 2 * H)), e((n1, n2)), e((B, n1))
        self.h1t, self.h2t = self._filled(e((n1, cap))), self._filled(e((n2, cap)))
        self.da1t = self.da2t = self.xt = self.dsc = self.dqp = self.s1 = self.dq2 = None
        self.B, self.T, self.H, self.n1, self.n2, self.cap = B, T, H, n1, n2, cap

    def _filled(self, t):
        return t if self.fill is None else t.fill_(self.fill)

    def alloc_backward(self, dev):
        B, H, n1, n2, cap = self.B, self.H, self.n1, self.n2, self.cap
        e = lambda shape: self._filled(torch.empty(shape, dtype=torch.float32, device=dev))  # noqa: E731
        self.da1t, self.da2t, self.xt = e((n1, cap)), e((n2, cap)), e((2 * H, cap))
        self.dsc, self.dqp, self.s1, self.dq2 = e(cap), e((H, cap)), e((B, n1)), e((B, H))

    def struct(self):
        names = [f[0] for f in _lib.DrDinMlpBuf._fields_]
        return _lib.DrDinMlpBuf(*[ptr(getattr(self, n)) for n in names])


def din_mlp_forward(query, facts, mask, w1, b1, w2, b2, w3, b3):
    """Fused attention MLP (dr_din_mlp_forward): scores [B, T] at the valid
    positions (the padded ones are 0 here and masked by the pool), and the
    buffers its backward needs."""
    dev = _dev(facts)
    B, T, H = facts.shape
    n1, n2 = w1.shape[0], w2.shape[0]
    q, f, m = _c(query, torch.float32), _c(facts, torch.float32), _c(mask, torch.float32)
    w1c, b1c, w2c, b2c = (_c(x, torch.float32) for x in (w1, b1, w2, b2))
    w3c, b3c = _c(w3.reshape(-1), torch.float32), _c(b3.reshape(-1), torch.float32)
    buf = DinMlpBuffers(B, T, H, n1, n2, dev)
    scores = torch.zeros((B, T), dtype=torch.float32, device=dev)
    st = buf.struct()
    check(lib().dr_din_mlp_forward(ptr(q), ptr(f), ptr(m), B, T, H, ptr(w1c), ptr(b1c), n1,
                                   ptr(w2c), ptr(b2c), n2, ptr(w3c), ptr(b3c), ptr(scores),
                                   C.byref(st), stream_handle(dev)))
    _post(dev)
    return scores, buf


# the attention MLP's weight gradients: one hand split-K pass on the matrix
# cores (dr_din_mlp_wgrad_valid over the valid positions, default: 0.085 + 0.008
# ms at DIN's configs[3])
# or, DR_DIN_WGRAD=lib, library GEMMs + reductions (≈ 0.25 ms;
# profiles/r05_din_wgrad.log)
_DIN_WGRAD_HAND = os.environ.get("DR_DIN_WGRAD", "hand") == "hand"


def din_mlp_backward(query, facts, w1, w3, buf, grad_scores, grad_facts):
    """Backward of din_mlp_forward: adds the MLP's part to grad_facts (in
    place) and returns (grad_query, dW1, db1, dW2, db2, dw3, db3); the weight
    gradients come from the feature-major per-position buffers: one hand pass
    bounded by the valid count, or library split-K GEMMs over cap (for which
    the backward zeroes the columns past the valid count)."""
    dev = _dev(facts)
    B, T, H = facts.shape
    n1, n2, cap = buf.n1, buf.n2, buf.cap
    q, f = _c(query, torch.float32), _c(facts, torch.float32)
    w3c = _c(w3.reshape(-1), torch.float32)
    gs = _c(grad_scores, torch.float32)
    if not grad_facts.is_contiguous() or grad_facts.dtype != torch.float32:
        raise ValueError("grad_facts must be a contiguous fp32 tensor")
    buf.alloc_backward(dev)
    st = buf.struct()
    hand = _DIN_WGRAD_HAND and 2 * H in (32, 64, 72, 128) and (n1, n2) == (80, 40) and cap % 4 == 0
    # the hand pass stops at the valid count P itself: the columns p >= P of
    # the per-position buffers stay unwritten (1.25 KB per position less)
    check(lib().dr_din_mlp_backward_tail(ptr(q), ptr(f), B, T, H, n1, n2, ptr(w3c), ptr(gs),
                                         ptr(grad_facts), C.byref(st), 0 if hand else 1,
                                         stream_handle(dev)))
    _post(dev)
    S = 64
    while S > 1 and cap % S:
        S //= 2
    L = cap // S

    def kred(a_t, b_t):   # a_t [M, cap], b_t [N, cap] -> a_t b_t^T, split over cap
        M, N = a_t.shape[0], b_t.shape[0]
        return torch.bmm(a_t.view(M, S, L).transpose(0, 1),
                         b_t.view(N, S, L).permute(1, 2, 0)).sum(0)
    w1f = w1.float()
    A, Cm = w1f[:, :H], w1f[:, 2 * H:3 * H]
    gq = buf.s1 @ (A + Cm) + buf.dq2
    Gq = buf.s1.t() @ q
    db1 = buf.s1.sum(0)
    if hand:
        # one split-K pass for G, dW2, db2, dw3, db3 (dr_din_mlp_wgrad)
        gout, wout = n1 * 2 * H, n2 * n1
        out = torch.empty(gout + wout + 2 * n2 + 1, dtype=torch.float32, device=dev)
        wsb = lib().dr_din_mlp_wgrad_workspace_size(n1, 2 * H, n2)
        ws = workspace(wsb, dev)
        check(lib().dr_din_mlp_wgrad_valid(ptr(buf.da1t), ptr(buf.xt), ptr(buf.da2t),
                                           ptr(buf.h1t), ptr(buf.h2t), ptr(buf.dsc), cap,
                                           ptr(buf.off[B:]), n1, 2 * H, n2, ptr(out), ptr(ws), wsb,
                                           stream_handle(dev)))
        _post(dev)
        G = out[:gout].view(n1, 2 * H)
        dW2 = out[gout:gout + wout].view(n2, n1)
        db2 = out[gout + wout:gout + wout + n2]
        dw3 = out[gout + wout + n2:gout + wout + 2 * n2].view(1, n2)
        db3 = out[gout + wout + 2 * n2:].view(1)
    else:
        G = kred(buf.da1t, buf.xt)
        dW2 = kred(buf.da2t, buf.h1t)
        db2 = buf.da2t.sum(1)
        dw3 = (buf.h2t @ buf.dsc).view(1, n2)
        db3 = buf.dsc.sum().view(1)
    Gf, Gqf = G[:, :H], G[:, H:]
    dW1 = torch.cat([Gq, Gf, Gq - Gf, Gqf], 1)
    return gq, dW1, db1, dW2, db2, dw3, db3


def din_dice_forward(x, alpha, epsilon):
    """Dice (utils.py:12-35) over a [B, n] fp32 batch in one kernel
    (dr_din_dice_forward) -> (y [B, n], stats [2, n] = column mean, std)."""
    dev = _dev(x)
    B, n = x.shape
    xc, a = _c(x, torch.float32), _c(alpha, torch.float32)
    y = torch.empty((B, n), dtype=torch.float32, device=dev)
    st = torch.empty((2, n), dtype=torch.float32, device=dev)
    check(lib().dr_din_dice_forward(ptr(xc), ptr(a), B, n, float(epsilon), ptr(y), ptr(st),
                                    stream_handle(dev)))
    _post(dev)
    return y, st


def din_dice_backward(x, grad_y, alpha, stats, epsilon):
    """-> (grad_x [B, n], grad_alpha [n]) through the batch statistics."""
    dev = _dev(x)
    B, n = x.shape
    xc, g, a = _c(x, torch.float32), _c(grad_y, torch.float32), _c(alpha, torch.float32)
    gx = torch.empty((B, n), dtype=torch.float32, device=dev)
    ga = torch.empty(n, dtype=torch.float32, device=dev)
    check(lib().dr_din_dice_backward(ptr(xc), ptr(g), ptr(a), ptr(_c(stats, torch.float32)), B, n,
                                     float(epsilon), ptr(gx), ptr(ga), stream_handle(dev)))
    _post(dev)
    return gx, ga


def din_fcn_input_forward(uid, item, his_sum, att, gamma, beta, scale):
    """Model_DIN's fcn input + inference batch_normalization in one pass
    (dr_din_fcn_input_forward) -> [B, Du + 4H]."""
    dev = _dev(item)
    B, H = item.shape
    Du = uid.shape[1]
    u, i, h, a = (_c(t, torch.float32) for t in (uid, item, his_sum, att))
    gm, bt = _c(gamma, torch.float32), _c(beta, torch.float32)
    out = torch.empty((B, Du + 4 * H), dtype=torch.float32, device=dev)
    check(lib().dr_din_fcn_input_forward(ptr(u), ptr(i), ptr(h), ptr(a), ptr(gm), ptr(bt), B, Du,
                                         H, float(scale), ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def din_fcn_input_backward(grad, uid, item, his_sum, att, gamma, scale):
    """-> (g_uid, g_item, g_his_sum, g_att, g_gamma, g_beta)."""
    dev = _dev(item)
    B, H = item.shape
    Du = uid.shape[1]
    g = _c(grad, torch.float32)
    u, i, h, a = (_c(t, torch.float32) for t in (uid, item, his_sum, att))
    gm = _c(gamma, torch.float32)
    e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)  # noqa: E731
    gu, gi, gh, ga, gg, gb = e(B, Du), e(B, H), e(B, H), e(B, H), e(Du + 4 * H), e(Du + 4 * H)
    check(lib().dr_din_fcn_input_backward(ptr(g), ptr(u), ptr(i), ptr(h), ptr(a), ptr(gm), B, Du,
                                          H, float(scale), ptr(gu), ptr(gi), ptr(gh), ptr(ga),
                                          ptr(gg), ptr(gb), stream_handle(dev)))
    _post(dev)
    return gu, gi, gh, ga, gg, gb


def din_attention_pool(scores, mask, facts, with_sum=True):
    """Masked softmax over the history + weighted sum (din_attention, mode
    'SUM', utils.py:286-303) and the history sum (model.py:98) in one pass.
    scores / mask [B, T], facts [B, T, H] -> (att [B, H], his_sum [B, H] or
    None, alphas [B, T])."""
    dev = _dev(facts)
    B, T, H = facts.shape
    s, m, f = _c(scores, torch.float32), _c(mask, torch.float32), _c(facts, torch.float32)
    att = torch.empty((B, H), dtype=torch.float32, device=dev)
    hs = torch.empty((B, H), dtype=torch.float32, device=dev) if with_sum else None
    al = torch.empty((B, T), dtype=torch.float32, device=dev)
    check(lib().dr_din_attention_pool(ptr(s), ptr(m), ptr(f), B, T, H, ptr(att), ptr(hs), ptr(al),
                                      stream_handle(dev)))
    _post(dev)
    return att, hs, al


def din_attention_pool_grad(alphas, mask, facts, grad_att, grad_sum=None, out=None):
    """-> (grad_scores [B, T], grad_facts [B, T, H]); out: a contiguous fp32
    [B, T, H] buffer to write grad_facts into (e.g. a slice of the lookup's
    gradient)."""
    dev = _dev(facts)
    B, T, H = facts.shape
    a, m, f = _c(alphas, torch.float32), _c(mask, torch.float32), _c(facts, torch.float32)
    ga = _c(grad_att, torch.float32)
    gs = None if grad_sum is None else _c(grad_sum, torch.float32)
    gsc = torch.empty((B, T), dtype=torch.float32, device=dev)
    if out is not None:
        if out.shape != (B, T, H) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("out must be a contiguous fp32 [B, T, H] tensor")
        gf = out
    else:
        gf = torch.empty((B, T, H), dtype=torch.float32, device=dev)
    check(lib().dr_din_attention_pool_grad(ptr(a), ptr(m), ptr(f), ptr(ga), ptr(gs), B, T, H,
                                           ptr(gsc), ptr(gf), stream_handle(dev)))
    _post(dev)
    return gsc, gf


# ---------------------------------------------------------------------------
# Row-sharded exchange helpers
# ---------------------------------------------------------------------------
def partition_by_owner(keys, world, n_dev=None):
    """Stable bucket of keys by owner = key % world (SOK selectKernel,
    all2all_input_dispatcher.cu:36-126; EV rule embedding_ops.py:207-209).
    Returns (keys_sorted, perm, send_counts[world] int64)."""
    dev = _dev(keys)
    k = _c(keys, torch.int64)
    n = k.numel()
    ko = torch.empty_like(k)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    wsb = lib().dr_partition_workspace_size(n)
    ws = workspace(wsb, dev)
    check(lib().dr_partition_by_owner(ptr(k), n, ptr(n_dev), world, ptr(ko), ptr(perm),
                                      ptr(counts), ptr(ws), wsb, stream_handle(dev)))
    _post(dev)
    return ko, perm, counts


def partition_by_owner_mod(keys, world, premod, n_dev=None):
    """partition_by_owner with owner = (key % premod) % world (floor mods):
    premod = 1000 is the EV partition rule ids % 1000 % np
    (python/ops/embedding_ops.py:207-209)."""
    dev = _dev(keys)
    k = _c(keys, torch.int64)
    n = k.numel()
    ko = torch.empty_like(k)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    wsb = lib().dr_partition_workspace_size(n)
    ws = workspace(wsb, dev)
    check(lib().dr_partition_by_owner_mod(ptr(k), n, ptr(n_dev), world, int(premod), ptr(ko),
                                          ptr(perm), ptr(counts), ptr(ws), wsb,
                                          stream_handle(dev)))
    _post(dev)
    return ko, perm, counts


def rows_scatter(src, perm, out, n_dev=None):
    """out[perm[j]] = src[j]"""
    dev = _dev(src)
    check(lib().dr_rows_scatter(ptr(src), ptr(perm), perm.numel(), ptr(n_dev), src.shape[1],
                                ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def rows_pack(src, perm, out, n_dev=None):
    """out[j] = src[perm[j]]"""
    dev = _dev(src)
    check(lib().dr_rows_pack(ptr(src), ptr(perm), perm.numel(), ptr(n_dev), src.shape[1],
                             ptr(out), stream_handle(dev)))
    _post(dev)
    return out


def fill_synthetic(table, seed):
    """table[r, c] = hash(seed, r, c) in [-1, 1) (regenerable: synth_value)."""
    dev = _dev(table)
    check(lib().dr_fill_synthetic(ptr(table), table.shape[0], table.shape[1], seed,
                                  stream_handle(dev)))
    return table


def synth_value(seed, row, col):
    return lib().dr_synth_value(seed, row, col)
