"""embedding_lookup / embedding_lookup_sparse / safe_embedding_lookup_sparse /
fused_embedding_lookup_sparse with DeepRec's argument semantics
(python/ops/embedding_ops.py:94-675,1209-1344; python/ops/fused_embedding_ops.py:18-97),
executed by the HIP engine.

The sparse lookup is fused on the GPU: dedup (first-occurrence unique) ->
EV insert-on-miss resolve -> one grouped gather+pool kernel that reads the
table rows directly and reduces them in the reference's CPU association
order, so the [U, D] intermediate of the reference composition is never
materialised.  Backward produces IndexedSlices per unique id through the
deterministic segment-grad kernels and hands them to the optimizers
(training.py) via `pending_grads`, like TF's sparse gradient path.
"""
import os

import torch

from . import _lib, ops
from ._lib import COMBINERS, ORDER_ALI, ORDER_SEQ, DrPoolDesc, check, lib, ptr, stream_handle, workspace
from .kv_variable_ops import EmbeddingVariable, IndexedSlices, PendingRowSlices


class SparseTensor(object):
    """indices [nnz, 2] int64 (row-major canonical), values [nnz], dense_shape."""

    def __init__(self, indices, values, dense_shape):
        self.indices = indices
        self.values = values
        self.dense_shape = tuple(int(x) for x in dense_shape)

    @property
    def device(self):
        return self.values.device


class DenseTable(object):
    """A plain [rows, dim] embedding table (tf.Variable of a hash_bucket column;
    ResourceGather path, resource_variable_ops.cc:628).  Sparse gradients are
    queued in pending_grads as IndexedSlices (row ids)."""

    def __init__(self, weight):
        self.weight = weight.to(torch.float32).contiguous()
        self.dim = self.weight.shape[1]
        self.device = self.weight.device
        self.pending_grads = []

    def get_shape(self):
        return tuple(self.weight.shape)


def _anchor(holder):
    a = getattr(holder, "_anchor", None)
    if a is None:
        a = torch.zeros(1, device=holder.device, requires_grad=True)
        holder._anchor = a
    return a


# DEEPREC_AMD_FUSED_ONEHOT=0 selects the resolve -> pool pipeline for
# forward-only one-hot lookups (A/B measurement; both are HIP paths).
_FUSED_ONEHOT = os.environ.get("DEEPREC_AMD_FUSED_ONEHOT", "1") != "0"
# training lookups of filter-free EVs without Unique, backward regrouped by
# the resolved rows (A/B switch; both are HIP paths)
_ROWS_GRAD = os.environ.get("DEEPREC_AMD_ROWS_GRAD", "1") != "0"


def _ev_default_dev(ev):
    d = getattr(ev, "_default_dev", None)
    if d is None:
        d = ev.default_value.contiguous()
        ev._default_dev = d
    return d


class _Feature(object):
    """One feature's prepared lookup (everything the pool kernel needs).

    seg: sorted segment ids -- an int32/int64 vector, or the [nnz, 2] int64
    sp_ids.indices (read in place, stride 2: no per-step conversion)."""

    def __init__(self, params, values, seg, batch, weights, combiner, max_norm, onehot=False):
        vd = getattr(params, "value_dtype", torch.float32)
        if vd != torch.float32 and not (vd == torch.bfloat16 and isinstance(params,
                                                                           EmbeddingVariable)):
            # the pooled lookups are fp32 kernels, as the reference's fused
            # and GPU EV lookups are (double EVs: sparse_read); bf16 EVs pool
            # in fp32 and hand back bf16 (DR_POOL_BF16)
            raise _lib.DeepRecError(_lib.INVALID_ARGUMENT,
                                    "embedding lookups pool float32 / bf16 EVs; %s is %s"
                                    % (getattr(params, "name", params), params.value_dtype))
        self.bf16 = vd == torch.bfloat16
        if self.bf16 and (params.dim % 8 or max_norm is not None and torch.is_grad_enabled()):
            raise _lib.DeepRecError(_lib.INVALID_ARGUMENT,
                                    "bf16 EV lookups need dim % 8 == 0 (and no max_norm "
                                    "when a gradient is recorded)")
        self.params = params
        # one id per row (a valid [B, 1] SparseTensor with nnz == B): bag b is
        # nnz b, so the pool kernel needs no bag offsets (DR_POOL_ONEHOT).
        self.onehot = bool(onehot) and weights is None and max_norm is None
        self.bag_off = None
        self.group = None
        # ids as given: possibly a strided view (a column of a record-major
        # [B, T] id matrix), read in place by the fused one-hot lookup;
        # `values` is the contiguous vector every other kernel takes
        self.raw_values = values
        self._values = values if values.is_contiguous() else None
        if seg.dim() == 2:
            self.seg64, self.seg_stride = seg.contiguous(), seg.shape[1]
        elif seg.dtype == torch.int64:
            self.seg64, self.seg_stride = seg.contiguous(), 1
        else:
            self.seg64, self.seg_stride = seg.to(torch.int64).contiguous(), 1
        self._seg32 = seg if seg.dim() == 1 and seg.dtype == torch.int32 else None
        self.batch = batch
        self.weights = weights
        self.combiner = combiner
        self.max_norm = max_norm
        self.uniq = self.idx = self.U = self.rows = self.rowsel = None
        self.defaults = None

    @property
    def values(self):
        if self._values is None:
            self._values = self.raw_values.contiguous()
        return self._values

    @property
    def seg(self):
        """int32 segment ids (embedding_ops.py:587-589), built on demand."""
        if self._seg32 is None:
            s = self.seg64 if self.seg_stride == 1 else self.seg64[:, 0]
            self._seg32 = s.to(torch.int32).contiguous()
        return self._seg32


def _is_onehot(sp_ids, nnz):
    return len(sp_ids.dense_shape) == 2 and sp_ids.dense_shape[1] == 1 and \
        nnz == sp_ids.dense_shape[0]


def _bag_offsets_all(feats, skip_onehot=False):
    """CSR bag offsets of every feature in one launch."""
    import ctypes as C
    feats = [f for f in feats if f.bag_off is None and not (skip_onehot and f.onehot)]
    if not feats:
        return
    T = len(feats)
    dev = feats[0].values.device
    offs = [torch.empty(f.batch + 1, dtype=torch.int32, device=dev) for f in feats]
    B = feats[0].batch
    if any(f.batch != B for f in feats) or T > _lib.MAX_GROUP:
        for f, o in zip(feats, offs):
            f.bag_off = ops.bag_offsets(f.seg64 if f.seg_stride == 1 else f.seg, f.batch)
        return
    segs = (C.c_void_p * T)(*[f.seg64.data_ptr() for f in feats])
    strides = (C.c_int64 * T)(*[f.seg_stride for f in feats])
    ns = (C.c_int64 * T)(*[f.values.numel() for f in feats])
    outs = (C.c_void_p * T)(*[o.data_ptr() for o in offs])
    check(lib().dr_bag_offsets_grouped(segs, strides, ns, T, B, outs, stream_handle(dev)))
    ops._post(dev)
    for f, o in zip(feats, offs):
        f.bag_off = o


def _prepare(f, need_unique):
    dev = f.values.device
    _bag_offsets_all([f], skip_onehot=True)
    p = f.params
    if isinstance(p, EmbeddingVariable):
        with_counts = p.filter_freq != 0          # embedding_ops.py:592-596
        f.uniq, f.idx, cnt, f.U = ops.unique_device(f.values, with_counts)
        f.defaults = p._defaults_for(f.uniq.numel(), None)
        f.rows = p.resolve(f.uniq, n_dev=f.U, counts=cnt, defaults=f.defaults)
    elif need_unique:
        f.uniq, f.idx, _, f.U = ops.unique_device(f.values)


def _desc(f, out, out_stride):
    d = DrPoolDesc()
    p = f.params
    if isinstance(p, EmbeddingVariable) and f.rowsel is not None:
        d.pool = p.pool()
        d.pool_rows = 1 << 62
        d.ids = ptr(f.rowsel)                      # pre-resolved row per nnz
        d.default_rows = ptr(_ev_default_dev(p))
        d.default_stride = 0
    elif isinstance(p, EmbeddingVariable):
        d.pool = p.pool()
        d.pool_rows = 0
        d.idx = ptr(f.idx)
        d.rows = ptr(f.rows)
        if f.defaults is not None:
            d.default_rows = ptr(f.defaults)
            d.default_stride = p.dim
        else:
            d.default_rows = ptr(_ev_default_dev(p))
            d.default_stride = 0
    else:
        t = p.weight if isinstance(p, DenseTable) else p
        d.pool = ptr(t)
        d.pool_rows = t.shape[0]
        d.ids = ptr(f.values)
    d.bag_off = None if f.bag_off is None else ptr(f.bag_off)
    d.weights = ptr(f.weights)
    d.out = out.data_ptr()
    d.out_stride = out_stride   # elements of the output type
    d.combiner = COMBINERS[f.combiner]
    d.max_norm = -1.0 if f.max_norm is None else float(f.max_norm)
    return d


def _grad_to_slices(f, g, col, top_stride):
    """Pooled grad (feature columns from `col` of rows of `top_stride`
    floats) -> IndexedSlices over the unique ids, through the grouped
    backward kernel with one feature (chunked runs: a hot id does not
    serialise one wave)."""
    if f.uniq is None:
        f.uniq, f.idx, _, f.U = ops.unique_device(f.values)
    grp = _UniqueGroup([f], f.uniq, f.U, [0, f.values.numel()])
    return grp.grads(g, [col], top_stride)[0]


def _clip_grad(f, gs):
    """Backward of the max_norm clip (embedding_ops._clip, applied to the
    unique rows before pooling) on the per-unique grads gs, in place."""
    p = f.params
    if isinstance(p, EmbeddingVariable):
        if f.defaults is not None:
            dflt, stride = f.defaults, p.dim
        else:
            dflt, stride = _ev_default_dev(p), 0
        ops.clip_by_norm_grad(gs, p.pool(), f.rows, f.max_norm, default_rows=dflt,
                              default_stride=stride, n_dev=f.U)
    else:
        t = p.weight if isinstance(p, DenseTable) else p
        ops.clip_by_norm_grad(gs, t.detach(), f.uniq, f.max_norm, pool_rows=t.shape[0],
                              n_dev=f.U)


def _trainable_tensors(feats):
    """Plain torch tables of the features that require grad (each once)."""
    out = []
    for f in feats:
        p = f.params
        if torch.is_tensor(p) and p.requires_grad and all(p is not q for q in out):
            out.append(p)
    return out


def _dense_grad(p, sl):
    """IndexedSlices -> dense [R, D] gradient of a plain tensor table (the
    reference's IndexedSlices-to-Tensor conversion, an UnsortedSegmentSum in
    ascending slice order; rows past num_valid are skipped)."""
    n = sl.indices.numel()
    seg = sl.indices
    if sl.num_valid is not None:
        seg = torch.where(torch.arange(n, device=seg.device) < sl.num_valid, seg,
                          torch.full_like(seg, -1))
    return ops.unsorted_segment_sum(sl.values[:n], seg.to(torch.int32), p.shape[0])


class _LookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, feats, order, fused_rows, out_dtype, *tensors):
        ctx.feats = feats
        ctx.tensors = tensors
        if fused_rows:
            return _fused_onehot(feats, order, with_rows=True, out_dtype=out_dtype)
        return _pool_all(feats, order, out_dtype=out_dtype)

    @staticmethod
    def backward(ctx, grad_out):
        # gradients are fp32 whatever the table dtype (a bf16 EV's pooled
        # output hands a bf16 gradient back: widened once here)
        g = grad_out.float().contiguous()
        dense = _queue_grads(ctx.feats, g, 0, g.shape[1], ctx.tensors)
        return (None, None, None, None, None) + tuple(dense)


def _queue_grads(feats, g, col0, total, tensors=()):
    """Per-feature IndexedSlices from the pooled grad g (rows of `total`
    floats, feature columns starting at col0), queued on the variables;
    returns the dense grads of the trainable plain tensors `tensors`."""
    cols, col = [], col0
    for f in feats:
        cols.append(col)
        col += f.params.dim if not torch.is_tensor(f.params) else f.params.shape[1]
    dense = [None] * len(tensors)
    done = set()
    for i, f in enumerate(feats):
        holder = f.params
        if torch.is_tensor(holder):
            for j, t in enumerate(tensors):
                if t is holder:
                    d = _dense_grad(t, _grad_to_slices(f, g, cols[i], total))
                    dense[j] = d if dense[j] is None else dense[j] + d
            continue
        grp = getattr(f, "group", None)
        if grp is not None:
            if id(grp) in done:
                continue
            done.add(id(grp))
            pos = {id(x): j for j, x in enumerate(feats)}
            sls = grp.grads(g, [cols[pos[id(x)]] for x in grp.feats], total)
            for x, sl in zip(grp.feats, sls):
                x.params.pending_grads.append(sl)
            continue
        holder.pending_grads.append(_grad_to_slices(f, g, cols[i], total))
    return dense


class _StackFn(torch.autograd.Function):
    """[x0 | e_1 | ... | e_T] as one [B, 1+T, D] tensor: the pooling writes
    straight into the interaction input (no concat copy) and the backward
    reads the embeddings' grads in place with the row stride."""

    @staticmethod
    def forward(ctx, x0, anchor, feats, order):
        B, D = x0.shape
        T = len(feats)
        X = torch.empty((B, 1 + T, D), dtype=torch.float32, device=x0.device)
        X[:, 0].copy_(x0)
        _pool_all(feats, order, out=X.view(B, (1 + T) * D)[:, D:])
        ctx.feats = feats
        return X

    @staticmethod
    def backward(ctx, gX):
        g = gX.contiguous()
        B, F, D = g.shape
        _queue_grads(ctx.feats, g.view(B, F * D), D, F * D)
        return g[:, 0], None, None, None


def embedding_stack(x0, params_list, sp_ids_list, combiner="sum"):
    """torch.stack([x0] + [embedding_lookup_sparse(p, sp) ...], 1) for EVs of
    dim x0.shape[1] (DLRM's interaction input, modelzoo/DLRM/train.py:214-219)."""
    if any(getattr(p, "value_dtype", None) == torch.bfloat16 for p in params_list):
        raise _lib.DeepRecError(_lib.INVALID_ARGUMENT,
                                "embedding_stack builds the fp32 dot-interaction input; "
                                "bf16 EVs: embedding_lookup_sparse_multi")
    feats = []
    for p, sp in zip(params_list, sp_ids_list):
        v = sp.values.to(torch.int64).contiguous()
        feats.append(_Feature(p, v, _seg_of(sp), sp.dense_shape[0], None, combiner, None,
                              onehot=_is_onehot(sp, v.numel())))
    need_grad = torch.is_grad_enabled()
    if _groupable(feats):
        _prepare_group(feats, need_grad)
    else:
        for f in feats:
            _prepare(f, need_unique=False)
    anchor = [_anchor(f.params) for f in feats if not torch.is_tensor(f.params)][0]
    return _StackFn.apply(x0, anchor, feats, ORDER_ALI)


def _prepare_all(feats, need_grad):
    """One grouped Unique + resolve per set of EVs of equal dim (WDL's 64 / 128
    columns: two launches sets instead of 26 per-feature pipelines); other
    parameters one by one."""
    if _groupable(feats) or (need_grad and len(feats) == 1 and _rows_eligible(feats)):
        _prepare_group(feats, need_grad)
        return
    sets = {}
    for f in feats:
        p = f.params
        key = None
        if isinstance(p, EmbeddingVariable) and not callable(p.initializer):
            key = (p.dim, str(p.device), f.batch)
        sets.setdefault(key, []).append(f)
    for key, fs in sets.items():
        while fs:
            chunk, fs = fs[:_lib.MAX_GROUP], fs[_lib.MAX_GROUP:]
            if key is not None and _groupable(chunk):
                _prepare_group(chunk, need_grad)
            else:
                for f in chunk:
                    _prepare(f, need_unique=False)


def _groupable(feats):
    p0 = feats[0].params
    return (len(feats) > 1 and len(feats) <= _lib.MAX_GROUP
            and all(isinstance(f.params, EmbeddingVariable) and not callable(f.params.initializer)
                    and f.params.dim == p0.dim and f.params.device == p0.device for f in feats))


def _concat_values(feats, koff):
    """The features' ids as one vector; a view when they already sit back to
    back in one buffer (e.g. rows of a [T, nnz] id matrix), else a copy."""
    v0 = feats[0].values
    if all(f.values.dtype == torch.int64 and f.values.is_contiguous()
           and f.values.untyped_storage().data_ptr() == v0.untyped_storage().data_ptr()
           and f.values.data_ptr() == v0.data_ptr() + 8 * koff[t] for t, f in enumerate(feats)):
        return torch.as_strided(v0, (koff[-1],), (1,))
    return torch.cat([f.values for f in feats])


def _prepare_group(feats, need_grad=True):
    """All features of a step at once: one grouped unique, one grouped EV
    resolve (insert-on-miss + filters), then per-feature bag offsets.

    Forward-only lookups of filter-free EVs skip the Unique: every nnz is
    resolved straight into the EV's hash table, whose CAS insert is itself
    the dedup (LookupOrCreate is idempotent, embedding_var.h:320-339), so
    the outputs and the EV contents equal the unique -> gather pipeline's.
    Unique is still built when counts feed a Counter/Bloom filter or when a
    gradient needs the unique ids (embedding_ops.py:592-596)."""
    import ctypes as C
    dev = feats[0].values.device
    T = len(feats)
    koff = [0]
    for f in feats:
        koff.append(koff[-1] + f.values.numel())
    vals = _concat_values(feats, koff)
    with_counts = any(f.params.filter_freq != 0 for f in feats)
    by_rows = need_grad and _rows_eligible(feats)
    if not with_counts and (not need_grad or by_rows):
        rowsel = torch.empty(koff[-1], dtype=torch.int64, device=dev)
        handles = (C.c_void_p * T)(*[f.params.handle.value for f in feats])
        wsb = lib().dr_ev_resolve_workspace_size(koff[-1])
        ws = workspace(wsb, dev)
        check(lib().dr_ev_resolve_grouped(handles, T, ptr(vals), ops._koff_array(koff), None, None,
                                          ptr(rowsel), ptr(ws), wsb, stream_handle(dev)))
        ops._post(dev)
        _bag_offsets_all(feats, skip_onehot=True)
        for t, f in enumerate(feats):
            f.uniq = f.idx = f.rows = f.U = f.defaults = f.group = None
            f.rowsel = rowsel[koff[t]:koff[t + 1]]
        if by_rows:
            group = _RowGroup(feats, vals, rowsel, koff)
            for f in feats:
                f.group = group
        return
    uniq, idx, cnt, U = ops.unique_grouped(vals, koff, with_counts)
    rows = torch.empty(koff[-1], dtype=torch.int64, device=dev)
    handles = (C.c_void_p * T)(*[f.params.handle.value for f in feats])
    ndev = (C.c_void_p * T)(*[U.data_ptr() + 8 * t for t in range(T)])
    wsb = lib().dr_ev_resolve_workspace_size(koff[-1])
    ws = workspace(wsb, dev)
    check(lib().dr_ev_resolve_grouped(handles, T, ptr(uniq), ops._koff_array(koff), ndev, ptr(cnt),
                                      ptr(rows), ptr(ws), wsb, stream_handle(dev)))
    rowsel = torch.empty(koff[-1], dtype=torch.int64, device=dev)
    check(lib().dr_rows_per_nnz(ptr(rows), ptr(idx), ops._koff_array(koff), T, ptr(rowsel),
                                stream_handle(dev)))
    ops._post(dev)
    _bag_offsets_all(feats, skip_onehot=True)
    for t, f in enumerate(feats):
        f.uniq = uniq[koff[t]:koff[t + 1]]
        f.idx = idx[koff[t]:koff[t + 1]]
        f.rows = rows[koff[t]:koff[t + 1]]
        f.rowsel = rowsel[koff[t]:koff[t + 1]]
        f.U = U[t:t + 1]
        f.defaults = None
    group = _UniqueGroup(feats, uniq, U, koff)
    for f in feats:
        f.group = group


def _rows_eligible(feats):
    """The training forward may skip the Unique when every feature is a
    filter-free EV without max_norm (the clip's backward needs the unique
    rows): the backward then regroups by the resolved rows
    (dr_pool_grad_rows_grouped, same IndexedSlices as Unique would give)."""
    if not _ROWS_GRAD or len(feats) > _lib.MAX_GROUP:
        return False
    p0 = feats[0].params
    return all(isinstance(f.params, EmbeddingVariable) and f.params.filter_freq == 0
               and not callable(f.params.initializer) and f.max_norm is None
               and f.params.dim == p0.dim and f.params.device == p0.device
               and f.batch == feats[0].batch for f in feats)


class _RowGroup(object):
    """Features resolved straight into their EVs (no Unique): the backward is
    one dr_pool_grad_rows_grouped over the forward's rows.  Unique ids come
    out in first-occurrence order, gradients by address (kv_variable_ops.
    IndexedSlices.grad_ptr) so the optimizer reads the pooled gradient in
    place."""

    def __init__(self, feats, vals, rowsel, koff, rows_record=False):
        self.feats = feats
        self.vals = vals
        self.rowsel = rowsel
        self.koff = koff
        self.rows_record = rows_record   # rowsel record-major [B, T] (DR_LOOKUP_ROWS_RECORD)

    def grads(self, g, cols, top_stride):
        dev = g.device
        D = self.feats[0].params.dim
        T = len(self.feats)
        descs = (_lib.DrPoolGradDesc * T)()
        keep = [g]
        for t, f in enumerate(self.feats):
            d = descs[t]
            if f.weights is not None:
                _bag_offsets_all([f])
                d.weights = ptr(f.weights)
                if f.combiner != "sum":
                    q = ops.bag_weight_scale(f.weights, f.bag_off, f.combiner)
                    keep.append(q)
                    d.bag_scale = ptr(q)
            d.top_grad = g.data_ptr() + 4 * cols[t]
            d.top_stride = top_stride
            if f.onehot:
                d.bag_off, d.seg, d.seg_stride = None, None, 0
            else:
                _bag_offsets_all([f])
                d.bag_off = ptr(f.bag_off)
                d.seg = ptr(f.seg64)
                d.seg_stride = f.seg_stride
            d.nnz = f.values.numel()
            d.combiner = COMBINERS[f.combiner]
        pend = _RowsPending(self, descs, tuple(keep), D, dev)
        if pend.fusable() or pend.launch_side():
            return [PendingRowSlices(pend, t, D) for t in range(T)]
        return pend.materialize()


# record-major row records of the one-hot training lookup (A/B switch)
_ROWS_RECORD = os.environ.get("DR_ROWS_RECORD", "1") != "0"

# SGD applies of row-grouped backwards fused with the backward (A/B switch)
_FUSED_SGD = os.environ.get("DR_ROWS_FUSED_SGD", "1") != "0"

# Row-grouped backwards that are not fused into an SGD apply run on a side
# stream, joined when their IndexedSlices are first used (A/B switch
# DR_ROWS_SIDE_STREAM=0): the serial walk of a long run (DIN's padding id, a
# popular category) keeps a few CUs for hundreds of microseconds, and the
# lookups of one step (DIN's uid, target and history) then walk at once,
# beside the dense backward, instead of one after another.
_SIDE_STREAM = os.environ.get("DR_ROWS_SIDE_STREAM", "1") != "0"
# ... also inside a captured hipGraph (the fork and join captured as events;
# A/B, off: bit-equal, but the DIN graph step measured 3.27-3.29 ms with it
# against 3.19 without -- the walk is the critical path either way)
_SIDE_STREAM_CAPTURE = os.environ.get("DR_ROWS_SIDE_STREAM_CAPTURE", "0") == "1"
_SIDE_STREAMS = {}
_N_SIDE = 4


def _side_stream(dev):
    pool = _SIDE_STREAMS.get(dev.index)
    if pool is None:
        pool = _SIDE_STREAMS[dev.index] = [[torch.cuda.Stream(device=dev)
                                            for _ in range(_N_SIDE)], 0]
    s = pool[0][pool[1] % _N_SIDE]
    pool[1] += 1
    return s


class _RowsPending(object):
    """A row-grouped backward waiting for its consumer (PendingRowSlices):
    materialize() forms the IndexedSlices (dr_pool_grad_rows_grouped_ex, as
    the eager backward), apply_sgd() runs the backward fused with the SGD
    update (dr_ev_pool_grad_rows_apply_sgd).  Holds the pooled gradient and
    the forward's rows until then."""

    def __init__(self, group, descs, keep, D, dev):
        self.group, self.descs, self.keep, self.D, self.dev = group, descs, keep, D, dev
        self.evs = [f.params for f in group.feats]
        self.slices = None
        self.applied = False
        self.done = None   # side-stream launch: the event its consumer waits on
        self._alive = None  # (captured fork) buffers held until the join

    def fusable(self):
        if (not _FUSED_SGD or self.slices is not None or self.applied or self.D % 4
                or self.done is not None):
            return False
        if len({id(e) for e in self.evs}) != len(self.evs):
            return False          # one EV twice: sequential rounds, not one fused pass
        return all(d.top_grad % 16 == 0 and d.top_stride % 4 == 0 for d in self.descs)

    def materialize(self):
        if self.done is not None:   # formed on a side stream: the consumer waits for it
            torch.cuda.current_stream(self.dev).wait_event(self.done)
            self.done = None
            self._alive = None
            ops._post(self.dev)
        if self.slices is None:
            if self.applied:
                raise RuntimeError("this gradient was already applied (fused SGD)")
            self.slices = self._form()
        return self.slices

    def launch_side(self):
        """Form the IndexedSlices now on a side stream (after everything the
        current stream has queued, the pooled gradient included); the first
        use of any of them makes its stream wait for the result.  Every
        buffer the launch touches is recorded on the side stream, so the
        caching allocator does not hand it out again before the launch ends.
        While a graph is being captured (DR_ROWS_SIDE_STREAM_CAPTURE=1, A/B)
        the fork and its join are captured too: instead of
        record_stream, every buffer is held by this object until the join in
        materialize(), which the step's optimizer reaches inside the same
        capture (an unjoined fork would fail the capture loudly)."""
        capturing = torch.cuda.is_current_stream_capturing()
        if (not _SIDE_STREAM or self.dev.type != "cuda" or self.slices is not None
                or (capturing and not _SIDE_STREAM_CAPTURE)):
            return False
        main = torch.cuda.current_stream(self.dev)
        side = _side_stream(self.dev)
        side.wait_stream(main)
        used = []
        self.slices = self._form(side, used)
        if capturing:
            self._alive = used + [self.group.rowsel, self.group.vals] + list(self.keep)
        else:
            for t in used + [self.group.rowsel, self.group.vals] + list(self.keep):
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(side)
        self.done = torch.cuda.Event()
        self.done.record(side)
        return True

    def _form(self, side=None, used=None):
        grp, dev, D = self.group, self.dev, self.D
        T = len(grp.feats)
        n = grp.koff[-1]
        m = max(n, 1)
        uniq = torch.empty(m, dtype=torch.int64, device=dev)
        U = torch.empty(T, dtype=torch.int64, device=dev)
        gptr = torch.empty(m, dtype=torch.int64, device=dev)
        urows = torch.empty(m, dtype=torch.int64, device=dev)
        gu = torch.empty((m, D), dtype=torch.float32, device=dev)
        keep = self.keep + (gu,)
        limit = max(lib().dr_ev_row_capacity(f.params.handle) for f in grp.feats)
        wsb = lib().dr_pool_grad_rows_workspace_size(n)
        ws = workspace(wsb, dev)
        if used is not None:
            used += [uniq, U, gptr, urows, gu, ws]
        check(lib().dr_pool_grad_rows_grouped_ex2(
            self.descs, T, grp.feats[0].batch, D, ptr(grp.rowsel), int(grp.rows_record),
            max(int(limit), 1), ptr(grp.vals), 1, ptr(uniq), ptr(urows), ptr(U), ptr(gptr),
            ptr(gu), ptr(ws), wsb, side.cuda_stream if side is not None else stream_handle(dev)))
        if side is None:
            ops._post(dev)
        k = grp.koff
        return [IndexedSlices(None, uniq[k[t]:k[t + 1]], U[t:t + 1], True,
                              grad_ptr=gptr[k[t]:k[t + 1]], dim=D, keep=keep,
                              rows=urows[k[t]:k[t + 1]])
                for t in range(T)]

    def apply_sgd(self, lr, global_step, stream):
        import ctypes as C
        grp = self.group
        T = len(grp.feats)
        n = grp.koff[-1]
        wsb = lib().dr_ev_pool_grad_rows_sgd_workspace_size(n, self.D)
        ws = workspace(wsb, self.dev)
        P = C.c_void_p * T
        check(lib().dr_ev_pool_grad_rows_apply_sgd_ex(
            P(*[e.handle.value for e in self.evs]), self.descs, T, grp.feats[0].batch, self.D,
            ptr(grp.rowsel), int(grp.rows_record), lr, global_step, ptr(ws), wsb, stream))
        ops._post(self.dev)
        self.applied = True
        self.keep = ()


class _UniqueGroup(object):
    """Features that went through one dr_unique_grouped call: their backward
    runs as one dr_pool_grad_grouped (one sort for all features)."""

    def __init__(self, feats, uniq, U, koff):
        self.feats = feats
        self.uniq = uniq
        self.U = U
        self.koff = koff

    def grads(self, g, cols, top_stride):
        """g: the pooled grad (base tensor), cols[t]: column of feature t.
        Returns one IndexedSlices per feature."""
        dev = g.device
        p0 = self.feats[0].params
        D = p0.shape[1] if torch.is_tensor(p0) else p0.dim
        descs = (_lib.DrPoolGradDesc * len(self.feats))()
        keep = []   # per-bag weight divisors, alive until the launch is queued
        for t, f in enumerate(self.feats):
            d = descs[t]
            if f.weights is not None:
                # embedding_ops.py:609-651: (g / weight_sum) * w, unsorted_segment_sum
                _bag_offsets_all([f])
                d.weights = ptr(f.weights)
                if f.combiner != "sum":
                    q = ops.bag_weight_scale(f.weights, f.bag_off, f.combiner)
                    keep.append(q)
                    d.bag_scale = ptr(q)
            d.top_grad = g.data_ptr() + 4 * cols[t]
            d.top_stride = top_stride
            if f.onehot:
                d.bag_off, d.seg, d.seg_stride = None, None, 0
            else:
                _bag_offsets_all([f])
                d.bag_off = ptr(f.bag_off)
                d.seg = ptr(f.seg64)
                d.seg_stride = f.seg_stride
            d.idx = ptr(f.idx)
            d.nnz = f.values.numel()
            d.num_unique = ptr(f.U)
            d.combiner = COMBINERS[f.combiner]
        n = self.koff[-1]
        gu = torch.empty((max(n, 1), D), dtype=torch.float32, device=dev)
        wsb = lib().dr_pool_grad_grouped_workspace_size(n)
        ws = workspace(wsb, dev)
        check(lib().dr_pool_grad_grouped(descs, len(self.feats), self.feats[0].batch, D, ptr(gu),
                                         ptr(ws), wsb, stream_handle(dev)))
        ops._post(dev)
        k = self.koff
        for t, f in enumerate(self.feats):
            if f.max_norm is not None and k[t + 1] > k[t]:
                _clip_grad(f, gu[k[t]:k[t + 1]])
        return [IndexedSlices(gu[k[t]:k[t + 1]], self.uniq[k[t]:k[t + 1]], self.U[t:t + 1], True)
                for t in range(len(self.feats))]


# feature-major one-hot lookups visiting the ids table by table: A/B switch,
# off -- measured slower than output order (profiles/r03_ab_table_order.log)
_TABLE_ORDER = os.environ.get("DR_LOOKUP_TABLE_ORDER", "0") == "1"


def _fused_onehot_ok(feats):
    p0 = feats[0].params
    if not (len(feats) <= _lib.MAX_GROUP and isinstance(p0, EmbeddingVariable)):
        return False
    B = feats[0].batch
    D = p0.dim
    for f in feats:
        p = f.params
        if not (isinstance(p, EmbeddingVariable) and f.onehot and f.batch == B
                and p.dim == D and p.device == p0.device and p.filter_freq == 0
                and not callable(p.initializer) and f.raw_values.numel() == B
                and p.value_dtype == p0.value_dtype):
            return False
    W = p0.row_words
    return W % 4 == 0 and W <= 256 and len(feats) * B < (1 << 31)


def _record_major(feats):
    """Base address of a record-major [B, T] int64 id matrix whose column t
    is feature t's ids (SparseTensor values = ids[:, t], e.g. a Criteo
    record batch of 26 categorical ids per sample), else None."""
    T = len(feats)
    v0 = feats[0].raw_values
    if T < 2 or v0.dtype != torch.int64 or v0.dim() != 1 or v0.stride(0) != T:
        return None
    st = v0.untyped_storage().data_ptr()
    for t, f in enumerate(feats):
        v = f.raw_values
        if (v.dtype != torch.int64 or v.dim() != 1 or v.stride(0) != T
                or v.untyped_storage().data_ptr() != st or v.data_ptr() != v0.data_ptr() + 8 * t):
            return None
    return v0.data_ptr()


def _out_dtype(feats, out_dtype):
    """Pooled output dtype: fp32 (bf16 EVs too: the reference casts bf16
    embeddings to float32 before pooling, embedding_ops.py:606-607), or bf16
    when asked for and every feature is a bf16 EV (the DCN-v2 input path)."""
    if out_dtype in (None, torch.float32):
        return torch.float32
    if out_dtype == torch.bfloat16 and all(f.bf16 for f in feats):
        return torch.bfloat16
    raise _lib.DeepRecError(_lib.INVALID_ARGUMENT,
                            "out_dtype %s: float32, or bfloat16 for bf16 EVs" % (out_dtype,))


def _fused_onehot(feats, order, with_rows=False, out_dtype=None):
    """One-hot lookup of filter-free EVs in one fused launch
    (dr_ev_lookup_onehot: probe + row copy, no resolve pass).  Forward-only,
    or (with_rows) a training forward that also records the row of every id
    for the row-grouped backward (_RowGroup).  Returns the [B, T*D] output,
    or None when the features do not qualify."""
    import ctypes as C
    if not _fused_onehot_ok(feats):
        return None
    p0 = feats[0].params
    B = feats[0].batch
    D = p0.dim
    T = len(feats)
    dev = feats[0].raw_values.device
    koff = [t * B for t in range(T + 1)]
    odt = _out_dtype(feats, out_dtype)
    # bf16 EVs: widened into an fp32 output, or copied bitwise into a bf16 one
    flags = _lib.LOOKUP_OUT_BF16 if odt == torch.bfloat16 else 0
    out = torch.empty((B, T * D), dtype=odt, device=dev)
    handles = (C.c_void_p * T)(*[f.params.handle.value for f in feats])
    wsb = lib().dr_ev_lookup_onehot_workspace_size(T, B)
    ws = workspace(wsb, dev)
    rec = None if with_rows else _record_major(feats)
    if rec is not None:
        # the features are the columns of one record-major [B, T] id matrix:
        # read in place, in the kernel's (b, t) visiting order
        check(lib().dr_ev_lookup_onehot_ex(handles, T, rec, T, 1, B, ptr(out), T * D, order, flags,
                                           None, ptr(ws), wsb, stream_handle(dev)))
        ops._post(dev)
        return out
    vals = _concat_values(feats, koff)
    if _TABLE_ORDER:
        # feature-major [T, B] ids: visit them table by table so the id reads
        # and the row records are contiguous (same results)
        flags |= _lib.LOOKUP_TABLE_ORDER
    if with_rows:
        rowsel = torch.empty(T * B, dtype=torch.int64, device=dev)
        # the row records record-major [B, T] (whole lines in output order;
        # the backward reads them strided): A/B switch DR_ROWS_RECORD=0
        rec = _ROWS_RECORD and not (flags & _lib.LOOKUP_TABLE_ORDER)
        if rec:
            flags |= _lib.LOOKUP_ROWS_RECORD
        check(lib().dr_ev_lookup_onehot_ex(handles, T, ptr(vals), 1, B, B, ptr(out), T * D, order,
                                           flags, ptr(rowsel), ptr(ws), wsb, stream_handle(dev)))
        group = _RowGroup(feats, vals, rowsel, koff, rows_record=rec)
        for t, f in enumerate(feats):
            f.uniq = f.idx = f.rows = f.U = f.defaults = None
            # (a per-feature slice exists only in position order)
            f.rowsel = None if rec else rowsel[koff[t]:koff[t + 1]]
            f.group = group
    else:
        check(lib().dr_ev_lookup_onehot_ex(handles, T, ptr(vals), 1, B, B, ptr(out), T * D, order,
                                           flags, None, ptr(ws), wsb, stream_handle(dev)))
    ops._post(dev)
    return out


def _run(feats, order=ORDER_ALI, need_grad=None, out_dtype=None):
    """Grouped pooled lookup of features sharing the batch -> [B, sum(D_t)]."""
    tensors = _trainable_tensors(feats) if torch.is_grad_enabled() else []
    if need_grad is None:
        need_grad = torch.is_grad_enabled() and (
            bool(tensors) or any(not torch.is_tensor(f.params) for f in feats))
    if not need_grad and _FUSED_ONEHOT:
        out = _fused_onehot(feats, order, out_dtype=out_dtype)
        if out is not None:
            return out
    # training forward of one-hot filter-free EVs: the fused probe + copy
    # kernel records the rows for the row-grouped backward
    fused_rows = (need_grad and _FUSED_ONEHOT and not tensors and _rows_eligible(feats)
                  and _fused_onehot_ok(feats))
    if not fused_rows:
        _prepare_all(feats, need_grad)
    if need_grad:
        anchors = [_anchor(f.params) for f in feats if not torch.is_tensor(f.params)]
        return _LookupFn.apply(anchors[0] if anchors else None, feats, order, fused_rows,
                               out_dtype, *tensors)
    return _pool_all(feats, order, out_dtype=out_dtype)


def _pool_all(feats, order, out=None, out_dtype=None):
    dev = feats[0].values.device
    B = feats[0].batch
    dims = [f.params.dim if not torch.is_tensor(f.params) else f.params.shape[1] for f in feats]
    total = sum(dims)
    bf16 = feats[0].bf16
    if any(f.bf16 != bf16 for f in feats):
        raise _lib.DeepRecError(_lib.INVALID_ARGUMENT,
                                "one pooled output: all features bf16 EVs or none")
    odt = _out_dtype(feats, out_dtype if out is None else out.dtype)
    if out is None:
        out = torch.empty((B, total), dtype=odt, device=dev)
    elif out.shape[0] != B or out.stride(1) != 1 or out.shape[1] < total:
        raise ValueError("out must be a [B, >= %d] view with unit column stride" % total)
    stride = out.stride(0)
    # group consecutive features of equal dim into <= 32-table launches
    col = 0
    i = 0
    while i < len(feats):
        j = i
        while j < len(feats) and dims[j] == dims[i] and j - i < _lib.MAX_GROUP:
            j += 1
        onehot = all(f.onehot for f in feats[i:j])
        if not onehot:
            _bag_offsets_all(feats[i:j])
        descs = []
        c = col
        for f in feats[i:j]:
            descs.append(_desc(f, out[:, c:], stride))
            c += dims[i]
        ops.pool_grouped(descs, B, dims[i], order, dev, onehot=onehot, bf16=bf16,
                         out_bf16=odt == torch.bfloat16)
        col = c
        i = j
    return out


def _seg_of(sp_ids):
    # segment_ids = sp_ids.indices[:, 0] (embedding_ops.py:587-589), read in
    # place from the [nnz, 2] indices; the int32 cast happens on demand.
    ind = sp_ids.indices
    if ind.dtype != torch.int64:
        ind = ind.to(torch.int64)
    return ind.contiguous()


def embedding_lookup_sparse(params, sp_ids, sp_weights=None, partition_strategy="mod", name=None,
                            combiner=None, max_norm=None):
    """tf.nn.embedding_lookup_sparse (embedding_ops.py:480-675), 2-D sp_ids."""
    if combiner is None:
        combiner = "mean"
    if combiner not in ("mean", "sqrtn", "sum", "tile"):
        raise ValueError("combiner must be one of 'mean', 'sqrtn', 'sum' or 'tile'")
    if combiner == "tile":
        return _tile_lookup_sparse(params if isinstance(params, (list, tuple)) else [params],
                                   sp_ids, sp_weights, partition_strategy, max_norm)
    if isinstance(params, (list, tuple)):
        if len(params) == 1:
            params = params[0]
        else:
            return _partitioned_lookup_sparse(params, sp_ids, sp_weights, partition_strategy,
                                              combiner, max_norm)
    values = sp_ids.values.to(torch.int64).contiguous()
    w = None if sp_weights is None else sp_weights.values.to(torch.float32).contiguous()
    f = _Feature(params, values, _seg_of(sp_ids), sp_ids.dense_shape[0], w, combiner, max_norm,
                 onehot=_is_onehot(sp_ids, values.numel()))
    return _run([f])


def embedding_lookup_sparse_multi(params_list, sp_ids_list, combiner="mean", max_norm=None,
                                  out_dtype=None):
    """Grouped lookup of several features (one pooled launch per 32 tables);
    returns the input_layer concatenation [B, sum(D_t)], fp32 -- or, for
    bf16 EVs with out_dtype=torch.bfloat16, bf16 (one-id bags copied
    bitwise, longer bags pooled in fp32 and rounded once)."""
    feats = []
    for p, sp in zip(params_list, sp_ids_list):
        v = sp.values.to(torch.int64)      # strided views stay views (_record_major)
        feats.append(_Feature(p, v, _seg_of(sp), sp.dense_shape[0], None, combiner, max_norm,
                              onehot=_is_onehot(sp, v.numel())))
    return _run(feats, out_dtype=out_dtype)


def embedding_lookup(params, ids, partition_strategy="mod", name=None, max_norm=None,
                     ev_init_value=None, counts=None):
    """tf.nn.embedding_lookup (embedding_ops.py:94-342, 346)."""
    if isinstance(params, (list, tuple)) and len(params) == 1:
        params = params[0]
    if isinstance(params, (list, tuple)):
        flat = ids.reshape(-1).to(torch.int64).contiguous()
        init = None
        if ev_init_value is not None:
            D = params[0].dim if not torch.is_tensor(params[0]) else params[0].shape[1]
            init = torch.as_tensor(ev_init_value, dtype=torch.float32, device=flat.device)
            init = init.expand(flat.numel(), D).contiguous()
        res = _partitioned_gather(params, flat, None, counts, init, partition_strategy)
        res = res.reshape(tuple(ids.shape) + (res.shape[1],))
    elif isinstance(params, EmbeddingVariable):
        res = params.sparse_read(ids, counts=counts, ev_init_value=ev_init_value)
    else:
        t = params.weight if isinstance(params, DenseTable) else params
        res = ops.gather(t, ids)
    if max_norm is not None:
        r2 = res.reshape(-1, res.shape[-1])
        l2 = torch.sqrt((r2 * r2).sum(1, keepdim=True))
        r2 = r2 * max_norm / torch.maximum(l2, torch.tensor(max_norm, device=r2.device))
        res = r2.reshape(res.shape)
    return res


def _partition_plan(params, flat, n_dev, partition_strategy):
    """dynamic_partition of ids over the partitions (embedding_ops.py:207-252):
    EVs by ids % 1000 % np, dense tables by "mod" (id % np, id // np) or
    "div" (dim-0 boundaries).  Returns (perm [n] int32, offs host list[np+1],
    per-partition new ids [n] int64 in partition order); entries past n_dev
    (device count) fall outside every partition.  One host read of the
    partition sizes, as dynamic_partition's own output shapes need."""
    np_ = len(params)
    n = flat.numel()
    if isinstance(params[0], EmbeddingVariable):
        keys, perm, counts = ops.partition_by_owner_mod(flat, np_, 1000, n_dev=n_dev)
        new_ids = keys
    else:
        if partition_strategy == "mod":
            assign = flat
        elif partition_strategy == "div":
            sizes = [p.get_shape()[0] if not torch.is_tensor(p) else p.shape[0] for p in params]
            total = sum(sizes)
            ipp, extras = total // np_, total % np_
            assign = torch.maximum(flat // (ipp + 1), (flat - extras) // max(ipp, 1))
        else:
            raise ValueError("Unrecognized partition strategy: " + partition_strategy)
        _, perm, counts = ops.partition_by_owner(assign, np_, n_dev=n_dev)
        src = flat.index_select(0, perm.to(torch.int64).clamp_(0, max(n - 1, 0)))
        if partition_strategy == "mod":
            new_ids = src // np_
        else:
            pa = torch.maximum(src // (ipp + 1), (src - extras) // max(ipp, 1))
            new_ids = torch.where(pa < extras, src % (ipp + 1), (src - extras) % max(ipp, 1))
    c = counts.cpu().tolist()
    offs = [0]
    for x in c:
        offs.append(offs[-1] + int(x))
    return perm, offs, new_ids


class _PartitionedGatherFn(torch.autograd.Function):
    """embedding_lookup over a partitioned variable: dynamic_partition ->
    per-partition gather (EV KvResourceGather[V1] / dense ResourceGather) ->
    parallel_dynamic_stitch (embedding_ops.py:207-299).  Backward: the
    stitch's grad gathered back per partition = IndexedSlices queued on each
    EV / DenseTable (or a dense grad for a plain tensor partition)."""

    @staticmethod
    def forward(ctx, anchor, params, flat, n_dev, counts, init, strategy, *tensors):
        dev = flat.device
        n = flat.numel()
        p0 = params[0]
        D = p0.dim if not torch.is_tensor(p0) else p0.shape[1]
        perm, offs, new_ids = _partition_plan(params, flat, n_dev, strategy)
        perm64 = perm.to(torch.int64)
        emb_part = torch.empty((max(n, 1), D), dtype=torch.float32, device=dev)
        for p, prm in enumerate(params):
            a, b = offs[p], offs[p + 1]
            if b == a:
                continue
            ids_p = new_ids[a:b]
            if isinstance(prm, EmbeddingVariable):
                sel = perm64[a:b]
                cnt = None if counts is None else counts.index_select(0, sel)
                ini = None if init is None else init.index_select(0, sel)
                dflt = prm._defaults_for(b - a, None) if ini is None else ini
                emb_part[a:b] = _ev_sparse_read(prm, ids_p, cnt, dflt)
            else:
                t = prm.weight if isinstance(prm, DenseTable) else prm
                emb_part[a:b] = ops.gather(t.detach(), ids_p)
        out = torch.zeros((n, D), dtype=torch.float32, device=dev)
        if offs[-1]:
            ops.rows_scatter(emb_part, perm[:offs[-1]], out)
        ctx.params, ctx.perm, ctx.offs, ctx.new_ids = params, perm, offs, new_ids
        ctx.tensors = tensors
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        offs, params = ctx.offs, ctx.params
        D = g.shape[1]
        gp = torch.empty((max(offs[-1], 1), D), dtype=torch.float32, device=g.device)
        if offs[-1]:
            ops.rows_pack(g, ctx.perm[:offs[-1]], gp)
        dense = [None] * len(ctx.tensors)
        for p, prm in enumerate(params):
            a, b = offs[p], offs[p + 1]
            if b == a:
                continue
            sl = IndexedSlices(gp[a:b], ctx.new_ids[a:b], unique=True)
            if torch.is_tensor(prm):
                for j, t in enumerate(ctx.tensors):
                    if t is prm:
                        d = _dense_grad(t, sl)
                        dense[j] = d if dense[j] is None else dense[j] + d
            else:
                prm.pending_grads.append(sl)
        return (None,) * 7 + tuple(dense)


def _ev_sparse_read(ev, ids, counts, defaults):
    """KvResourceGather[V1] of device ids with an explicit [n, D] default
    block (or None = the EV's default row)."""
    n = ids.numel()
    out = torch.empty((n, ev.dim), dtype=torch.float32, device=ev.device)
    cnt = None if counts is None else counts.to(torch.int32).contiguous()
    wsb = lib().dr_ev_gather_workspace_size(n)
    ws = workspace(wsb, ev.device)
    check(lib().dr_ev_gather(ev.handle, ptr(ids.contiguous()), n, ptr(defaults), ptr(cnt), ptr(out),
                             ptr(ws), wsb, stream_handle(ev.device)))
    ops._post(ev.device)
    return out


def _partitioned_gather(params, flat, n_dev, counts, init, strategy):
    tensors = [p for p in params if torch.is_tensor(p) and p.requires_grad]
    anchors = [_anchor(p) for p in params if not torch.is_tensor(p)]
    if torch.is_grad_enabled() and (anchors or tensors):
        return _PartitionedGatherFn.apply(anchors[0] if anchors else None, params, flat, n_dev,
                                          counts, init, strategy, *tensors)
    with torch.no_grad():
        return _PartitionedGatherFn.forward(_Ctx(), None, params, flat, n_dev, counts, init,
                                            strategy)


class _Ctx(object):
    pass


class _TileSumFn(torch.autograd.Function):
    """unsorted_segment_sum of the gathered rows onto row * C + column
    (_tile_combine_embedding, embedding_ops.py:468-476): the serial-order
    HIP segment sum forward; backward gathers the output gradient at each
    position's segment (UnsortedSegmentSum's gradient, math_grad.py)."""

    @staticmethod
    def forward(ctx, rows, seg, nseg):
        ctx.save_for_backward(seg)
        return ops.unsorted_segment_sum(rows, seg, nseg)

    @staticmethod
    def backward(ctx, g):
        (seg,) = ctx.saved_tensors
        return g.contiguous().index_select(0, seg.to(torch.int64)), None, None


def _tile_lookup_sparse(params, sp_ids, sp_weights, partition_strategy, max_norm):
    """combiner="tile" (embedding_ops.py:646-651,665-671): the embedding of
    each (row, column) of sp_ids lands in its own D-wide column block of a
    [B, C * D] output (C = dense_shape[1]); entries sharing a (row, column)
    are summed.  unique (with counts for EV filters) -> gather of the unique
    ids (EV / dense / partitioned, with its backward) -> max_norm clip ->
    gather by idx (x weights) -> segment sum onto row * C + column."""
    values = sp_ids.values.to(torch.int64).contiguous()
    B, C = int(sp_ids.dense_shape[0]), int(sp_ids.dense_shape[1])
    with_counts = isinstance(params[0], EmbeddingVariable) and params[0].filter_freq != 0
    uniq, idx, cnt, U = ops.unique_device(values, with_counts)
    emb = _partitioned_gather(list(params), uniq, U, cnt, None, partition_strategy)
    if max_norm is not None:
        l2 = torch.sqrt((emb * emb).sum(1, keepdim=True))
        emb = emb * max_norm / torch.maximum(l2, torch.tensor(max_norm, device=emb.device))
    rows = emb.index_select(0, idx.to(torch.int64))
    if sp_weights is not None:
        rows = rows * sp_weights.values.to(rows.dtype).reshape(-1, 1)
    ind = sp_ids.indices.to(torch.int64)
    seg = (ind[:, 0] * C + ind[:, 1]).to(torch.int32).contiguous()
    out = _TileSumFn.apply(rows.contiguous(), seg, B * C)
    return out.reshape(B, C * out.shape[1])


def _partitioned_lookup_sparse(params, sp_ids, sp_weights, partition_strategy, combiner,
                               max_norm):
    """embedding_lookup_sparse over a partitioned variable
    (embedding_ops.py:589-651): unique (with counts when an EV filter needs
    them) -> partitioned gather of the unique ids -> pooled by idx.  The
    gathered [U, D] block is the pooling's table, so max_norm / weights /
    combiner and their backward are the single-table path's."""
    values = sp_ids.values.to(torch.int64).contiguous()
    B = sp_ids.dense_shape[0]
    with_counts = isinstance(params[0], EmbeddingVariable) and params[0].filter_freq != 0
    uniq, idx, cnt, U = ops.unique_device(values, with_counts)
    emb = _partitioned_gather(params, uniq, U, cnt, None, partition_strategy)
    w = None if sp_weights is None else sp_weights.values.to(torch.float32).contiguous()
    f = _Feature(emb, idx.to(torch.int64), _seg_of(sp_ids), B, w, combiner, max_norm)
    return _run([f])


# ---------------------------------------------------------------------------
# safe_embedding_lookup_sparse (embedding_ops.py:1209-1344)
# ---------------------------------------------------------------------------
def sparse_prune_fill(sp_ids, sp_weights=None, default_id=0, prune=0):
    """_prune_invalid_ids / _prune_invalid_weights (prune 1 / 2) and
    sparse_fill_empty_rows (embedding_ops.py:1299-1310) in one GPU call
    (dr_sparse_prune_fill).  Returns (SparseTensor ids, SparseTensor weights
    or None, is_row_empty bool [B], reverse_index_map int64 [nnz])."""
    ind = sp_ids.indices.to(torch.int64).contiguous()
    val = sp_ids.values.to(torch.int64).contiguous()
    dev = val.device
    w = None if sp_weights is None else sp_weights.values.to(torch.float32).contiguous()
    n = val.numel()
    rank = ind.shape[1] if ind.dim() == 2 else 2
    B = int(sp_ids.dense_shape[0])
    cap = n + B
    oind = torch.empty((max(cap, 1), rank), dtype=torch.int64, device=dev)
    oval = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
    ow = None if w is None else torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
    rev = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    empty = torch.empty(max(B, 1), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    wsb = lib().dr_sparse_fill_workspace_size(n, B)
    ws = workspace(wsb, dev)
    check(lib().dr_sparse_prune_fill(ptr(ind), rank, ptr(val), ptr(w), n, B, int(prune),
                                     int(default_id or 0), 1.0, ptr(oind), ptr(oval), ptr(ow),
                                     ptr(rev), ptr(empty), ptr(cnt), ptr(ws), wsb,
                                     stream_handle(dev)))
    ops._post(dev)
    m = int(cnt.item())          # the output's size (SparseFillEmptyRows allocates it too)
    sp = SparseTensor(oind[:m], oval[:m], sp_ids.dense_shape)
    spw = None if ow is None else SparseTensor(oind[:m], ow[:m], sp_ids.dense_shape)
    return sp, spw, empty[:B].to(torch.bool), rev[:n]


def sparse_fill_empty_rows(sp_input, default_value, name=None):
    """tf.sparse.fill_empty_rows (SparseFillEmptyRows) for int64 ids:
    returns (filled SparseTensor, empty_row_indicator)."""
    sp, _, empty, _ = sparse_prune_fill(sp_input, None, default_value, 0)
    return sp, empty


def _prune_and_fill(sp_ids, sp_weights, combiner, default_id, prune):
    mode = 0 if not prune else (2 if sp_weights is not None and combiner != "sum" else 1)
    sp, spw, empty, _ = sparse_prune_fill(sp_ids, sp_weights, default_id, mode)
    return sp, spw, empty


def safe_embedding_lookup_sparse(embedding_weights, sparse_ids, sparse_weights=None,
                                 combiner="mean", default_id=None, name=None,
                                 partition_strategy="div", max_norm=None, prune=True):
    if embedding_weights is None:
        raise ValueError("Missing embedding_weights %s." % embedding_weights)
    sp, spw, empty = _prune_and_fill(sparse_ids, sparse_weights, combiner, default_id, prune)
    res = embedding_lookup_sparse(embedding_weights, sp, spw, partition_strategy=partition_strategy,
                                  combiner=combiner, max_norm=max_norm)
    if default_id is None:
        res = torch.where(empty[:, None], torch.zeros_like(res), res)
    return res


# ---------------------------------------------------------------------------
# fused_embedding_lookup_sparse (python/ops/fused_embedding_ops.py:18-72),
# local variant: FusedEmbeddingLocalSparseLookUp semantics (sequential sum,
# then combiner; max_norm per row).
# ---------------------------------------------------------------------------
class _FusedLocalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, sp_values, sp_indices, batch, combiner, max_norm):
        out, vo = ops.fused_embedding_local_sparse_look_up(sp_values, sp_indices, (batch, 0),
                                                           table, combiner, max_norm)
        ctx.save_for_backward(table, sp_values, vo)
        ctx.combiner, ctx.max_norm = combiner, max_norm
        return out

    @staticmethod
    def backward(ctx, g):
        table, sp_values, vo = ctx.saved_tensors
        grad_vals = ops.fused_embedding_local_sparse_look_up_grad(
            g.contiguous(), table, sp_values, vo, ctx.combiner, ctx.max_norm)
        dense = torch.zeros_like(table)
        dense.index_add_(0, sp_values.to(torch.int64), grad_vals)
        return dense, None, None, None, None, None


class _FusedPartitionedFn(torch.autograd.Function):
    """fused_embedding_lookup_sparse (python/ops/fused_embedding_ops.py:45-67):
    PreLookUp -> one Gather per partition -> PostLookUp; backward
    PostLookUpGrad (:88-98) -> the Gather grads, IndexedSlices(grad_shard,
    partitioned_values[i]) per partition."""

    @staticmethod
    def forward(ctx, anchor, parts, sp_values, sp_indices, dense_shape, combiner, max_norm,
                *tensors):
        tabs = [p.weight if isinstance(p, DenseTable) else p.detach() for p in parts]
        pv, pi = ops.fused_embedding_sparse_pre_look_up([t.shape for t in tabs], sp_values,
                                                        sp_indices)
        shards = [ops.gather(t, v) for t, v in zip(tabs, pv)]
        out, fnum = ops.fused_embedding_sparse_post_look_up(shards, pi, dense_shape, pv, combiner,
                                                            max_norm)
        ctx.parts, ctx.pv, ctx.pi, ctx.shards, ctx.fnum = parts, pv, pi, shards, fnum
        ctx.combiner, ctx.max_norm, ctx.tensors = combiner, max_norm, tensors
        return out

    @staticmethod
    def backward(ctx, g):
        grads = ops.fused_embedding_sparse_post_look_up_grad(
            g.contiguous(), ctx.shards, ctx.pi, ctx.fnum, ctx.combiner, ctx.max_norm)
        dense = [None] * len(ctx.tensors)
        for prm, gs, v in zip(ctx.parts, grads, ctx.pv):
            sl = IndexedSlices(gs, v)
            if isinstance(prm, DenseTable):
                prm.pending_grads.append(sl)
                continue
            for j, t in enumerate(ctx.tensors):
                if t is prm:
                    d = _dense_grad(t, sl)
                    dense[j] = d if dense[j] is None else dense[j] + d
        return (None,) * 7 + tuple(dense)


def fused_embedding_lookup_sparse(embedding_weights, sparse_ids, combiner=None, name=None,
                                  max_norm=None):
    """python/ops/fused_embedding_ops.py:18-67 over one table or a list of
    partitions ("div" by partition_shapes[i][0]), dense tables (DenseTable
    or torch tensors) as in the reference."""
    if embedding_weights is None:
        raise ValueError("Missing embedding_weights %s." % embedding_weights)
    parts = list(embedding_weights) if isinstance(embedding_weights, (list, tuple)) \
        else [embedding_weights]
    if not parts:
        raise ValueError("Missing embedding_weights %s." % embedding_weights)
    if combiner is None:
        combiner = "mean"
    if combiner not in ("mean", "sqrtn", "sum"):
        raise ValueError("combiner must be one of 'mean', 'sqrtn' or 'sum'")
    if not isinstance(sparse_ids, SparseTensor):
        raise TypeError("sparse_ids must be SparseTensor")
    for p in parts:
        if isinstance(p, EmbeddingVariable):
            raise TypeError("fused_embedding_lookup_sparse takes dense tables (the reference's "
                            "fused ops do not support EmbeddingVariables)")
    tensors = [p for p in parts if torch.is_tensor(p) and p.requires_grad] \
        if torch.is_grad_enabled() else []
    anchors = [_anchor(p) for p in parts if isinstance(p, DenseTable)] \
        if torch.is_grad_enabled() else []
    vals = sparse_ids.values.to(torch.int64).contiguous()
    ind = sparse_ids.indices.to(torch.int64).contiguous()
    args = (parts, vals, ind, sparse_ids.dense_shape, combiner, max_norm)
    if anchors or tensors:
        return _FusedPartitionedFn.apply(anchors[0] if anchors else None, *args, *tensors)
    with torch.no_grad():
        return _FusedPartitionedFn.forward(_Ctx(), None, *args)
