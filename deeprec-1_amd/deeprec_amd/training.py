"""Sparse optimizers for EmbeddingVariables (DeepRec's EV dispatch in
python/training/{gradient_descent,adagrad,adam}.py -> KvResourceSparseApply*
kernels in core/kernels/training_ali_ops.cc), running the HIP apply kernels.

Gradients arrive as IndexedSlices queued on each variable by the lookup's
backward.  Several slices for one variable are deduplicated first with
unique + unsorted_segment_sum, as _deduplicate_indexed_slices does
(python/training/optimizer.py:68-83).
"""
import os

import torch

from . import ops
from ._lib import check, lib, ptr, stream_handle
from .embedding_ops import DenseTable
from .kv_variable_ops import (EmbeddingVariable, IndexedSlices, PendingRowSlices,
                              _flush_deferred_releases)


def _concat(slices):
    vals, idxs = [], []
    for s in slices:
        n = s.indices.numel() if s.num_valid is None else int(s.num_valid.item())
        vals.append(s.values[:n])
        idxs.append(s.indices[:n])
    return torch.cat(vals), torch.cat(idxs)


def _dedup(slices):
    """_deduplicate_indexed_slices (optimizer.py:68-83): unique + sum."""
    if len(slices) == 1 and slices[0].unique:
        return slices[0]           # one lookup's backward: ids already distinct
    v, i = _concat(slices)
    u, pos = ops.unique(i)
    summed = ops.unsorted_segment_sum(v, pos, u.numel())
    return IndexedSlices(summed, u, unique=True)


def _rounds(slices):
    """Split possibly repeated indices into rounds of distinct ids, round r
    holding every id's r-th occurrence (in index order).  Applying the rounds
    in order replays a kernel that walks the indices sequentially."""
    if len(slices) == 1 and slices[0].unique:
        return slices
    v, i = _concat(slices)
    if i.numel() == 0:
        return []
    _, pos = ops.unique(i)
    pos = pos.to(torch.int64)
    order = torch.sort(pos, stable=True).indices
    sp = pos[order]
    start = torch.ones_like(sp, dtype=torch.bool)
    start[1:] = sp[1:] != sp[:-1]
    first = torch.cummax(torch.where(start, torch.arange(sp.numel(), device=sp.device),
                                     torch.zeros_like(sp)), 0).values
    rank = torch.empty_like(sp)
    rank[order] = torch.arange(sp.numel(), device=sp.device) - first
    out = []
    for r in range(int(rank.max().item()) + 1):
        m = rank == r
        out.append(IndexedSlices(v[m], i[m], unique=True))
    return out


# SGD applies of row-grouped backwards use the forward's rows (A/B switch)
_KNOWN_ROWS = os.environ.get("DR_APPLY_PROBE") != "1"

# KV Adam with its beta powers in HBM (A/B switch DR_KV_ADAM_DEVICE_POWERS=0)
_ADAM_DEVICE_POWERS = os.environ.get("DR_KV_ADAM_DEVICE_POWERS", "1") != "0"


def _grad_rows(grp, fn_name):
    """The gradient argument of a grouped EV apply: by address when every
    slice came from a row-grouped lookup backward (no [U, D] gradient copy:
    the kernel reads the pooled gradient in place), else the value blocks."""
    if all(sl.grad_ptr is not None and sl._values is None for _, sl in grp):
        return [sl.grad_ptr for _, sl in grp], getattr(lib(), fn_name + "_ptr")
    return [sl.values.contiguous() for _, sl in grp], getattr(lib(), fn_name)


class _Locked(object):
    """use_locking=True (optimizer.py Optimizer(use_locking)): the EV applies
    take each variable's exclusive update lock, as the reference's
    MaybeLockEmbeddingVariableInputMutexesInOrder does (training_ali_ops.cc:
    104).  dr_ev_lock_updates serialises host threads on the variables'
    mutexes (in address order, like the reference) and orders this stream
    after the last locked apply issued on any other stream."""

    def __init__(self, enabled, handles, stream):
        import ctypes as C
        self.enabled, self.stream = enabled, stream
        self.arr = (C.c_void_p * len(handles))(*handles)
        self.n = len(handles)

    def __enter__(self):
        if self.enabled:
            check(lib().dr_ev_lock_updates(self.arr, self.n, self.stream))

    def __exit__(self, *exc):
        if self.enabled:
            check(lib().dr_ev_unlock_updates(self.arr, self.n, self.stream))
        return False


class _Optimizer(object):
    _opt = None   # DR_OPT_* code of the EV apply kernel

    def __init__(self, learning_rate, use_locking=False):
        self.lr = float(learning_rate)
        self.use_locking = bool(use_locking)

    # How repeated indices reach the EV apply kernel: summed first (the
    # default _resource_apply_sparse_duplicate_indices, optimizer.py:1060-1083)
    # or applied one after another (GradientDescent overrides it and hands
    # the raw indices to KvResourceSparseApplyGradientDescent,
    # gradient_descent.py:71-76, whose kernel walks them in order).
    _ev_duplicates = "sum"

    def apply_gradients(self, var_list, global_step=None):
        gs = -1 if global_step is None else int(global_step)
        if self._opt == 0 and _KNOWN_ROWS:
            self._apply_fused_rows(var_list, gs)
        rounds = []   # rounds[r] = [(var, slices)] applied in one grouped launch
        for var in var_list:
            if not var.pending_grads:
                continue
            pending = var.pending_grads
            var.pending_grads = []
            if isinstance(var, EmbeddingVariable):
                sls = (_rounds(pending) if self._ev_duplicates == "sequential"
                       else [_dedup(pending)])
                for r, sl in enumerate(sls):
                    if r == len(rounds):
                        rounds.append([])
                    rounds[r].append((var, sl))
            elif isinstance(var, DenseTable):
                self._apply_dense(var, _dedup(pending))
            else:
                raise TypeError("unsupported variable %r" % (var,))
        for items in rounds:
            self._apply_ev_batch(items, gs)
        self._finish()
        _flush_deferred_releases()   # EVs collected meanwhile (no-op while capturing)

    def _apply_fused_rows(self, var_list, gs):
        """SGD over every EV of a row-grouped lookup backward whose gradient
        is still pending (PendingRowSlices, nothing else read it): one fused
        backward + update (dr_ev_pool_grad_rows_apply_sgd), the same values as
        forming the IndexedSlices and applying them.  A group only partly in
        var_list, or an EV with more than that one pending gradient, takes the
        ordinary path."""
        groups = {}
        for var in var_list:
            pg = var.pending_grads
            if (isinstance(var, EmbeddingVariable) and len(pg) == 1
                    and isinstance(pg[0], PendingRowSlices) and pg[0].fusable()):
                groups.setdefault(id(pg[0]._pending), (pg[0]._pending, []))[1].append(var)
        for pend, vs in groups.values():
            if len(vs) != len(pend.evs) or {id(v) for v in vs} != {id(e) for e in pend.evs}:
                continue
            st = stream_handle(pend.dev)
            with _Locked(self.use_locking, [e.handle.value for e in pend.evs], st):
                pend.apply_sgd(self.lr, gs, st)
            for v in vs:
                v.pending_grads = []

    def _slots(self, var):
        return None, None

    def _scalars(self):
        return (0.0, 0.0, 0.0, 0.0, 0.0)

    def _apply_ev_batch(self, items, gs):
        """One dr_ev_apply_grouped per (device, dim) group of variables."""
        import ctypes as C
        groups = {}
        for var, sl in items:
            groups.setdefault((str(var.device), var.dim, var.value_dtype), []).append((var, sl))
        b1p, b2p, b1, b2, eps = self._scalars()
        for grp in groups.values():
            T = len(grp)
            dev = grp[0][0].device
            if (self._opt == 0 and _KNOWN_ROWS
                    and all(sl.grad_ptr is not None and sl._values is None and sl.rows is not None
                            and var.filter_freq == 0 for var, sl in grp)):
                # SGD of row-grouped lookup backwards: the forward's rows, no
                # key-table probe (dr_ev_apply_grouped_ptr_rows)
                P = C.c_void_p * T
                st = stream_handle(dev)
                idxs = [sl.indices.contiguous() for _, sl in grp]
                with _Locked(self.use_locking, [var.handle.value for var, _ in grp], st):
                    check(lib().dr_ev_apply_grouped_ptr_rows(
                        self._opt, P(*[var.handle.value for var, _ in grp]), T,
                        P(*[sl.grad_ptr.data_ptr() for _, sl in grp]),
                        P(*[i.data_ptr() for i in idxs]),
                        P(*[sl.rows.data_ptr() for _, sl in grp]),
                        (C.c_int64 * T)(*[i.numel() for i in idxs]),
                        P(*[ptr(sl.num_valid) for _, sl in grp]), self.lr, gs, st))
                ops._post(dev)
                continue
            grads, fn = _grad_rows(grp, "dr_ev_apply_grouped")
            idxs = [sl.indices.contiguous() for _, sl in grp]
            slots = [self._slots(var) for var, _ in grp]
            P = C.c_void_p * T
            s1 = P(*[a.handle.value if a is not None else None for a, _ in slots])
            s2 = P(*[b.handle.value if b is not None else None for _, b in slots])
            st = stream_handle(dev)
            with _Locked(self.use_locking, [var.handle.value for var, _ in grp], st):
                check(fn(
                    self._opt, P(*[var.handle.value for var, _ in grp]), s1, s2, T,
                    P(*[v.data_ptr() for v in grads]), P(*[i.data_ptr() for i in idxs]),
                    (C.c_int64 * T)(*[i.numel() for i in idxs]),
                    P(*[ptr(sl.num_valid) for _, sl in grp]), self.lr, b1p, b2p, b1, b2, eps, gs,
                    st))
            ops._post(dev)

    def _finish(self):
        pass

    def _apply_dense(self, var, sl):
        n = sl.indices.numel() if sl.num_valid is None else int(sl.num_valid.item())
        self._dense_update(var, sl.indices[:n], sl.values[:n])


class GradientDescentOptimizer(_Optimizer):
    """KvResourceSparseApplyGradientDescent (training_ali_ops.cc:1597-1678)."""

    _opt = 0
    _ev_duplicates = "sequential"

    def _dense_update(self, var, idx, g):
        var.weight.index_add_(0, idx, g * (-self.lr))


class AdagradOptimizer(_Optimizer):
    """KvSparseApplyAdagrad (training_ali_ops.cc:61-145)."""

    _opt = 1

    def __init__(self, learning_rate, initial_accumulator_value=0.1, use_locking=False):
        super().__init__(learning_rate, use_locking)
        self.init_acc = float(initial_accumulator_value)
        self._dense_acc = {}

    def _slots(self, var):
        return var.slot("Adagrad", self.init_acc), None

    def _dense_update(self, var, idx, g):
        acc = self._dense_acc.setdefault(id(var), torch.full_like(var.weight, self.init_acc))
        a = acc[idx] + g * g
        acc[idx] = a
        var.weight[idx] = var.weight[idx] - (g * self.lr) * torch.rsqrt(a)


def _capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _not_capturing(what):
    if _capturing():
        raise RuntimeError("%s is not graph-safe: its per-step host scalars would be frozen "
                           "at their capture-time values in every replay" % what)


class AdamOptimizer(_Optimizer):
    """KvSparseApplyAdam (training_ali_ops.cc:848-975); beta powers advance
    once per apply_gradients like the optimizer's non-slot variables."""

    _opt = 2

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 use_locking=False):
        super().__init__(learning_rate, use_locking)
        self.beta1, self.beta2, self.eps = float(beta1), float(beta2), float(epsilon)
        self._dense_mv = {}
        self.b1p = torch.tensor(self.beta1, dtype=torch.float32).item()
        self.b2p = torch.tensor(self.beta2, dtype=torch.float32).item()
        self._pw = {}   # device -> (float[2] beta powers in HBM, float[2] betas)

    def _slots(self, var):
        return var.slot("Adam", 0.0), var.slot("Adam_1", 0.0)

    def _scalars(self):
        return (self.b1p, self.b2p, self.beta1, self.beta2, self.eps)

    def prepare(self, device):
        """Create the device beta powers for `device` now (eagerly): a graph
        that captures the first EV apply then finds them in place."""
        self._device_powers(torch.device(device))

    def sync_host_powers(self):
        """The device powers are the source of truth once steps replay from a
        hipGraph (a replay advances only them): copy them back into the host
        b1p / b2p (one device sync; not under capture)."""
        if not self._pw:
            return
        _not_capturing("AdamOptimizer.sync_host_powers")
        b1p, b2p = next(iter(self._pw.values()))[0].tolist()
        self.b1p, self.b2p = b1p, b2p

    def _device_powers(self, dev):
        """The beta powers as a device float[2] (created from the host values
        on first use, or by prepare() -- never under a graph capture), advanced
        in _finish by an fp32 multiply on the device: the same roundings as the
        host values, and no per-step host scalar in the EV apply (capturable).
        Under replays only these advance; sync_host_powers() brings the host
        copies (used by dense tables and the DR_KV_ADAM_DEVICE_POWERS=0 A/B
        path, neither graph-safe) up to date."""
        key = str(dev)
        if key not in self._pw:
            if _capturing():
                raise RuntimeError("AdamOptimizer: the device beta powers are created on the "
                                   "first EV apply, which is under a graph capture here; run one "
                                   "eager step or call prepare(device) before capturing")
            self._pw[key] = (torch.tensor([self.b1p, self.b2p], dtype=torch.float32, device=dev),
                             torch.tensor([self.beta1, self.beta2], dtype=torch.float32,
                                          device=dev))
        return self._pw[key][0]

    def _apply_ev_batch(self, items, gs):
        """dr_ev_apply_adam_grouped_dev per (device, dim, dtype) group: alpha
        formed in the kernel from the HBM beta powers (A/B switch
        DR_KV_ADAM_DEVICE_POWERS=0: host powers, dr_ev_apply_grouped)."""
        if not _ADAM_DEVICE_POWERS:
            _not_capturing("AdamOptimizer with DR_KV_ADAM_DEVICE_POWERS=0 (host beta powers)")
            return _Optimizer._apply_ev_batch(self, items, gs)
        import ctypes as C
        groups = {}
        for var, sl in items:
            groups.setdefault((str(var.device), var.dim, var.value_dtype), []).append((var, sl))
        for grp in groups.values():
            T = len(grp)
            dev = grp[0][0].device
            by_addr = all(sl.grad_ptr is not None and sl._values is None for _, sl in grp)
            grads = [sl.grad_ptr if by_addr else sl.values.contiguous() for _, sl in grp]
            idxs = [sl.indices.contiguous() for _, sl in grp]
            slots = [self._slots(var) for var, _ in grp]
            pw = self._device_powers(dev)
            P = C.c_void_p * T
            st = stream_handle(dev)
            with _Locked(self.use_locking, [var.handle.value for var, _ in grp], st):
                check(lib().dr_ev_apply_adam_grouped_dev(
                    int(by_addr), P(*[var.handle.value for var, _ in grp]),
                    P(*[a.handle.value for a, _ in slots]), P(*[b.handle.value for _, b in slots]),
                    T, P(*[g.data_ptr() for g in grads]), P(*[i.data_ptr() for i in idxs]),
                    (C.c_int64 * T)(*[i.numel() for i in idxs]),
                    P(*[ptr(sl.num_valid) for _, sl in grp]), pw.data_ptr(), self.lr, self.beta1,
                    self.beta2, self.eps, gs, st))
            ops._post(dev)

    def _finish(self):
        f32 = lambda x: torch.tensor(x, dtype=torch.float32)
        self.b1p = (f32(self.b1p) * f32(self.beta1)).item()
        self.b2p = (f32(self.b2p) * f32(self.beta2)).item()
        for pw, betas in self._pw.values():   # the device copies, on their streams
            pw.mul_(betas)

    def _dense_update(self, var, idx, g):
        """_apply_sparse_shared (adam.py:183-207) on a dense table: m and v
        decay on every row, the deduplicated gradient is scatter-added, and
        every row of var moves by lr_t * m / (sqrt(v) + eps) (TF's non-lazy
        sparse Adam), lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)."""
        _not_capturing("AdamOptimizer on a dense table (lr_t from host beta powers)")
        w = var.weight
        m, v = self._dense_mv.setdefault(id(var), (torch.zeros_like(w), torch.zeros_like(w)))
        f32 = lambda x: torch.tensor(x, dtype=torch.float32)
        lr = (f32(self.lr) * torch.sqrt(1 - f32(self.b2p)) / (1 - f32(self.b1p))).item()
        # (1 - beta) in fp32, as adam.py's tensors compute it (1.0f - 0.9f =
        # 0.100000024f, not the double 0.1 rounded)
        c1 = (f32(1.0) - f32(self.beta1)).item()
        c2 = (f32(1.0) - f32(self.beta2)).item()
        with torch.no_grad():
            m.mul_(self.beta1).index_add_(0, idx, g * c1)
            v.mul_(self.beta2).index_add_(0, idx, (g * g) * c2)
            w.sub_(lr * m / (torch.sqrt(v) + self.eps))


class FtrlOptimizer(_Optimizer):
    """KvResourceSparseApplyFtrl[V2] (training_ali_ops.cc:167-331) on EVs:
    slots accum (initial_accumulator_value) and linear (0); l2_shrinkage > 0
    selects FtrlV2.  Dense tables use the elementwise ResourceSparseApplyFtrl
    of training_ops.cc (per-element |linear| instead of the KV op's row norm)."""

    _opt = 3

    def __init__(self, learning_rate, learning_rate_power=-0.5, initial_accumulator_value=0.1,
                 l1_regularization_strength=0.0, l2_regularization_strength=0.0,
                 l2_shrinkage_regularization_strength=0.0, use_locking=False):
        super().__init__(learning_rate, use_locking)
        self.lr_power = float(learning_rate_power)
        self.init_acc = float(initial_accumulator_value)
        self.l1 = float(l1_regularization_strength)
        self.l2 = float(l2_regularization_strength)
        self.l2_shrinkage = float(l2_shrinkage_regularization_strength)
        self._dense = {}

    def _slots(self, var):
        return var.slot("Ftrl", self.init_acc), var.slot("Ftrl_1", 0.0)

    def _apply_ev_batch(self, items, gs):
        import ctypes as C
        groups = {}
        for var, sl in items:
            groups.setdefault((str(var.device), var.dim, var.value_dtype), []).append((var, sl))
        for grp in groups.values():
            T = len(grp)
            dev = grp[0][0].device
            grads, fn = _grad_rows(grp, "dr_ev_apply_ftrl_grouped")
            idxs = [sl.indices.contiguous() for _, sl in grp]
            slots = [self._slots(var) for var, _ in grp]
            P = C.c_void_p * T
            st = stream_handle(dev)
            with _Locked(self.use_locking, [var.handle.value for var, _ in grp], st):
                check(fn(
                    P(*[var.handle.value for var, _ in grp]),
                    P(*[a.handle.value for a, _ in slots]), P(*[b.handle.value for _, b in slots]),
                    T, P(*[v.data_ptr() for v in grads]), P(*[i.data_ptr() for i in idxs]),
                    (C.c_int64 * T)(*[i.numel() for i in idxs]),
                    P(*[ptr(sl.num_valid) for _, sl in grp]), self.lr, self.l1, self.l2,
                    self.lr_power, self.l2_shrinkage, gs, st))
            ops._post(dev)

    def dense_step(self, params):
        """Elementwise FTRL (ApplyFtrl, training_ops.cc) on dense torch
        parameters with .grad set (a WDL linear part's numeric weights / bias)."""
        with torch.no_grad():
            for p in params:
                if p.grad is None:
                    continue
                acc, lin = self._dense.setdefault(
                    id(p), (torch.full_like(p, self.init_acc), torch.zeros_like(p)))
                g = p.grad
                gu = g + 2.0 * self.l2_shrinkage * p if self.l2_shrinkage > 0 else g
                na = acc + gu * gu
                pw = -self.lr_power
                lin.add_(gu - (na.pow(pw) - acc.pow(pw)) / self.lr * p)
                quad = na.pow(pw) / self.lr + 2.0 * self.l2
                p.copy_(torch.where(lin.abs() > self.l1,
                                    (torch.sign(lin) * self.l1 - lin) / quad,
                                    torch.zeros_like(p)))
                acc.add_(g * g)

    def _dense_update(self, var, idx, g):
        """ResourceSparseApplyFtrl[V2] (training_ops.cc:2587-2614) on the rows
        idx of a dense table (indices already distinct after _dedup)."""
        w = var.weight
        acc_t, lin_t = self._dense.setdefault(
            id(var), (torch.full_like(w, self.init_acc), torch.zeros_like(w)))
        with torch.no_grad():
            x, acc, lin = w[idx], acc_t[idx], lin_t[idx]
            gs = g + 2.0 * self.l2_shrinkage * x if self.l2_shrinkage > 0 else g
            na = acc + g * g
            if self.lr_power == -0.5:
                pn, po = torch.sqrt(na), torch.sqrt(acc)
            else:
                pn, po = na.pow(-self.lr_power), acc.pow(-self.lr_power)
            lin = lin + (gs - (pn - po) / self.lr * x)
            y = pn / self.lr + 2.0 * self.l2
            w[idx] = (lin.clamp(-self.l1, self.l1) - lin) / y
            lin_t[idx] = lin
            acc_t[idx] = acc + g * g


class AdamAsyncOptimizer(_Optimizer):
    """KvSparseApplyAdamAsync (training_ali_ops.cc:1404-1575) on EVs, the
    optimizer of python/training/adam_async.py.  Slots m, v (zeros); the beta
    powers are per variable (adam_async.py:117-141: beta1 / beta2 initial,
    one pair per EV) and live on the device, as the reference keeps them in
    an EV of their own (:1523-1526): the apply kernel forms alpha from them
    and a follow-up kernel advances them only when the gradient's effective
    row count -- the device num_valid of a fixed-capacity slice -- is > 0
    (`if (N > 0)`, :1482; :1558-1559), so no host read is needed and the step
    can be graph-captured.  The reference multiplies them once per Shard()
    work chunk of its CPU thread pool, so its count depends on the host's
    threading for large N; here they advance once per apply, the single-chunk
    case.  apply_sparse_rmsprop: v = b2 v + (1 - b2) g^2, m = b1 m + lr g /
    sqrt(v + eps), var -= m (:1506-1513); the powers are then not used.
    Dense tables take the same two updates on the indexed rows
    (SparseApplyAdamAsync) with fp32 coefficients (T(1) - beta1 in T)."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 use_locking=False, apply_sparse_rmsprop=False):
        super().__init__(learning_rate, use_locking)
        self.beta1, self.beta2, self.eps = float(beta1), float(beta2), float(epsilon)
        self.apply_sparse_rmsprop = bool(apply_sparse_rmsprop)
        self._opt = 4 if self.apply_sparse_rmsprop else 3
        self._powers = {}     # id(var) -> device float32[2] {beta1_power, beta2_power}
        self._dense_mv = {}

    def _slots(self, var):
        return var.slot("AdamAsync", 0.0), var.slot("AdamAsync_1", 0.0)

    def _power_t(self, var):
        dev = var.weight.device if isinstance(var, DenseTable) else var.device
        p = self._powers.get(id(var))
        if p is None:
            # fill kernels, not a host copy: legal inside a hipGraph capture
            p = torch.empty(2, dtype=torch.float32, device=dev)
            p[0].fill_(self.beta1)
            p[1].fill_(self.beta2)
            self._powers[id(var)] = p
        return p

    def _power(self, var):
        """(beta1_power, beta2_power) as host floats (reads the device)."""
        return self._power_t(var).tolist()

    def _apply_ev_batch(self, items, gs):
        import ctypes as C
        groups = {}
        for var, sl in items:
            groups.setdefault((str(var.device), var.dim, var.value_dtype), []).append((var, sl))
        for grp in groups.values():
            T = len(grp)
            dev = grp[0][0].device
            grads, _ = _grad_rows(grp, "dr_ev_apply_grouped")
            by_addr = all(sl.grad_ptr is not None and sl._values is None for _, sl in grp)
            idxs = [sl.indices.contiguous() for _, sl in grp]
            slots = [self._slots(var) for var, _ in grp]
            pw = [self._power_t(var) for var, _ in grp]
            P = C.c_void_p * T
            st = stream_handle(dev)
            with _Locked(self.use_locking, [var.handle.value for var, _ in grp], st):
                check(lib().dr_ev_apply_adam_async_grouped(
                    1 if self.apply_sparse_rmsprop else 0, 1 if by_addr else 0,
                    P(*[var.handle.value for var, _ in grp]),
                    P(*[a.handle.value for a, _ in slots]), P(*[b.handle.value for _, b in slots]),
                    T, P(*[v.data_ptr() for v in grads]), P(*[i.data_ptr() for i in idxs]),
                    (C.c_int64 * T)(*[i.numel() for i in idxs]),
                    P(*[ptr(sl.num_valid) for _, sl in grp]), P(*[p.data_ptr() for p in pw]),
                    self.lr, self.beta1, self.beta2, self.eps, gs, st))
            ops._post(dev)

    def _dense_update(self, var, idx, g):
        w = var.weight
        m, v = self._dense_mv.setdefault(id(var), (torch.zeros_like(w), torch.zeros_like(w)))
        f32 = lambda x: torch.tensor(x, dtype=torch.float32, device=w.device)
        one, b1, b2 = f32(1.0), f32(self.beta1), f32(self.beta2)
        with torch.no_grad():
            mi, vi = m[idx], v[idx]
            vi = vi * b2 + (g * g) * (one - b2)
            if self.apply_sparse_rmsprop:
                mi = mi * b1 + torch.rsqrt(vi + f32(self.eps)) * f32(self.lr) * g
                w[idx] = w[idx] - mi
            else:
                p = self._power_t(var)
                alpha = f32(self.lr) * torch.sqrt(one - p[1]) / (one - p[0])
                mi = mi * b1 + g * (one - b1)
                w[idx] = w[idx] - (mi * alpha) / (torch.sqrt(vi) + f32(self.eps))
                if idx.numel() > 0:           # the op's `if (N > 0)`
                    p.mul_(torch.stack([b1, b2]))
            m[idx], v[idx] = mi, vi


class AdagradDecayOptimizer(_Optimizer):
    """KvSparseApplyAdagradDecay (training_ali_ops.cc:703-823) on EVs, the
    optimizer of python/training/adagrad_decay.py.  Slots: accumulator
    (initial_accumulator_value, also the decay baseline) and
    accumulator_decay_power (zeros, var-shaped: the count is element 0 of a
    row, adagrad_decay.py:104-124).  The kernels see global_step + 1 (the
    optimizer's _global_step_on_worker, :140), which also stamps versions.
    Dense tables: SparseApplyAdagradDecay (:495-670) with one count per row."""

    def __init__(self, learning_rate, global_step=None, initial_accumulator_value=0.1,
                 accumulator_decay_step=100000, accumulator_decay_rate=0.9, use_locking=False):
        if initial_accumulator_value <= 0.0:
            raise ValueError("initial_accumulator_value must be positive: %s"
                             % initial_accumulator_value)
        if accumulator_decay_step <= 0:
            raise ValueError("accumulator_decay_step must be positive: %s"
                             % accumulator_decay_step)
        if accumulator_decay_rate <= 0.0 or accumulator_decay_rate >= 1.0:
            raise ValueError("accumulator_decay_rate must be in (0.0, 1.0): %s"
                             % accumulator_decay_rate)
        super().__init__(learning_rate, use_locking)
        self.global_step = global_step
        self.init_acc = float(initial_accumulator_value)
        self.decay_step = int(accumulator_decay_step)
        self.decay_rate = float(accumulator_decay_rate)
        self._dense = {}

    def apply_gradients(self, var_list, global_step=None):
        gs = self.global_step if global_step is None else global_step
        if gs is None:
            raise ValueError("AdagradDecayOptimizer needs a global step")
        self._gs = int(gs) + 1
        return _Optimizer.apply_gradients(self, var_list, self._gs)

    def _slots(self, var):
        return var.slot("AdagradDecay", self.init_acc), var.slot("AdagradDecay_1", 0.0)

    def _apply_ev_batch(self, items, gs):
        import ctypes as C
        groups = {}
        for var, sl in items:
            groups.setdefault((str(var.device), var.dim, var.value_dtype), []).append((var, sl))
        for grp in groups.values():
            T = len(grp)
            dev = grp[0][0].device
            grads, _ = _grad_rows(grp, "dr_ev_apply_grouped")
            by_addr = all(sl.grad_ptr is not None and sl._values is None for _, sl in grp)
            idxs = [sl.indices.contiguous() for _, sl in grp]
            slots = [self._slots(var) for var, _ in grp]
            P = C.c_void_p * T
            st = stream_handle(dev)
            with _Locked(self.use_locking, [var.handle.value for var, _ in grp], st):
                check(lib().dr_ev_apply_adagrad_decay_grouped(
                    P(*[var.handle.value for var, _ in grp]),
                    P(*[a.handle.value for a, _ in slots]), P(*[b.handle.value for _, b in slots]),
                    T, P(*[v.data_ptr() for v in grads]), 1 if by_addr else 0,
                    P(*[i.data_ptr() for i in idxs]),
                    (C.c_int64 * T)(*[i.numel() for i in idxs]),
                    P(*[ptr(sl.num_valid) for _, sl in grp]), self.lr, self.decay_step,
                    self.decay_rate, self.init_acc, gs, st))
            ops._post(dev)

    def _dense_update(self, var, idx, g):
        w = var.weight
        acc, pw = self._dense.setdefault(
            id(var), (torch.full_like(w, self.init_acc),
                      torch.zeros(w.shape[0], dtype=torch.int64, device=w.device)))
        with torch.no_grad():
            a = acc[idx]
            dec = (self._gs // self.decay_step) > pw[idx]
            a = torch.where(dec[:, None], torch.clamp_min(a * self.decay_rate, self.init_acc), a)
            pw[idx] = pw[idx] + dec.to(torch.int64)
            a = a + g * g
            acc[idx] = a
            w[idx] = w[idx] - (g * self.lr) * torch.rsqrt(a)
