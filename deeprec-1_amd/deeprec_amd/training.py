"""Sparse optimizers for EmbeddingVariables (DeepRec's EV dispatch in
python/training/{gradient_descent,adagrad,adam}.py -> KvResourceSparseApply*
kernels in core/kernels/training_ali_ops.cc), running the HIP apply kernels.

Gradients arrive as IndexedSlices queued on each variable by the lookup's
backward.  Several slices for one variable are deduplicated first with
unique + unsorted_segment_sum, as _deduplicate_indexed_slices does
(python/training/optimizer.py:68-83).
"""
import torch

from . import ops
from ._lib import check, lib, ptr, stream_handle
from .embedding_ops import DenseTable
from .kv_variable_ops import EmbeddingVariable, IndexedSlices


def _dedup(slices):
    if len(slices) == 1:
        return slices[0]           # one lookup's slices are already unique ids
    vals, idxs = [], []
    for s in slices:
        n = s.indices.numel() if s.num_valid is None else int(s.num_valid.item())
        vals.append(s.values[:n])
        idxs.append(s.indices[:n])
    v = torch.cat(vals)
    i = torch.cat(idxs)
    u, pos = ops.unique(i)
    summed = ops.unsorted_segment_sum(v, pos, u.numel())
    return IndexedSlices(summed, u)


class _Optimizer(object):
    def __init__(self, learning_rate):
        self.lr = float(learning_rate)

    def apply_gradients(self, var_list, global_step=None):
        gs = -1 if global_step is None else int(global_step)
        for var in var_list:
            if not var.pending_grads:
                continue
            sl = _dedup(var.pending_grads)
            var.pending_grads = []
            if isinstance(var, EmbeddingVariable):
                self._apply_ev(var, sl, gs)
            elif isinstance(var, DenseTable):
                self._apply_dense(var, sl)
            else:
                raise TypeError("unsupported variable %r" % (var,))
        self._finish()

    def _finish(self):
        pass

    def _apply_dense(self, var, sl):
        n = sl.indices.numel() if sl.num_valid is None else int(sl.num_valid.item())
        self._dense_update(var, sl.indices[:n], sl.values[:n])


class GradientDescentOptimizer(_Optimizer):
    """KvResourceSparseApplyGradientDescent (training_ali_ops.cc:1597-1678)."""

    def _apply_ev(self, var, sl, gs):
        dev = var.device
        check(lib().dr_ev_apply_sgd(var.handle, self.lr, ptr(sl.values.contiguous()),
                                    ptr(sl.indices.contiguous()), sl.indices.numel(),
                                    ptr(sl.num_valid), gs, stream_handle(dev)))
        ops._post(dev)

    def _dense_update(self, var, idx, g):
        var.weight.index_add_(0, idx, g * (-self.lr))


class AdagradOptimizer(_Optimizer):
    """KvSparseApplyAdagrad (training_ali_ops.cc:61-145)."""

    def __init__(self, learning_rate, initial_accumulator_value=0.1):
        super().__init__(learning_rate)
        self.init_acc = float(initial_accumulator_value)
        self._dense_acc = {}

    def _apply_ev(self, var, sl, gs):
        acc = var.slot("Adagrad", self.init_acc)
        dev = var.device
        check(lib().dr_ev_apply_adagrad(var.handle, acc.handle, self.lr,
                                        ptr(sl.values.contiguous()), ptr(sl.indices.contiguous()),
                                        sl.indices.numel(), ptr(sl.num_valid), gs,
                                        stream_handle(dev)))
        ops._post(dev)

    def _dense_update(self, var, idx, g):
        acc = self._dense_acc.setdefault(id(var), torch.full_like(var.weight, self.init_acc))
        a = acc[idx] + g * g
        acc[idx] = a
        var.weight[idx] = var.weight[idx] - (g * self.lr) * torch.rsqrt(a)


class AdamOptimizer(_Optimizer):
    """KvSparseApplyAdam (training_ali_ops.cc:848-975); beta powers advance
    once per apply_gradients like the optimizer's non-slot variables."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8):
        super().__init__(learning_rate)
        self.beta1, self.beta2, self.eps = float(beta1), float(beta2), float(epsilon)
        self.b1p = torch.tensor(self.beta1, dtype=torch.float32).item()
        self.b2p = torch.tensor(self.beta2, dtype=torch.float32).item()

    def _apply_ev(self, var, sl, gs):
        m = var.slot("Adam", 0.0)
        v = var.slot("Adam_1", 0.0)
        dev = var.device
        check(lib().dr_ev_apply_adam(var.handle, m.handle, v.handle, self.b1p, self.b2p, self.lr,
                                     self.beta1, self.beta2, self.eps,
                                     ptr(sl.values.contiguous()), ptr(sl.indices.contiguous()),
                                     sl.indices.numel(), ptr(sl.num_valid), gs,
                                     stream_handle(dev)))
        ops._post(dev)

    def _finish(self):
        f32 = lambda x: torch.tensor(x, dtype=torch.float32)
        self.b1p = (f32(self.b1p) * f32(self.beta1)).item()
        self.b2p = (f32(self.b2p) * f32(self.beta2)).item()

    def _dense_update(self, var, idx, g):
        raise NotImplementedError("dense-table Adam: use an EmbeddingVariable")
