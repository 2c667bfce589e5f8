"""Model glue around the hot path: the DLRM and DeepFM
training steps of DeepRec's modelzoo, built from this engine's ops.

Only the embedding side and the interactions are this engine's kernels
(EV lookup + pooled backward + KV optimizer, dot interaction fwd/bwd, FM
second order fwd/bwd); the MLPs are plain library GEMMs (torch.nn.Linear ->
hipBLASLt), as the north_star asks.

* DLRM: modelzoo/DLRM/train.py:105-290 -- bottom MLP over the 13 dense
  features (ReLU after every layer), `dot_op` over [bottom, e_1..e_26]
  (strictly-lower triangle of X X^T, :150-163), concat with the bottom
  output, top MLP (ReLU), a last 1-unit layer, sigmoid, binary
  cross-entropy, GradientDescent.
* DeepFM: modelzoo/DeepFM/train.py:150-225 -- linear part = sum of the wide
  (dim-1) embeddings, FM second order over the field embeddings (:205-209),
  DNN over the concatenated embeddings, final DNN over [dnn, linear, fm],
  a last 1-unit layer, sigmoid.

Inputs are one-hot ids ([T, B] int64, Criteo hotness 1) and dense features
[B, 13] fp32.
"""
import torch

from . import ops
from .embedding_ops import SparseTensor, embedding_lookup_sparse_multi, embedding_stack


class DotInteraction(torch.autograd.Function):
    """dr_dot_interaction / dr_dot_interaction_grad."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return ops.dot_interaction(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return ops.dot_interaction_grad(x, g)


class FMSecondOrder(torch.autograd.Function):
    """dr_fm2 / dr_fm2_grad."""

    @staticmethod
    def forward(ctx, emb):
        ctx.save_for_backward(emb)
        return ops.fm_second_order(emb)

    @staticmethod
    def backward(ctx, g):
        (emb,) = ctx.saved_tensors
        return ops.fm_second_order_grad(emb, g)


def _mlp(sizes, last_act=True):
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(torch.nn.Linear(sizes[i], sizes[i + 1]))
        if last_act or i < len(sizes) - 2:
            layers.append(torch.nn.ReLU())
    return torch.nn.Sequential(*layers)


class _OneHotLookup(object):
    """T one-hot features -> [B, T*D] through embedding_lookup_sparse_multi
    (grouped Unique -> EV resolve -> fused pooling; grads queued on the EVs),
    or stacked behind a dense row into [B, 1+T, D] (stack())."""

    def __init__(self, evs):
        self.evs = evs
        self._ind = {}

    def _sps(self, ids):
        T, B = ids.shape
        key = (B, ids.device)
        if key not in self._ind:
            r = torch.arange(B, device=ids.device)
            self._ind[key] = torch.stack([r, torch.zeros_like(r)], 1)
        ind = self._ind[key]
        return [SparseTensor(ind, ids[t], (B, 1)) for t in range(T)]

    def __call__(self, ids):
        return embedding_lookup_sparse_multi(self.evs, self._sps(ids), combiner="sum")

    def stack(self, x0, ids):
        return embedding_stack(x0, self.evs, self._sps(ids), combiner="sum")


class _MaybeBF16(object):
    """The reference's bf16 switch: MLPs run in bf16 on fp32 master weights
    (variable_scope(...).keep_weights(), DLRM train.py:183-195), outputs
    cast back to fp32."""

    def __init__(self, on):
        self.on = on

    def __call__(self, mlp, x):
        if not self.on:
            return mlp(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return mlp(x).float()


class DLRM(torch.nn.Module):
    """modelzoo/DLRM/train.py DLRM with interaction_op='dot'."""

    def __init__(self, evs, num_dense=13, mlp_bot=(512, 256), mlp_top=(512, 256), bf16=False):
        super().__init__()
        self.bf16 = _MaybeBF16(bf16)
        self.evs = list(evs)
        self.dim = self.evs[0].dim
        self.T = len(self.evs)
        # the bottom MLP ends at the embedding dim so it stacks with the
        # embeddings (the reference: mlp_bot [512, 256, 64, 16] with dim 16)
        self.bottom = _mlp([num_dense] + list(mlp_bot) + [self.dim])
        F = self.T + 1
        self.top = _mlp([self.dim + F * (F - 1) // 2] + list(mlp_top))
        self.last = torch.nn.Linear(mlp_top[-1], 1)
        self.lookup = _OneHotLookup(self.evs)

    def forward(self, dense, ids):
        x0 = self.bf16(self.bottom, dense)
        X = self.lookup.stack(x0, ids)                             # [B, 1+T, D], no concat copy
        z = DotInteraction.apply(X)
        net = self.bf16(self.top, torch.cat([x0, z], 1))
        return torch.sigmoid(self.bf16(self.last, net)).squeeze(1)


class DeepFM(torch.nn.Module):
    """modelzoo/DeepFM/train.py DeepFM (no batch norm)."""

    def __init__(self, evs, wide_evs, dnn=(256, 128, 64), final=(128, 64)):
        super().__init__()
        self.evs = list(evs)
        self.wide_evs = list(wide_evs)
        self.dim = self.evs[0].dim
        self.T = len(self.evs)
        self.dnn = _mlp([self.T * self.dim] + list(dnn))
        self.final = _mlp([dnn[-1] + 1 + self.dim] + list(final))
        self.last = torch.nn.Linear(final[-1], 1)
        self.lookup = _OneHotLookup(self.evs)
        self.wide_lookup = _OneHotLookup(self.wide_evs)

    def forward(self, dense, ids):
        B = ids.shape[1]
        emb = self.lookup(ids)                                     # [B, T*D]
        wide = self.wide_lookup(ids)                               # [B, T]
        linear = wide.sum(1, keepdim=True)
        fm = FMSecondOrder.apply(emb.view(B, self.T, self.dim))
        net = self.final(torch.cat([self.dnn(emb), linear, fm], 1))
        return torch.sigmoid(self.last(net)).squeeze(1)


def train_step(model, dense, ids, labels, dense_opt, ev_opt, global_step=None):
    """One step: forward, BCE loss (tf.keras BinaryCrossentropy on the
    sigmoid output), backward, dense optimizer, KV optimizer on every EV."""
    pred = model(dense, ids)
    eps = 1e-7                                   # keras backend epsilon clip
    p = pred.clamp(eps, 1 - eps)
    loss = -(labels * torch.log(p) + (1 - labels) * torch.log(1 - p)).mean()
    dense_opt.zero_grad(set_to_none=True)
    loss.backward()
    dense_opt.step()
    evs = list(model.evs) + list(getattr(model, "wide_evs", []))
    ev_opt.apply_gradients(evs, global_step=global_step)
    return loss
