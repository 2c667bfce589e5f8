"""Model glue around the hot path: the DLRM, DeepFM, DIN
and WDL training steps of DeepRec's modelzoo, and DCN-v2 (BASELINE
configs[4]), built from this engine's ops.

Only the embedding side and the interactions are this engine's kernels
(EV lookup + pooled backward + KV optimizer, dot interaction fwd/bwd, FM
second order fwd/bwd, DIN attention fwd/bwd, the bf16 MFMA cross layer);
the MLPs are plain library GEMMs (torch.nn.Linear -> hipBLASLt), as the
north_star asks.

* DLRM: modelzoo/DLRM/train.py:105-290 -- bottom MLP over the 13 dense
  features (ReLU after every layer), `dot_op` over [bottom, e_1..e_26]
  (strictly-lower triangle of X X^T, :150-163), concat with the bottom
  output, top MLP (ReLU), a last 1-unit layer, sigmoid, binary
  cross-entropy, GradientDescent.
* DeepFM: modelzoo/DeepFM/train.py:150-225 -- linear part = sum of the wide
  (dim-1) embeddings, FM second order over the field embeddings (:205-209),
  DNN over the concatenated embeddings, final DNN over [dnn, linear, fm],
  a last 1-unit layer, sigmoid.
* DIN: modelzoo/DIN/script/model.py:11-150,368-392 (DIN class below).
* WDL: modelzoo/WDL/train.py:182-335 (WDL class below).
* DCN-v2: stacked cross network on the MFMA kernel (DCNv2 class below).

Inputs are one-hot ids ([T, B] int64, Criteo hotness 1) and dense features
[B, 13] fp32.
"""
import os

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


class DotConcatBf16(torch.autograd.Function):
    """DLRM's dot layer, concat and --bf16 cast as one node (train.py:211-226):
    X [B, F, D] with X[:, 0] = the bottom-MLP output -> the zero-padded bf16
    top-MLP input [B, cols] (dr_dot_interaction_concat_bf16[_grad])."""

    @staticmethod
    def forward(ctx, x, cols):
        ctx.save_for_backward(x)
        return ops.dot_interaction_concat_bf16(x, cols)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        if g.stride(1) != 1:
            g = g.contiguous()
        return ops.dot_interaction_concat_grad_bf16(x, g.to(torch.bfloat16)), None


class FMSecondOrderBf16Copy(torch.autograd.Function):
    """DeepFM --bf16 input side as one node: emb [B, F, D] fp32 -> (the FM
    second-order term, fp32, and the bf16 dnn input [B, F*D]); backward: the
    FM gradient plus the dnn input's bf16 gradient in one pass
    (dr_fm2_bf16_copy / dr_fm2_grad_add_bf16)."""

    @staticmethod
    def forward(ctx, emb):
        ctx.save_for_backward(emb)
        return ops.fm_second_order_bf16_copy(emb)

    @staticmethod
    def backward(ctx, g_fm, g_h):
        (emb,) = ctx.saved_tensors
        B, F, D = emb.shape
        if g_fm is None:
            g_fm = torch.zeros((B, D), dtype=torch.float32, device=emb.device)
        if g_h is None:
            return ops.fm_second_order_grad(emb, g_fm)
        if g_h.stride(1) != 1:
            g_h = g_h.contiguous()
        return ops.fm_second_order_grad_add_bf16(emb, g_fm, g_h.to(torch.bfloat16))


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


def _dw_split(tiles, rows, slots=512):
    """Row splits of a weight-gradient GEMM: the smallest s within 3 % of the
    fewest block rounds per unit of rows, ceil(tiles * s / slots) / s (2
    blocks per CU x 256 CUs = 512 resident blocks), s <= 64 and each split
    >= 512 rows.  (The old rule, min(64, 512 // tiles), left a 144-tile
    layer at 3 splits = 432 blocks, one partly filled round.)"""
    smax = max(1, min(64, rows // 512))
    cost = {s: -(-tiles * s // slots) / s for s in range(1, smax + 1)}
    best = min(cost.values())
    return min(s for s, c in cost.items() if c <= 1.03 * best)


# A/B switch: DR_TOWER_TN_DW=0 = transposes + NT GEMM for the weight gradients
_TN_DW = os.environ.get("DR_TOWER_TN_DW", "1") != "0"


class _MfmaTowerFn(torch.autograd.Function):
    """A bf16 ReLU MLP tower as ONE autograd node on the hand MFMA GEMM
    (dr_gemm_nt_bf16[_ex]): layer l computes y_l = act(h_l W_l^T + b_l),
    bf16 operands, fp32 accumulate, bf16 out, h_0 = the zero-padded input
    (Kp % 64 == 0), fp32 master weights (the reference's keep_weights).
    Backward, layer by layer from the top: db_l = sum of g_l (fp32, from the
    per-tile column sums the transpose of g_l writes), dW_l =
    g_l^T h_l (both operands transposed, then a split-K GEMM over the batch:
    its output is only N_l x K_l), and the input gradient g_{l-1} = g_l W_l
    with the layer below's ReLU mask applied in the GEMM's epilogue (aux =
    y_{l-1} = h_l) -- no separate mask / multiply passes."""

    @staticmethod
    def forward(ctx, h0, last_act, head, *params):
        # head: the DLRM output layer (N = 1, dr_mlp_head_*) rides on the
        # tower -- its weight and bias are the last two params, the node
        # returns the [B, 1] logit, and its backward hands the tower the
        # ReLU-masked gradient of the last layer directly
        L = (len(params) - (2 if head else 0)) // 2
        ws, bs = params[:L], params[L:2 * L]
        hs, wbs = [h0], []
        h = h0
        for l in range(L):
            relu = last_act or l < L - 1
            wb = torch.nn.functional.pad(ws[l].detach(), (0, h.shape[1] - ws[l].shape[1]))
            wb = wb.to(torch.bfloat16)
            h = ops.gemm_nt(h, wb, bs[l].detach(), ops.ACT_RELU if relu else ops.ACT_NONE)
            hs.append(h)
            wbs.append(wb)
        ctx.L, ctx.last_act, ctx.head = L, last_act, head
        ctx.ks = [w.shape[1] for w in ws]
        if head:
            # head 1: the bf16 output layer (bf16 w, rounded logit); 2: the
            # fp32 output layer on the widened tower output (fp32 w)
            wh = params[2 * L].detach().reshape(-1)
            wh = wh.to(torch.bfloat16) if head == 1 else wh.float().contiguous()
            z = ops.mlp_head_forward(h, wh, params[2 * L + 1].detach())
            ctx.head_shapes = (params[2 * L].shape, params[2 * L + 1].shape)
            ctx.save_for_backward(*hs, *wbs, wh)
            return z.view(-1, 1)
        ctx.save_for_backward(*hs, *wbs)
        # widened here rather than by the caller, so the gradient arrives in
        # fp32 and the ReLU-mask + bf16 cast is one pass (dr_relu_grad_bf16)
        return h.float()

    @staticmethod
    def backward(ctx, go):
        L = ctx.L
        saved = ctx.saved_tensors
        hs, wbs = saved[:L + 1], saved[L + 1:2 * L + 1]
        head_grads = ()
        if ctx.head:
            # grad_h = bf16(gz w) masked by the last layer's ReLU, dw / db of the head
            g, dwh, dbh = ops.mlp_head_backward(hs[L], saved[2 * L + 1], go)
            head_grads = (dwh.view(ctx.head_shapes[0]), dbh.view(ctx.head_shapes[1]))
        elif (ctx.last_act and go.stride(1) == 1 and go.shape[1] % 8 == 0
              and go.stride(0) % 4 == 0 and go.data_ptr() % 16 == 0):
            g = ops.relu_grad_bf16(go, hs[L])     # cast + ReLU mask in one pass
        else:
            g = go.to(torch.bfloat16)
            if ctx.last_act:
                g = g * (hs[L] > 0)
            g = g.contiguous()
        B = g.shape[0]
        dws, dbs = [None] * L, [None] * L
        for l in reversed(range(L)):
            x = hs[l]
            N, Kp = g.shape[1], x.shape[1]
            tiles = ((N + 127) // 128) * ((Kp + 127) // 128)
            split = _dw_split(tiles, B)
            if _TN_DW and B % 64 == 0:
                # dW = g^T x straight from the row-major operands (transposing
                # LDS reads), db from the same pass's A fragments
                dw, dbs[l] = ops.gemm_tn(g, x, split_k=split, colsum=True)
            else:
                # db from the column partials the g transpose writes
                gt, dbs[l] = ops.transpose_bf16(g, colsum=True)
                dw = ops.gemm_nt(gt, ops.transpose_bf16(x), out_fp32=True,
                                 split_k=split)                      # [N, Kp] fp32
            dws[l] = dw[:, :ctx.ks[l]]
            if l > 0 or ctx.needs_input_grad[0]:
                # gradient of h_l; below the top layer h_l = y_{l-1} = ReLU output
                g = ops.gemm_nt(g, wbs[l].t().contiguous(), mask=x if l > 0 else None)
        return (g if ctx.needs_input_grad[0] else None, None, None, *dws, *dbs, *head_grads)


class _MfmaMLP(torch.nn.Module):
    """The bf16 MLP of the reference's --bf16 switch (fp32 master weights,
    bf16 compute, modelzoo/DLRM/train.py:183-221) on the hand MFMA GEMMs:
    the same Linear / ReLU stack as _mlp(sizes), run as one _MfmaTowerFn;
    the input is zero-padded to a multiple of 64 features.  A tower with an
    output width not a multiple of 64 (the contraction of its input
    gradient), or a batch not a multiple of 512, runs through torch autocast
    instead."""

    def __init__(self, sizes, last_act=True):
        super().__init__()
        self.net = _mlp(sizes, last_act)
        self.sizes = list(sizes)
        self.last_act = last_act

    @property
    def kp(self):
        """The zero-padded input width the MFMA tower takes."""
        return (self.sizes[0] + 63) // 64 * 64

    def mfma_ok(self, batch):
        lins = [m for m in self.net if isinstance(m, torch.nn.Linear)]
        return batch % 512 == 0 and all(l.out_features % 64 == 0 for l in lins)

    def forward(self, x):
        B, K = x.shape
        if not self.mfma_ok(B):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return self.net(x).float()
        h = x.to(torch.bfloat16)
        if self.kp != K:
            h = torch.nn.functional.pad(h, (0, self.kp - K))
        return self.forward_padded(h.contiguous())

    def forward_padded(self, h):
        """The tower on an input already in bf16 and zero-padded to kp columns."""
        lins = [m for m in self.net if isinstance(m, torch.nn.Linear)]
        return _MfmaTowerFn.apply(h, self.last_act, 0, *[l.weight for l in lins],
                                  *[l.bias for l in lins])

    def head_ok(self, head):
        return (self.last_act and isinstance(head, torch.nn.Linear) and head.out_features == 1
                and head.bias is not None and self.sizes[-1] in (64, 128, 256, 512))

    def forward_padded_head(self, h, head, fp32=False):
        """forward_padded followed by the N = 1 Linear `head` in the same
        node: [B, 1] fp32 logit.  fp32=False: the bf16 layer (DLRM's
        dense(units=1) under --bf16, bf16-rounded logit); True: an fp32
        layer on the widened output (DeepFM's final dense).  Needs
        head_ok(head)."""
        lins = [m for m in self.net if isinstance(m, torch.nn.Linear)]
        return _MfmaTowerFn.apply(h, self.last_act, 2 if fp32 else 1,
                                  *[l.weight for l in lins], *[l.bias for l in lins],
                                  head.weight, head.bias)

    def forward_head(self, x, head, fp32=False):
        """forward() (cast + zero pad of an fp32 input) then the head."""
        h = x.to(torch.bfloat16)
        if self.kp != x.shape[1]:
            h = torch.nn.functional.pad(h, (0, self.kp - x.shape[1]))
        return self.forward_padded_head(h.contiguous(), head, fp32)


class _MaybeBF16(object):
    """The reference's bf16 switch: MLPs run in bf16 on fp32 master weights
    (variable_scope(...).keep_weights(), DLRM train.py:183-195), outputs
    cast back to fp32.  _MfmaMLP towers run on the hand MFMA GEMMs; other
    modules under torch autocast."""

    def __init__(self, on):
        self.on = on

    def __call__(self, mlp, x):
        if not self.on:
            return mlp(x)
        if isinstance(mlp, _MfmaMLP):
            return mlp(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return mlp(x).float()


class _ShardedLookupFn(torch.autograd.Function):
    """T one-hot features looked up through a multi-GPU row-sharded engine
    (sharded.ShardedLookup, XgmiShardedLookup or NativeShardedLookup) as one
    autograd node: forward = the engine's exchange + owner serve + pooling
    ([B, T*D] fp32); backward hands the [B, T*D] gradient to the engine,
    which delivers every key's gradient rows to its owner's EV shard as
    IndexedSlices -- the KV optimizer applies them there (SOK DLRM's sparse
    path, modelzoo/SOK/DLRM)."""

    # The engines keep the routing state of ONE gradient-carrying forward
    # (inbox / send order / unique ids) for the backward.  Each such forward
    # bumps the engine's generation; a backward whose forward is no longer
    # the latest (a second forward -- an eval pass, another micro-batch --
    # ran in between) raises instead of routing gradients by the wrong batch.

    @staticmethod
    def forward(ctx, anchor, engine, ids):
        from .sharded import XgmiShardedLookup
        ctx.engine = engine
        gen = getattr(engine, "_dr_fwd_gen", 0) + 1
        engine._dr_fwd_gen = gen
        ctx.gen = gen
        if isinstance(engine, XgmiShardedLookup):   # keeps its inbox for the backward
            out = engine.forward(ids)
        else:
            out = engine.forward(ids, need_grad=True)
        return out

    @staticmethod
    def backward(ctx, g):
        if getattr(ctx.engine, "_dr_fwd_gen", None) != ctx.gen:
            raise RuntimeError(
                "sharded lookup backward: another forward ran on this engine since this "
                "one (its routing state is gone); run backward before the next forward, "
                "or run the other forward under torch.no_grad()")
        ctx.engine.backward(g.float().contiguous())
        return None, None, None


def _sharded_lookup(anchor, engine, ids):
    """The engine's lookup as an autograd node when gradients are recorded;
    under torch.no_grad() (an eval pass) a plain forward that keeps no
    routing state (need_grad off: the engines' cheaper direct path)."""
    if torch.is_grad_enabled():
        return _ShardedLookupFn.apply(anchor, engine, ids)
    # this forward overwrites the engine's exchange buffers too: a pending
    # backward of an earlier forward must refuse
    engine._dr_fwd_gen = getattr(engine, "_dr_fwd_gen", 0) + 1
    from .sharded import XgmiShardedLookup
    if isinstance(engine, XgmiShardedLookup):
        return engine.forward(ids)
    return engine.forward(ids, need_grad=False)


class DLRM(torch.nn.Module):
    """modelzoo/DLRM/train.py DLRM with interaction_op='dot'.  engine: a
    row-sharded multi-GPU lookup over this rank's EV shards (evs = the
    shards; ids = this rank's [T, B_local] batch) -- the data-parallel DLRM
    of modelzoo/SOK/DLRM, trained with train_step_sharded."""

    def __init__(self, evs, num_dense=13, mlp_bot=(512, 256), mlp_top=(512, 256), bf16=False,
                 engine=None, replicated=()):
        super().__init__()
        self.bf16 = _MaybeBF16(bf16)
        self.engine = engine
        self._sh_anchor = None
        self.evs = list(evs)
        # hybrid placement: features in `replicated` hold their whole table on
        # every rank (looked up locally, gradients synchronised by
        # train_step_sharded); the engine covers the others, in feature order
        self.replicated = sorted(replicated)
        self.replicated_evs = [self.evs[t] for t in self.replicated]
        self._rep_lookup = _OneHotLookup(self.replicated_evs) if self.replicated else None
        self.dim = self.evs[0].dim
        self.T = len(self.evs)
        # the bottom MLP ends at the embedding dim so it stacks with the
        # embeddings (the reference: mlp_bot [512, 256, 64, 16] with dim 16)
        # bf16: the towers run on the hand MFMA GEMMs (dr_gemm_nt_bf16)
        mlp = _MfmaMLP if bf16 else _mlp
        self.bottom = mlp([num_dense] + list(mlp_bot) + [self.dim])
        F = self.T + 1
        self.top = mlp([self.dim + F * (F - 1) // 2] + list(mlp_top))
        self.last = torch.nn.Linear(mlp_top[-1], 1)
        self.lookup = _OneHotLookup(self.evs)

    # --bf16 with MFMA towers: dot + concat + cast as one kernel writing the
    # padded bf16 top-MLP input (DotConcatBf16); False (or the A/B switch
    # DR_DLRM_FUSE_DOT_CONCAT=0) = the composed dot -> cat -> cast -> pad
    fuse_dot_concat = os.environ.get("DR_DLRM_FUSE_DOT_CONCAT", "1") != "0"
    # and the output layer riding on the top tower (dr_mlp_head_*; A/B
    # switch DR_DLRM_FUSE_HEAD=0 = autocast Linear)
    fuse_head = os.environ.get("DR_DLRM_FUSE_HEAD", "1") != "0"

    def _stack(self, x0, ids):
        if self.engine is None:
            return self.lookup.stack(x0, ids)                      # [B, 1+T, D], no concat copy
        if self._sh_anchor is None:
            self._sh_anchor = torch.zeros(1, device=x0.device, requires_grad=True)
        B = x0.shape[0]
        if not self.replicated:
            emb = _sharded_lookup(self._sh_anchor, self.engine, ids)
            return torch.cat([x0.float().unsqueeze(1), emb.view(B, self.T, self.dim)], 1)
        rep = self.replicated
        sh = [t for t in range(self.T) if t not in rep]
        key = x0.device
        if getattr(self, "_hyb_idx", (None,))[0] != key:
            mk = lambda v: torch.tensor(v, dtype=torch.int64, device=key)  # noqa: E731
            self._hyb_idx = (key, mk(rep), mk(sh), mk([0]), mk([1 + t for t in rep]),
                             mk([1 + t for t in sh]))
        _, irep, ish, i0, xrep, xsh = self._hyb_idx
        er = self._rep_lookup(ids.index_select(0, irep)).view(B, len(rep), self.dim)
        es = _sharded_lookup(self._sh_anchor, self.engine,
                             ids.index_select(0, ish)).view(B, len(sh), self.dim)
        X = x0.new_empty((B, 1 + self.T, self.dim), dtype=torch.float32)
        X = X.index_copy(1, i0, x0.float().unsqueeze(1))
        X = X.index_copy(1, xrep, er)
        return X.index_copy(1, xsh, es)

    def forward(self, dense, ids):
        x0 = self.bf16(self.bottom, dense)
        X = self._stack(x0, ids)
        if (self.fuse_dot_concat and self.bf16.on and isinstance(self.top, _MfmaMLP)
                and self.top.mfma_ok(X.shape[0]) and X.shape[1] <= 32
                and X.shape[2] in (16, 32, 64, 128)):
            h0 = DotConcatBf16.apply(X, self.top.kp)
            if self.fuse_head and self.top.head_ok(self.last):
                return torch.sigmoid(self.top.forward_padded_head(h0, self.last)).squeeze(1)
            net = self.top.forward_padded(h0)
            return torch.sigmoid(self.bf16(self.last, net)).squeeze(1)
        z = DotInteraction.apply(X)
        net = self.bf16(self.top, torch.cat([x0, z], 1))
        return torch.sigmoid(self.bf16(self.last, net)).squeeze(1)


class DeepFM(torch.nn.Module):
    """modelzoo/DeepFM/train.py DeepFM (no batch norm).  bf16=True is the
    reference's --bf16 (train.py:186-217): the dnn and final_dnn towers in
    bf16 on fp32 master weights (keep_weights) -- here the hand MFMA towers
    -- their output cast back to fp32 before the fp32 output layer; the FM
    and linear parts stay fp32 (their bf16 input cast only rounds values the
    fp32 kernels then read: kept fp32 here)."""

    def __init__(self, evs, wide_evs, dnn=(256, 128, 64), final=(128, 64), bf16=False):
        super().__init__()
        self.bf16 = _MaybeBF16(bf16)
        self.evs = list(evs)
        self.wide_evs = list(wide_evs)
        self.dim = self.evs[0].dim
        self.T = len(self.evs)
        mlp = _MfmaMLP if bf16 else _mlp
        self.dnn = mlp([self.T * self.dim] + list(dnn))
        self.final = mlp([dnn[-1] + 1 + self.dim] + list(final))
        self.last = torch.nn.Linear(final[-1], 1)
        self.lookup = _OneHotLookup(self.evs)
        self.wide_lookup = _OneHotLookup(self.wide_evs)

    def forward(self, dense, ids):
        B = ids.shape[1]
        emb = self.lookup(ids)                                     # [B, T*D]
        wide = self.wide_lookup(ids)                               # [B, T]
        linear = wide.sum(1, keepdim=True)
        if (self.fuse_fm_copy and isinstance(self.dnn, _MfmaMLP) and self.dnn.mfma_ok(B)
                and self.dnn.kp == self.T * self.dim and self.dim % 4 == 0 and self.T <= 32):
            # FM + the dnn input's bf16 cast in one pass (no cast / pad copies,
            # no separate add of the two embedding gradients)
            fm, h0 = FMSecondOrderBf16Copy.apply(emb.view(B, self.T, self.dim))
            dnn_out = self.dnn.forward_padded(h0)
        else:
            fm = FMSecondOrder.apply(emb.view(B, self.T, self.dim))
            dnn_out = self.bf16(self.dnn, emb)
        cat = torch.cat([dnn_out, linear, fm], 1)
        if (self.fuse_head and isinstance(self.final, _MfmaMLP) and self.final.mfma_ok(B)
                and self.final.head_ok(self.last)):
            # the fp32 output layer (train.py:219) riding on the final tower
            return torch.sigmoid(self.final.forward_head(cat, self.last, fp32=True)).squeeze(1)
        net = self.bf16(self.final, cat)
        return torch.sigmoid(self.last(net)).squeeze(1)

    # A/B switch DR_DEEPFM_FUSE_HEAD=0 = torch's fp32 Linear
    fuse_head = os.environ.get("DR_DEEPFM_FUSE_HEAD", "1") != "0"

    # A/B switch DR_DEEPFM_FUSE_FM_COPY=0 = the composed FM + cast + pad path
    fuse_fm_copy = os.environ.get("DR_DEEPFM_FUSE_FM_COPY", "1") != "0"


class DinAttentionInput(torch.autograd.Function):
    """dr_din_attention_input / _grad: [q, f, q - f, q * f]."""

    @staticmethod
    def forward(ctx, query, facts):
        ctx.save_for_backward(query, facts)
        return ops.din_attention_input(query, facts)

    @staticmethod
    def backward(ctx, g):
        query, facts = ctx.saved_tensors
        return ops.din_attention_input_grad(query, facts, g)


class DinAttentionPool(torch.autograd.Function):
    """dr_din_attention_pool / _grad: masked softmax + weighted sum of the
    history, and the plain history sum, from one pass over the facts."""

    @staticmethod
    def forward(ctx, scores, mask, facts):
        att, his_sum, alphas = ops.din_attention_pool(scores, mask, facts)
        ctx.save_for_backward(alphas, mask, facts)
        return att, his_sum

    @staticmethod
    def backward(ctx, g_att, g_sum):
        alphas, mask, facts = ctx.saved_tensors
        if g_att is None:
            g_att = torch.zeros(facts.shape[0], facts.shape[2], device=facts.device)
        gs, gf = ops.din_attention_pool_grad(alphas, mask, facts, g_att, g_sum)
        return gs, None, gf


class DinAttentionFused(torch.autograd.Function):
    """The whole attention of din_attention (utils.py:264-309, mode 'SUM')
    as one node: the fused MLP (dr_din_mlp_forward: din_all never written,
    only the valid positions) -> masked softmax + weighted sum + history sum
    (dr_din_attention_pool); backward: pool grad -> dr_din_mlp_backward (the
    MLP's facts / query gradients and per-position buffers) -> the weight
    gradients as split-K GEMMs."""

    @staticmethod
    def forward(ctx, query, facts, mask, w1, b1, w2, b2, w3, b3):
        scores, buf = ops.din_mlp_forward(query, facts, mask, w1, b1, w2, b2, w3, b3)
        att, his_sum, alphas = ops.din_attention_pool(scores, mask, facts)
        ctx.save_for_backward(query, facts, mask, w1, w3, alphas)
        ctx.buf = buf
        return att, his_sum

    @staticmethod
    def backward(ctx, g_att, g_sum):
        query, facts, mask, w1, w3, alphas = ctx.saved_tensors
        if g_att is None:
            g_att = torch.zeros(facts.shape[0], facts.shape[2], device=facts.device)
        gs, gf = ops.din_attention_pool_grad(alphas, mask, facts, g_att, g_sum)
        gq, dW1, db1, dW2, db2, dw3, db3 = ops.din_mlp_backward(query, facts, w1, w3, ctx.buf,
                                                                 gs, gf)
        ctx.buf = None
        return gq, gf, None, dW1, db1, dW2, db2, dw3, db3


class DinAttentionFusedAll(torch.autograd.Function):
    """DinAttentionFused over the merged item lookup's output allv [B + B T,
    H] (target rows, then the history rows): returns (item_eb, att, his_sum)
    and, in the backward, writes the gradient of allv in one buffer -- the
    history rows by the pool / MLP backward kernels in place, the target rows
    as the attention's query gradient plus item_eb's downstream gradient --
    instead of autograd's zero fill + slice copies + add for two views of
    allv."""

    @staticmethod
    def forward(ctx, allv, mask, w1, b1, w2, b2, w3, b3):
        B, T = mask.shape
        query = allv[:B]
        facts = allv[B:].view(B, T, -1)
        scores, buf = ops.din_mlp_forward(query, facts, mask, w1, b1, w2, b2, w3, b3)
        att, his_sum, alphas = ops.din_attention_pool(scores, mask, facts)
        ctx.save_for_backward(allv, mask, w1, w3, alphas)
        ctx.buf = buf
        return query.clone(), att, his_sum

    @staticmethod
    def backward(ctx, g_item, g_att, g_sum):
        allv, mask, w1, w3, alphas = ctx.saved_tensors
        B, T = mask.shape
        query = allv[:B]
        facts = allv[B:].view(B, T, -1)
        if g_att is None:
            g_att = torch.zeros(B, facts.shape[2], device=facts.device)
        g_all = torch.empty_like(allv)
        gf = g_all[B:].view(B, T, -1)
        gs, _ = ops.din_attention_pool_grad(alphas, mask, facts, g_att, g_sum, out=gf)
        gq, dW1, db1, dW2, db2, dw3, db3 = ops.din_mlp_backward(query, facts, w1, w3, ctx.buf,
                                                                 gs, gf)
        ctx.buf = None
        if g_item is None:
            g_all[:B].copy_(gq)
        else:
            torch.add(gq, g_item, out=g_all[:B])
        return g_all, None, dW1, db1, dW2, db2, dw3, db3


class WDL(torch.nn.Module):
    """modelzoo/WDL/train.py WDL (BASELINE configs[0]) on EVs.

    Deep part (:238-281): tf.feature_column.input_layer over the embedding
    columns (one EV per categorical column, combiner 'mean') and the 13
    min-max normalised numeric columns, in input_layer's order -- columns
    sorted by name ('C10_embedding' < 'C1_embedding' < ... < 'I1' < 'I10'
    ...) -- then dnn [1024, 512, 256] ReLU and a 1-unit logits layer.  Wide
    part (:283-295): linear_model with sparse_combiner 'sum' over the same
    categorical ids (dim-1 EVs), one weight per numeric column, one bias.
    logits = dnn_logits + linear_logits.

    identity: {name: num_buckets} of numeric inputs the reference reads as
    categorical_column_with_identity (IDENTITY_NUM_BUCKETS = {'I10': 10},
    :150-155): an indicator_column ('I10_indicator', num_buckets one-hot
    columns) in the deep input and a [num_buckets, 1] weight table in the
    linear model.  num_min / num_range: the numeric columns' min-max scaler
    (col - min) / range (:141-145, 169-175), applied in fp32 to the
    non-identity columns."""

    def __init__(self, cat_names, deep_evs, wide_evs, num_names, hidden=(1024, 512, 256),
                 bf16=False, identity=None, num_min=None, num_range=None):
        super().__init__()
        self.bf16 = _MaybeBF16(bf16)
        self.cat_names, self.num_names = list(cat_names), list(num_names)
        self.deep_evs, self.wide_evs = list(deep_evs), list(wide_evs)
        self.evs = self.deep_evs + self.wide_evs
        self.identity = dict(identity or {})
        dims = [ev.dim for ev in self.deep_evs]
        plain = [n for n in self.num_names if n not in self.identity]
        self.plain_idx = [self.num_names.index(n) for n in plain]
        # input_layer column order: sort by column name, then lay out
        cols, off = {}, 0
        for name, d in zip(self.cat_names, dims):
            cols[name + "_embedding"] = list(range(off, off + d))
            off += d
        for j, name in enumerate(self.num_names):
            if name in self.identity:
                cols[name + "_indicator"] = list(range(off, off + self.identity[name]))
                off += self.identity[name]
            else:
                cols[name] = [off]
                off += 1
        perm = [c for name in sorted(cols) for c in cols[name]]
        self.register_buffer("perm", torch.tensor(perm, dtype=torch.int64), persistent=False)
        # the same order without a column gather: the embedding columns are
        # whole EV blocks and sort before the numeric ones ('C..' < 'I..'),
        # so looking the EVs up in sorted-name order and permuting only the
        # 13 numeric columns lays the input out as input_layer does
        emb_names = [n + "_embedding" for n in self.cat_names]
        self.ev_order = sorted(range(len(emb_names)), key=lambda i: emb_names[i])
        self.block_order = all(n < m for n in emb_names for m in self.num_names)
        if self.identity and not self.block_order:
            raise ValueError("identity columns need the embedding columns to sort first")
        dn = {n if n not in self.identity else n + "_indicator": j
              for j, n in enumerate(self.num_names)}
        self.dense_layout = [(dn[k], self.identity.get(self.num_names[dn[k]], 0))
                             for k in sorted(dn)]
        self.register_buffer("num_perm", torch.tensor(
            sorted(range(len(self.num_names)), key=lambda j: self.num_names[j]),
            dtype=torch.int64), persistent=False)
        self.register_buffer("ev_perm", torch.tensor(self.ev_order, dtype=torch.int64),
                             persistent=False)
        scale = num_min is not None
        self.register_buffer("num_min", torch.tensor(
            num_min if scale else [0.0] * len(self.num_names), dtype=torch.float32),
            persistent=False)
        self.register_buffer("num_range", torch.tensor(
            num_range if scale else [1.0] * len(self.num_names), dtype=torch.float32),
            persistent=False)
        self.scale = scale
        # --bf16 (train.py:250-266): dnn and the logits layer in bf16 on fp32
        # master weights (keep_weights), the logit cast back to fp32 -- the
        # MFMA tower with the bf16 head
        self.dnn = (_MfmaMLP if bf16 else _mlp)([off] + list(hidden))
        self.logits = torch.nn.Linear(hidden[-1], 1)
        self.linear_num = torch.nn.Parameter(torch.zeros(len(plain), 1))
        self.linear_ident = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.zeros(self.identity[n], 1))
             for n in self.num_names if n in self.identity])
        self.linear_bias = torch.nn.Parameter(torch.zeros(1))
        self.deep_lookup = _OneHotLookup(self.deep_evs)
        self.wide_lookup = _OneHotLookup(self.wide_evs)

    def deep_parameters(self):
        return list(self.dnn.parameters()) + list(self.logits.parameters())

    def wide_parameters(self):
        return [self.linear_num] + list(self.linear_ident) + [self.linear_bias]

    def _scaled(self, dense):
        if not self.scale:
            return dense
        return (dense - self.num_min.view(1, -1)) / self.num_range.view(1, -1)

    def forward(self, dense, ids):
        dn = self._scaled(dense)
        if self.identity:
            parts = []
            for j, nb in self.dense_layout:
                if nb:
                    parts.append(torch.nn.functional.one_hot(dense[:, j].long(), nb).float())
                else:
                    parts.append(dn[:, j:j + 1])
            dense_block = torch.cat(parts, 1)
        elif self.block_order:
            dense_block = dn.index_select(1, self.num_perm)
        if self.block_order:
            evs = [self.deep_evs[i] for i in self.ev_order]
            emb = embedding_lookup_sparse_multi(evs, self.deep_lookup._sps(ids[self.ev_perm]),
                                                combiner="mean")
            net = torch.cat([emb, dense_block], 1)
        else:
            emb = embedding_lookup_sparse_multi(self.deep_evs, self.deep_lookup._sps(ids),
                                                combiner="mean")
            net = torch.cat([emb, dn], 1).index_select(1, self.perm)
        if (isinstance(self.dnn, _MfmaMLP) and self.dnn.mfma_ok(net.shape[0])
                and self.dnn.head_ok(self.logits)):
            dnn_logits = self.dnn.forward_head(net, self.logits)   # bf16 logit, as fp32
        else:
            dnn_logits = self.bf16(self.logits, self.bf16(self.dnn, net))
        wide = self.wide_lookup(ids)                                # [B, T] (sum of dim-1 rows)
        # dense @ linear_num as a row-wise product sum: the matmul's backward
        # (a [13, B] x [B, 1] GEMM with K = 65 536) ran 0.24 ms on the library
        plain = dn if not self.identity else dn[:, self.plain_idx]
        num = (plain * self.linear_num.view(1, -1)).sum(1, keepdim=True)
        linear_logits = wide.sum(1, keepdim=True) + num + self.linear_bias
        k = 0
        for j, n in enumerate(self.num_names):
            if n in self.identity:
                linear_logits = linear_logits + self.linear_ident[k][dense[:, j].long()]
                k += 1
        return (dnn_logits + linear_logits).squeeze(1)


def wdl_train_step(model, dense, ids, labels, deep_opt, deep_ev_opt, wide_opt, wide_ev_opt,
                   global_step=None):
    """One WDL step (modelzoo/WDL/train.py:302-335): sigmoid cross entropy
    (mean over the batch); deep variables (dnn + embedding EVs) by deep_opt /
    deep_ev_opt (the reference: Adagrad 0.01, accumulator 0.1), linear
    variables by wide_opt / wide_ev_opt (the reference: Ftrl 0.2, l1 = l2 =
    0).  A training.FtrlOptimizer as wide_opt updates the dense linear
    weights elementwise (ApplyFtrl)."""
    from .training import FtrlOptimizer
    logits = model(dense, ids)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, labels)
    deep_opt.zero_grad(set_to_none=True)
    for p in model.wide_parameters():
        p.grad = None
    loss.backward()
    deep_opt.step()
    if isinstance(wide_opt, FtrlOptimizer):
        wide_opt.dense_step(model.wide_parameters())
    else:
        wide_opt.step()
    deep_ev_opt.apply_gradients(model.deep_evs, global_step=global_step)
    wide_ev_opt.apply_gradients(model.wide_evs, global_step=global_step)
    return loss


# DR_CROSSNET_DX_LIB=1 (A/B switch): the input gradient as the library's addmm
_CROSS_DX_LIB = os.environ.get("DR_CROSSNET_DX_LIB", "0") == "1"


def _cross_dx(u, wb, g):
    """dx_l = u W + g of a cross layer: the hand 256^2 MFMA kernel
    (dr_crossnet_dx_bf16, on W^T), one rounding of the fp32 result as
    torch.addmm(g, u, W) in bf16."""
    if _CROSS_DX_LIB:
        return torch.addmm(g, u, wb)
    return ops.crossnet_dx(u, wb.t().contiguous(), g)


# The cross layers' weight gradient: the hand TN MFMA kernel (default;
# dr_crossnet_dw_bf16, 1.35-1.37 ms at B = 65 536, d = 3 392,
# profiles/r05_cross_dw_w4.log) or, DR_CROSSNET_DW=lib, the library GEMM
# writing fp32 (1.43-1.64 ms there)
_CROSS_DW_HAND = os.environ.get("DR_CROSSNET_DW", "hand") == "hand"


def _cross_dw(u, x):
    """dW = u^T x of a cross layer in fp32 (fp32 accumulation, no bf16
    rounding of the result): the hand kernel (dr_crossnet_dw_bf16, 1.35 ms
    at B = 65536, d = 3392 against 1.43-1.64 ms for hipBLASLt); for shapes it
    does not take, or with DR_CROSSNET_DW=lib (A/B), torch.mm with
    out_dtype=float32, the bf16 product widened where that overload is
    absent."""
    if _CROSS_DW_HAND:
        dw = ops.crossnet_dw(u, x)
        if dw is not None:
            return dw
    try:
        return torch.mm(u.t(), x, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        return torch.matmul(u.t(), x).float()


class CrossLayer(torch.autograd.Function):
    """DCN-v2 cross layer x_{l+1} = x0 * (x_l W^T + b) + x_l (BASELINE
    configs[4]; absent from the reference).  Forward: the
    fused bf16 MFMA kernel (dr_crossnet_forward_bf16), which also hands back
    lin = x_l W^T + b for the backward.  Backward (fp32 accumulate): u = g *
    x0, dW = u^T x_l (library GEMM), db = sum u, dx_l = u W + g (the hand
    MFMA kernel), dx0 = g * lin."""

    @staticmethod
    def forward(ctx, x0, xl, weight, bias):
        wb = weight.to(torch.bfloat16)
        out, lin = ops.crossnet_forward(x0, xl, wb, bias, with_lin=True)
        ctx.save_for_backward(x0, xl, wb, lin)
        return out

    @staticmethod
    def backward(ctx, g):
        x0, xl, wb, lin = ctx.saved_tensors
        g = g.to(torch.bfloat16)
        u = g * x0
        dW = _cross_dw(u, xl)
        db = u.float().sum(0)
        dxl = _cross_dx(u, wb, g)
        dx0 = g * lin
        return dx0, dxl, dW, db


class CrossStack(torch.autograd.Function):
    """L stacked cross layers x_{l+1} = x0 * (x_l W_l^T + b_l) + x_l as one
    autograd node.  Forward: the fused MFMA kernel per layer (which hands back
    lin_l for the backward).  Backward, layer by layer in reverse: ONE
    elementwise pass (dr_crossnet_backward_elem_bf16) forms u = g * x0, adds
    g * lin_l into a running fp32 dx0 and the column sums db_l; dW_l = u^T
    x_l (library GEMM) and g <- u W_l + g (= dx_l, the hand MFMA kernel).  The x0
    gradient is the running sum plus the first layer's dx_l (x_0 = x0) --
    what CrossLayer's per-layer autograd adds up in separate bf16 passes."""

    @staticmethod
    def forward(ctx, x0, *params):
        L = len(params) // 2
        ws = [w.to(torch.bfloat16) for w in params[:L]]
        bs = params[L:]
        x = x0
        xs, lins = [], []
        for w, b in zip(ws, bs):
            xs.append(x)
            x, lin = ops.crossnet_forward(x0, x, w, b, with_lin=True)
            lins.append(lin)
        ctx.save_for_backward(x0, *ws, *xs, *lins)
        ctx.L = L
        return x

    @staticmethod
    def backward(ctx, g):
        L = ctx.L
        saved = ctx.saved_tensors
        x0, ws, xs, lins = saved[0], saved[1:1 + L], saved[1 + L:1 + 2 * L], saved[1 + 2 * L:]
        g = g.to(torch.bfloat16).contiguous()
        acc = None
        dws, dbs = [None] * L, [None] * L
        for l in reversed(range(L)):
            u, acc, db = ops.crossnet_backward_elem(g, x0, lins[l], acc)
            dws[l] = _cross_dw(u, xs[l])
            dbs[l] = db
            g = _cross_dx(u, ws[l], g)
        dx0 = (acc + g.float()).to(torch.bfloat16)
        return (dx0, *dws, *dbs)


class DCNv2(torch.nn.Module):
    """DCN-v2 (stacked): x0 = [dense | e_1 .. e_T] zero-padded to a multiple
    of 64 features, bf16; L cross layers on the MFMA kernel; a bf16 deep MLP
    over x_L; one logit, sigmoid, BCE (as DLRM / DeepFM here).  Cross weights
    are fp32 master copies cast to bf16 per step (the reference's bf16 +
    keep_weights convention, modelzoo/DLRM/train.py:183-195).

    bf16=False: the deep MLP and the output layer under torch autocast (bf16
    library GEMMs).  bf16=True: the same bf16 MLP on the hand MFMA towers
    (_MfmaMLP, the cross output x_L is already the padded bf16 input) with
    the output layer riding on the tower node (bf16 weight, rounded logit:
    what autocast's Linear computes), when the batch is a multiple of 512."""

    def __init__(self, evs, num_dense=13, layers=3, deep=(1024, 512), bf16=False, engine=None):
        super().__init__()
        self.mfma_deep = bool(bf16)
        # engine: a row-sharded lookup over this rank's EV shards (BASELINE
        # configs[4] on 8 GPUs; train with train_step_sharded)
        self.engine = engine
        self._sh_anchor = None
        self.evs = list(evs)
        self.dim = self.evs[0].dim
        self.T = len(self.evs)
        self.num_dense = num_dense
        self.d = num_dense + self.T * self.dim
        self.dp = (self.d + 63) // 64 * 64
        dp = self.dp
        ws = []
        for _ in range(layers):
            w = torch.zeros(dp, dp)
            w[:self.d, :self.d] = torch.randn(self.d, self.d) / self.d ** 0.5
            ws.append(torch.nn.Parameter(w))
        self.cross_w = torch.nn.ParameterList(ws)
        self.cross_b = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(dp))
                                               for _ in range(layers)])
        self.deep = (_MfmaMLP if self.mfma_deep else _mlp)([dp] + list(deep))
        self.last = torch.nn.Linear(deep[-1], 1)
        self.lookup = _OneHotLookup(self.evs)

    def forward(self, dense, ids):
        B = dense.shape[0]
        if self.engine is None:
            emb = self.lookup(ids)                                 # [B, T*D] fp32
        else:
            if self._sh_anchor is None:
                self._sh_anchor = torch.zeros(1, device=dense.device, requires_grad=True)
            emb = _sharded_lookup(self._sh_anchor, self.engine, ids)
        if self.mfma_deep:
            # x0 cast column block by column block into one bf16 buffer (no
            # fp32 [B, dp] concat in between); the slice copies keep autograd
            x0 = torch.zeros(B, self.dp, device=dense.device, dtype=torch.bfloat16)
            x0[:, :self.num_dense] = dense
            x0[:, self.num_dense:self.d] = emb
        else:
            pad = torch.zeros(B, self.dp - self.d, device=dense.device, dtype=dense.dtype)
            x0 = torch.cat([dense, emb, pad], 1).to(torch.bfloat16)
        x = CrossStack.apply(x0, *self.cross_w, *self.cross_b)
        if (self.mfma_deep and self.deep.mfma_ok(B) and self.deep.head_ok(self.last)
                and x.shape[1] == self.deep.kp):
            return torch.sigmoid(self.deep.forward_padded_head(x.contiguous(), self.last)).squeeze(1)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            net = self.last(self.deep(x)).float()
        return torch.sigmoid(net).squeeze(1)


class _SplitKLinearFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is a split-K GEMM: for the DIN
    attention MLP x has B*T ~ 4e5 rows and W is 80 x 144, so dW = g^T x is a
    K = 4e5 reduction onto a 1e4-element output, which one library GEMM runs
    on ~15 workgroups (1 ms).  Here K is cut into S slices (a batched GEMM
    with S x more workgroups) and the S partial products are summed."""

    @staticmethod
    def forward(ctx, x, weight, bias, slices):
        ctx.save_for_backward(x, weight)
        ctx.slices = slices
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        gx = g @ weight
        K = x.shape[0]
        S = ctx.slices
        while S > 1 and K % S:
            S //= 2
        if S > 1:
            gw = torch.bmm(g.reshape(S, K // S, -1).transpose(1, 2),
                           x.reshape(S, K // S, -1)).sum(0)
        else:
            gw = g.t() @ x
        return gx, gw, g.sum(0), None


class SplitKLinear(torch.nn.Linear):
    """torch.nn.Linear with a split-K weight gradient for inputs of many rows."""

    def __init__(self, n_in, n_out, slices=64):
        super().__init__(n_in, n_out)
        self.slices = slices

    def forward(self, x):
        shape = x.shape
        y = _SplitKLinearFn.apply(x.reshape(-1, shape[-1]), self.weight, self.bias, self.slices)
        return y.reshape(shape[:-1] + (self.out_features,))


class _DiceFn(torch.autograd.Function):
    """Dice forward / backward as one kernel each (dr_din_dice_forward /
    _backward) instead of ~10 / ~25 elementwise and reduction launches."""

    @staticmethod
    def forward(ctx, x, alpha, epsilon):
        y, st = ops.din_dice_forward(x, alpha, epsilon)
        ctx.save_for_backward(x, alpha, st)
        ctx.epsilon = epsilon
        return y

    @staticmethod
    def backward(ctx, gy):
        x, alpha, st = ctx.saved_tensors
        gx, ga = ops.din_dice_backward(x, gy, alpha, st, ctx.epsilon)
        return gx, ga, None


class _DinFcnInputFn(torch.autograd.Function):
    """inp = [uid, item, his_sum, item * his_sum, att] and the inference
    batch_normalization (model.py:118-124) as one kernel each way
    (dr_din_fcn_input_forward / _backward)."""

    @staticmethod
    def forward(ctx, uid, item, his_sum, att, gamma, beta, scale):
        ctx.save_for_backward(uid, item, his_sum, att, gamma)
        ctx.scale = scale
        return ops.din_fcn_input_forward(uid, item, his_sum, att, gamma, beta, scale)

    @staticmethod
    def backward(ctx, g):
        uid, item, his_sum, att, gamma = ctx.saved_tensors
        gu, gi, gh, ga, gg, gb = ops.din_fcn_input_backward(g, uid, item, his_sum, att, gamma,
                                                            ctx.scale)
        return gu, gi, gh, ga, gg, gb, None


class Dice(torch.nn.Module):
    """dice() of modelzoo/DIN/script/utils.py:12-35 (batch statistics).  On
    the GPU one fused kernel each way (_DiceFn; DR_DIN_DICE_FUSED=0: the
    torch composition, A/B); CPU tensors take the torch composition."""

    fused = os.environ.get("DR_DIN_DICE_FUSED", "1") != "0"

    def __init__(self, n, epsilon=1e-9):
        super().__init__()
        self.alpha = torch.nn.Parameter(torch.zeros(n))
        self.epsilon = epsilon

    def forward(self, x):
        if self.fused and x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.shape[0]:
            return _DiceFn.apply(x, self.alpha, self.epsilon)
        mean = x.mean(0, keepdim=True)
        std = torch.sqrt(((x - mean) ** 2 + self.epsilon).mean(0, keepdim=True))
        xp = torch.sigmoid((x - mean) / (std + self.epsilon))
        return self.alpha * (1.0 - xp) * x + xp * x


class DIN(torch.nn.Module):
    """modelzoo/DIN/script/model.py Model_DIN (use_negsampling=False) on EVs.

    Embedding layer (model.py:61-98): uid / mid / cat EVs of dim D; item_eb =
    [mid, cat] of the target, item_his_eb = [mid, cat] of every history
    position ([B, T, 2D], padding positions look up id 0 like the reference's
    zero-padded id matrix).  Attention (model.py:381-386, utils.py:264-309):
    din_all -> 80 sigmoid -> 40 sigmoid -> 1 -> masked softmax -> weighted
    sum.  FCN (model.py:118-138): batch_normalization in inference form
    (moving mean 0 / variance 1, epsilon 1e-3, trainable gamma / beta), 200
    Dice, 80 Dice, 2, softmax + 1e-8."""

    def __init__(self, uid_ev, mid_ev, cat_ev):
        super().__init__()
        self.uid_ev, self.mid_ev, self.cat_ev = uid_ev, mid_ev, cat_ev
        self.evs = [uid_ev, mid_ev, cat_ev]
        D = mid_ev.dim
        H = 2 * D
        self.f1_att = SplitKLinear(4 * H, 80)
        self.f2_att = SplitKLinear(80, 40)
        self.f3_att = SplitKLinear(40, 1)
        n_in = uid_ev.dim + 4 * H
        self.bn1_gamma = torch.nn.Parameter(torch.ones(n_in))
        self.bn1_beta = torch.nn.Parameter(torch.zeros(n_in))
        self.dnn1 = torch.nn.Linear(n_in, 200)
        self.dice_1 = Dice(200)
        self.dnn2 = torch.nn.Linear(200, 80)
        self.dice_2 = Dice(80)
        self.dnn3 = torch.nn.Linear(80, 2)
        self.uid_lookup = _OneHotLookup([uid_ev])
        self.item_lookup = _OneHotLookup([mid_ev, cat_ev])

    # the attention as one fused node (DinAttentionFused); A/B switch
    # DR_DIN_FUSED_ATTENTION=0 = din_all + library GEMMs + elementwise sigmoids
    fused_attention = os.environ.get("DR_DIN_FUSED_ATTENTION", "1") != "0"

    # the target item and the history in ONE lookup of the mid / cat EVs
    # (A/B switch DR_DIN_ONE_ITEM_LOOKUP=0: two lookups): each EV then gets
    # one gradient whose per-id sums are single serial chains in the order
    # [target positions, history positions] -- the reference's two
    # embedding_lookup gradients concatenated and summed per id by the
    # optimizer's unsorted_segment_sum (optimizer.py _deduplicate_indexed_
    # slices) -- instead of two per-lookup sums added afterwards (a
    # different rounding, and a unique + sort + segment-sum pass per step)
    one_item_lookup = os.environ.get("DR_DIN_ONE_ITEM_LOOKUP", "1") != "0"

    # with the merged lookup, the attention takes allv whole and forms its
    # gradient in one buffer (DinAttentionFusedAll; A/B DR_DIN_FUSED_ALLV=0)
    fused_allv = os.environ.get("DR_DIN_FUSED_ALLV", "1") != "0"

    # the fcn input (concat + inference batch_normalization) as one kernel
    # each way (_DinFcnInputFn; A/B DR_DIN_FUSED_FCN_INPUT=0)
    fused_fcn_input = os.environ.get("DR_DIN_FUSED_FCN_INPUT", "1") != "0"

    def forward(self, uids, mids, cats, mid_his, cat_his, mask):
        B, T = mid_his.shape
        uid_e = self.uid_lookup(uids.reshape(1, B))
        allv = None
        if self.one_item_lookup:
            ids = torch.stack([torch.cat([mids, mid_his.reshape(-1)]),
                               torch.cat([cats, cat_his.reshape(-1)])])
            allv = self.item_lookup(ids)                                           # [B + B T, 2D]
            item_eb = allv[:B]                                                     # [B, 2D]
            facts = allv[B:].view(B, T, -1)                                        # [B, T, 2D]
        else:
            item_eb = self.item_lookup(torch.stack([mids, cats]))                 # [B, 2D]
            his = torch.stack([mid_his.reshape(-1), cat_his.reshape(-1)])
            facts = self.item_lookup(his).view(B, T, -1)                           # [B, T, 2D]
        if (self.fused_attention and facts.shape[2] in ops.DIN_MLP_HIDDEN and allv is not None
                and self.fused_allv and allv.is_contiguous()):
            item_eb, att, his_sum = DinAttentionFusedAll.apply(
                allv, mask, self.f1_att.weight, self.f1_att.bias, self.f2_att.weight,
                self.f2_att.bias, self.f3_att.weight, self.f3_att.bias)
        elif self.fused_attention and facts.shape[2] in ops.DIN_MLP_HIDDEN:
            att, his_sum = DinAttentionFused.apply(
                item_eb, facts, mask, self.f1_att.weight, self.f1_att.bias, self.f2_att.weight,
                self.f2_att.bias, self.f3_att.weight, self.f3_att.bias)
        else:
            din_all = DinAttentionInput.apply(item_eb, facts)                     # [B, T, 4H]
            h = torch.sigmoid(self.f1_att(din_all))
            h = torch.sigmoid(self.f2_att(h))
            scores = self.f3_att(h).view(B, T)
            att, his_sum = DinAttentionPool.apply(scores, mask, facts)
        bn_scale = 1.0 / (1.0 + 1e-3) ** 0.5   # moving variance 1, epsilon 1e-3
        if self.fused_fcn_input and item_eb.is_cuda and item_eb.dtype == torch.float32:
            bn = _DinFcnInputFn.apply(uid_e, item_eb, his_sum, att, self.bn1_gamma,
                                      self.bn1_beta, bn_scale)
        else:
            inp = torch.cat([uid_e, item_eb, his_sum, item_eb * his_sum, att], -1)
            bn = inp * bn_scale * self.bn1_gamma + self.bn1_beta
        x = self.dice_1(self.dnn1(bn))
        x = self.dice_2(self.dnn2(x))
        return torch.softmax(self.dnn3(x), -1) + 1e-8


def din_train_step(model, batch, dense_opt, ev_opt, global_step=None, world=1, group=None,
                   staged=False):
    """One DIN step: ctr_loss = -mean(log(y_hat) * target) (model.py:137),
    backward, dense optimizer, KV optimizer on the uid / mid / cat EVs.
    world > 1: data parallel over replicated EVs (DIN's tables are small:
    every rank holds them whole) -- local loss / world, dense gradients
    all-reduced, every EV's gradient slices gathered in rank order
    (sharded.sync_replicated_grads), so every replica takes the same update
    (BASELINE configs[3], 1 -> 8 GPUs)."""
    uids, mids, cats, mid_his, cat_his, mask, target = batch
    y_hat = model(uids, mids, cats, mid_his, cat_his, mask)
    loss = -(torch.log(y_hat) * target).mean()
    dense_opt.zero_grad(set_to_none=True)
    if world > 1:
        (loss / world).backward()
        allreduce_dense_grads(list(model.parameters()), group=group, staged=staged)
        from .sharded import sync_replicated_grads
        sync_replicated_grads(list(model.evs), group=group, staged=staged)
    else:
        loss.backward()
    dense_opt.step()
    ev_opt.apply_gradients(model.evs, global_step=global_step)
    return loss


def allreduce_dense_grads(params, group=None, staged=False):
    """Sum the dense gradients over the ranks in one bucket per dtype (the
    data-parallel all-reduce; RCCL over xGMI, or host-staged over gloo for a
    rehearsal of several ranks on one GPU)."""
    import torch.distributed as dist
    # every parameter in a fixed order, zeros where this rank's batch left no
    # gradient (as DDP): all ranks reduce buckets of the same size
    by = {}
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        by.setdefault(p.grad.dtype, []).append(p.grad)
    for grads in by.values():
        flat = torch.cat([g.reshape(-1) for g in grads])
        if staged:
            h = flat.cpu()
            dist.all_reduce(h, group=group)
            flat.copy_(h)
        else:
            dist.all_reduce(flat, group=group)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n


def train_step_sharded(model, dense, ids, labels, dense_opt, ev_opt, world, group=None,
                       staged=False, global_step=None):
    """One data-parallel step of a model whose embeddings are row-sharded
    (DLRM(engine=...)): every rank's loss is its local mean / world, so the
    dense gradients summed by allreduce_dense_grads and the sparse gradient
    rows each owner receives from every rank both come to the gradient of
    the global-batch mean; then the dense optimizer (identical on every
    rank) and the KV optimizer on this rank's EV shards.  Returns the local
    mean loss."""
    pred = model(dense, ids)
    eps = 1e-7
    p = pred.clamp(eps, 1 - eps)
    loss = -(labels * torch.log(p) + (1 - labels) * torch.log(1 - p)).mean()
    dense_opt.zero_grad(set_to_none=True)
    (loss / world).backward()
    if world > 1:
        allreduce_dense_grads(list(model.parameters()), group=group, staged=staged)
        rep = list(getattr(model, "replicated_evs", []))
        if rep:
            from .sharded import sync_replicated_grads
            sync_replicated_grads(rep, group=group, staged=staged)
    dense_opt.step()
    ev_opt.apply_gradients(list(model.evs), global_step=global_step)
    return loss


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
