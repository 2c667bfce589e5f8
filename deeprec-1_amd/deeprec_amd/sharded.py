"""Row-sharded embedding lookup across the GPUs of one node.

Every rank holds, for each of the T features, the EV shard of the keys it
owns (owner = key % world, the reference's EV partition rule
key % 1000 % world for world | 1000, embedding_ops.py:207-209, and SOK's
key % G, all2all_input_dispatcher.cu:74).  One forward step:

  1. grouped first-occurrence dedup of the local batch (all features, one pass)
  2. route: stable (owner, feature)-blocked ordering of the uniques
  3. counts all-to-all (world x T int64), one host read of the split sizes
     (SOK syncs here too, all2all_input_dispatcher.cu:256-268)
  4. keys all-to-all (int64)                         -- RCCL over xGMI
  5. owner: tagged insert-on-miss resolve + row pack of the received keys
  6. rows all-to-all back (D fp32 per unique key)     -- RCCL over xGMI
  7. requester: fused gather+pool straight from the received rows
     (rowsel[perm[j]] = j), reference association order

backward() (SURVEY.md 8e backward) runs the exchange in reverse:

  1. requester: grouped segment grad per local unique id (SparseSegment*Grad
     = unsorted_segment_sum over ascending nnz, math_grad.py:321-368)
  2. rows packed into the forward's send order (owner, feature)
  3. grad-rows all-to-all to the owners (the forward's splits, reversed)
  4. owner: the received rows regrouped feature-major, source-rank-major
     inside a feature, and queued on the EV as one IndexedSlices per feature

The owner's slice for feature t is therefore the rank-order concatenation
of every rank's (unique ids, partial grads) for the keys it owns -- what a
data-parallel job hands the optimizer when the replicas' IndexedSlices are
gathered (Horovod's allgather of IndexedSlices, in rank order) -- and the
optimizer deduplicates it exactly as _deduplicate_indexed_slices does
(optimizer.py:68-83; ascending position = ascending source rank), or, for
SGD, applies repeated ids in order.  Deterministic, and equal bit for bit
to the oracle applying the same concatenation.

Parity: the per-bag reduction order is fixed by position within the bag,
never by arrival rank, so the G-GPU output equals the 1-GPU output bit for
bit.  The local steps go through a backend object so the exchange protocol
can be exercised on CPU with world_size-2 gloo (tests/); the product
backend is HipLocal (HIP kernels through the C ABI).
"""
import ctypes as C
import os

import torch
import torch.distributed as dist

from . import _lib, ops
from ._lib import COMBINERS, ORDER_ALI, DrPoolDesc, check, lib, ptr, stream_handle, workspace


class HipLocal(object):
    """Local engine steps on the GPU (the product backend)."""

    def __init__(self, evs, device):
        self.evs = evs
        self.device = device
        self.T = len(evs)
        self.dim = evs[0].dim
        # bf16 EVs exchange bf16 rows (half the link bytes) and pool into a
        # bf16 output; gradients stay fp32
        self.value_dtype = evs[0].value_dtype
        self.bf16 = self.value_dtype == torch.bfloat16
        self.handles = (C.c_void_p * self.T)(*[e.handle.value for e in evs])
        self.filter = any(e.filter_freq != 0 for e in evs)

    def unique_grouped(self, vals, koff):
        return ops.unique_grouped(vals, koff, self.filter)

    def route(self, uniq, koff, num_unique, world):
        return ops.route_by_owner(uniq, koff, num_unique, world)

    def resolve_pack(self, keys, tags, n, per_table):
        """Owner side: insert-on-miss resolve + row pack of n received keys
        (per_table: host list of how many of them belong to each table)."""
        rows = torch.empty(n, dtype=torch.int64, device=self.device)
        out = torch.empty((n, self.dim), dtype=self.value_dtype, device=self.device)
        if n == 0:
            return out
        wsb = lib().dr_ev_resolve_workspace_size(n)
        ws = workspace(wsb, self.device)
        st = stream_handle(self.device)
        pt = (C.c_int64 * self.T)(*[int(x) for x in per_table])
        check(lib().dr_ev_resolve_tagged(self.handles, self.T, ptr(keys), ptr(tags), n, None, pt,
                                         None, ptr(rows), ptr(ws), wsb, st))
        check(lib().dr_ev_gather_tagged(self.handles, self.T, ptr(tags), ptr(rows), n, None,
                                        ptr(out), st))
        ops._post(self.device)
        return out

    def pool_grad(self, grad, idx, koff, num_unique, bag_offs, batch, combiner):
        """Requester backward step 1: grad of every local unique id, in the
        grouped-unique layout (row koff[t] + u), [koff[-1], D] fp32."""
        T, D = self.T, self.dim
        n = koff[-1]
        descs = (_lib.DrPoolGradDesc * T)()
        keep = []
        for t in range(T):
            d = descs[t]
            d.top_grad = grad.data_ptr() + 4 * t * D
            d.top_stride = T * D
            if bag_offs is None:
                d.bag_off, d.seg, d.seg_stride = None, None, 0
            else:
                nt = koff[t + 1] - koff[t]
                seg = torch.repeat_interleave(
                    torch.arange(batch, dtype=torch.int64, device=self.device),
                    (bag_offs[t][1:] - bag_offs[t][:-1]).to(torch.int64), output_size=nt)
                keep.append(seg)
                d.bag_off = bag_offs[t].data_ptr()
                d.seg = seg.data_ptr()
                d.seg_stride = 1
            d.idx = idx.data_ptr() + 4 * koff[t]
            d.nnz = koff[t + 1] - koff[t]
            d.num_unique = num_unique.data_ptr() + 8 * t
            d.combiner = COMBINERS[combiner]
        gu = torch.empty((max(n, 1), D), dtype=torch.float32, device=self.device)
        wsb = lib().dr_pool_grad_grouped_workspace_size(n)
        ws = workspace(wsb, self.device)
        check(lib().dr_pool_grad_grouped(descs, T, batch, D, ptr(gu), ptr(ws), wsb,
                                         stream_handle(self.device)))
        ops._post(self.device)
        return gu

    def pack(self, src, perm):
        """out[j] = src[perm[j]] (perm int32)."""
        out = torch.empty((perm.numel(), self.dim), dtype=torch.float32, device=self.device)
        if perm.numel():
            ops.rows_pack(src, perm, out)
        return out

    def pool(self, rows_recv, rowsel, idx, koff, bag_offs, batch, combiner, out_dtype=None):
        """Requester: pooled [batch, T*D] from the received rows.  rowsel[u]
        is the received row of unique u (idx given: nnz -> unique) or of nnz
        u directly (idx None, the direct one-hot mode)."""
        T, D = self.T, self.dim
        # bf16 rows pool into fp32 (the reference's cast, embedding_ops.py:
        # 606-607) unless a bf16 output is asked for
        out_bf16 = self.bf16 and out_dtype == torch.bfloat16
        out = torch.empty((batch, T * D), dtype=torch.bfloat16 if out_bf16 else torch.float32,
                          device=self.device)
        es = out.element_size()
        descs = []
        for t in range(T):
            d = DrPoolDesc()
            d.pool = rows_recv.data_ptr()
            if idx is None:
                d.ids = rowsel.data_ptr() + 8 * koff[t]
                d.pool_rows = max(int(rows_recv.shape[0]), 1)
            else:
                d.idx = idx.data_ptr() + 4 * koff[t]
                d.rows = rowsel.data_ptr() + 8 * koff[t]
            d.default_rows = rows_recv.data_ptr()
            d.default_stride = 0
            d.bag_off = None if bag_offs is None else bag_offs[t].data_ptr()
            d.out = out.data_ptr() + es * t * D
            d.out_stride = T * D
            d.combiner = COMBINERS[combiner]
            d.max_norm = -1.0
            descs.append(d)
        ops.pool_grouped(descs, batch, D, ORDER_ALI, self.device, onehot=bag_offs is None,
                         bf16=self.bf16, out_bf16=out_bf16)
        return out


class ShardedLookup(object):
    """All-to-all row-sharded embedding_lookup_sparse over T features."""

    def __init__(self, evs, world, rank, batch, device, backend=None, group=None):
        self.evs = evs
        self.world = world
        self.rank = rank
        self.batch = batch
        self.device = device
        self.group = group
        self.backend = backend or HipLocal(evs, device)
        self.T = self.backend.T
        self.dim = self.backend.dim
        self.last_stats = {}
        self._saved = None

    def _a2a(self, out, inp, out_splits=None, in_splits=None):
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
        return out

    def forward(self, ids, bag_offs=None, combiner="sum", need_grad=False, out_dtype=None):
        """ids: [T, nnz] keys (hotness 1 when bag_offs is None: bag b = id b).

        Forward-only one-hot lookups of filter-free EVs route the raw ids
        (no Unique): the owner's insert-on-miss resolve dedups, exactly as
        in the single-GPU direct mode (embedding_ops._prepare_group)."""
        T, G, be = self.T, self.world, self.backend
        dev = ids.device
        nnz = ids.shape[1]
        if bag_offs is None and nnz != self.batch:
            raise ValueError("one-hot ids need nnz == batch (%d != %d)" % (nnz, self.batch))
        vals = ids.reshape(-1)
        koff = [t * nnz for t in range(T + 1)]
        direct = bag_offs is None and not need_grad and not be.filter
        if G == 1 and direct and isinstance(be, HipLocal):
            # a single rank owns every key: no exchange with itself, the
            # local fused lookup (same association order, same EV updates)
            from .embedding_ops import SparseTensor, embedding_lookup_sparse_multi
            ind = torch.stack([torch.arange(nnz, device=dev),
                               torch.zeros(nnz, dtype=torch.int64, device=dev)], 1)
            sps = [SparseTensor(ind, ids[t], (self.batch, 1)) for t in range(T)]
            self.last_stats = {"sent_keys": 0, "recv_keys": 0, "direct": True, "local": True}
            self._saved = None
            with torch.no_grad():
                return embedding_lookup_sparse_multi(self.evs, sps, combiner=combiner,
                                                     out_dtype=out_dtype)
        if direct:
            uniq, idx, U = vals, None, None
        else:
            uniq, idx, _cnt, U = be.unique_grouped(vals, koff)
        keys_s, tags_s, perm, counts = be.route(uniq, koff, U, G)
        # 3. counts exchange (peer-major [G, T]) and one host read of the splits
        recv_counts = torch.empty_like(counts)
        self._a2a(recv_counts.view(-1), counts.view(-1))
        both = torch.cat([counts.view(-1), recv_counts.view(-1)]).cpu()
        sc = both[:G * T].view(G, T)
        rc = both[G * T:].view(G, T)
        send_splits = sc.sum(1).tolist()
        recv_splits = rc.sum(1).tolist()
        S, R = int(sum(send_splits)), int(sum(recv_splits))
        # 4. keys all-to-all
        keys_r = torch.empty(R, dtype=torch.int64, device=dev)
        self._a2a(keys_r, keys_s[:S], recv_splits, send_splits)
        tags_r = torch.repeat_interleave(
            torch.arange(T, dtype=torch.int32, device=dev).repeat(G),
            recv_counts.view(-1), output_size=R)
        # 5. owner resolve + pack, 6. rows all-to-all back
        rows_s = be.resolve_pack(keys_r, tags_r, R, rc.sum(0).tolist())
        rows_r = torch.empty((S, self.dim), dtype=rows_s.dtype, device=dev)
        self._a2a(rows_r, rows_s, send_splits, recv_splits)
        # 7. requester: (unique | nnz) position -> row in the received buffer
        rowsel = torch.zeros(T * nnz, dtype=torch.int64, device=dev)
        rowsel[perm[:S].to(torch.int64)] = torch.arange(S, dtype=torch.int64, device=dev)
        if out_dtype is None:
            out = be.pool(rows_r, rowsel, idx, koff, bag_offs, self.batch, combiner)
        else:
            out = be.pool(rows_r, rowsel, idx, koff, bag_offs, self.batch, combiner, out_dtype)
        self.last_stats = {"sent_keys": S, "recv_keys": R, "direct": direct}
        self._saved = None
        if need_grad:
            self._saved = dict(idx=idx, koff=koff, U=U, perm=perm[:S], keys_r=keys_r, rc=rc,
                               send=send_splits, recv=recv_splits, bag_offs=bag_offs,
                               combiner=combiner)
        return out

    def backward(self, grad_out):
        """grad_out: [B, T*D] gradient of the last forward(need_grad=True).

        Returns, per feature t, the owner-side (keys [n_t], grads [n_t, D])
        slice (source-rank-major), and queues it on evs[t].pending_grads as an
        IndexedSlices for the optimizer (training.py)."""
        sv = self._saved
        if sv is None:
            raise RuntimeError("backward() needs a forward(..., need_grad=True) first")
        self._saved = None
        T, G, D, be = self.T, self.world, self.dim, self.backend
        g = grad_out.float().contiguous()
        if tuple(g.shape) != (self.batch, T * D):
            raise ValueError("grad must be [%d, %d]" % (self.batch, T * D))
        # 1-2. per-unique grads, packed into the forward's send order
        gu = be.pool_grad(g, sv["idx"], sv["koff"], sv["U"], sv["bag_offs"], self.batch,
                          sv["combiner"])
        grads_s = be.pack(gu, sv["perm"])
        # 3. grad rows to the owners (reverse of the rows all-to-all)
        R = int(sum(sv["recv"]))
        grads_r = torch.empty((R, D), dtype=torch.float32, device=g.device)
        self._a2a(grads_r, grads_s, sv["recv"], sv["send"])
        # 4. regroup [source][feature] blocks feature-major: a block permutation
        rc = sv["rc"]                                    # host [G, T]
        n_t = rc.sum(0).tolist()
        src_start = [[0] * T for _ in range(G)]
        acc = 0
        for p in range(G):
            for t in range(T):
                src_start[p][t] = acc
                acc += int(rc[p, t])
        blocks, starts, lens = [], [], []
        acc = 0
        for t in range(T):
            for p in range(G):
                blocks.append(src_start[p][t] - acc)
                lens.append(int(rc[p, t]))
                acc += int(rc[p, t])
        dev = g.device
        shift = torch.repeat_interleave(torch.tensor(blocks, dtype=torch.int64),
                                        torch.tensor(lens, dtype=torch.int64)).to(dev)
        perm_t = (torch.arange(R, dtype=torch.int64, device=dev) + shift).to(torch.int32)
        keys_t = sv["keys_r"][perm_t.to(torch.int64)]
        grads_t = be.pack(grads_r, perm_t)
        out, off = [], 0
        for t in range(T):
            k = keys_t[off:off + n_t[t]]
            v = grads_t[off:off + n_t[t]]
            off += n_t[t]
            out.append((k, v))
            if self.evs is not None:
                from .kv_variable_ops import IndexedSlices
                self.evs[t].pending_grads.append(IndexedSlices(v, k, unique=False))
        return out


class Comm(object):
    """A dr_comm (include/deeprec_amd.h): the collective of the native sharded
    engine (NativeShardedLookup).

    Comm.rccl(rank, world): RCCL over xGMI -- rank 0 draws the ncclUniqueId
    (dr_comm_rccl_unique_id) and torch.distributed hands it to every rank.
    Comm.host_staged(group): the all-to-all of a torch.distributed process
    group on host copies of the buffers (gloo: CPU collectives) through the
    callback table -- how a host framework plugs its own collective in, and
    how the engine is exercised on one GPU with several processes."""

    def __init__(self, handle, world, rank, keep=()):
        self.h = handle
        self.world, self.rank = world, rank
        self._keep = keep

    @classmethod
    def rccl(cls, rank, world, group=None):
        uid = (C.c_char * _lib.RCCL_UNIQUE_ID_BYTES)()
        if rank == 0:
            check(lib().dr_comm_rccl_unique_id(uid, _lib.RCCL_UNIQUE_ID_BYTES))
        box = [bytes(uid)]
        if world > 1:
            dist.broadcast_object_list(box, src=0, group=group)
        uid = (C.c_char * _lib.RCCL_UNIQUE_ID_BYTES).from_buffer_copy(box[0])
        h = C.c_void_p()
        check(lib().dr_comm_init(uid, rank, world, None, C.byref(h)))
        return cls(h, world, rank)

    @classmethod
    def host_staged(cls, group=None):
        import numpy as np
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        errors = []

        def a2a(user, send, sc, recv, rc, eb, stream):
            try:
                scl = [int(sc[i]) * eb for i in range(world)]
                rcl = [int(rc[i]) * eb for i in range(world)]
                hs = np.empty(max(sum(scl), 1), np.uint8)
                hr = np.empty(max(sum(rcl), 1), np.uint8)
                check(lib().dr_memcpy(hs.ctypes.data, send, sum(scl), 1, stream))
                dist.all_to_all_single(torch.from_numpy(hr[:sum(rcl)]),
                                       torch.from_numpy(hs[:sum(scl)]), rcl, scl, group=group)
                check(lib().dr_memcpy(recv, hr.ctypes.data, sum(rcl), 1, stream))
                return 0
            except Exception as e:  # noqa: BLE001 -- reported as the call's status
                errors.append(e)
                return 1

        def gather(user, send, nbytes, recv):
            # the XGMI engine's IPC handle exchange (setup only)
            try:
                mine = C.string_at(send, nbytes)
                allb = [None] * world
                dist.all_gather_object(allb, mine, group=group)
                C.memmove(recv, b"".join(allb), nbytes * world)
                return 0
            except Exception as e:  # noqa: BLE001
                errors.append(e)
                return 1

        def barrier(user, stream):
            # host-blocking: the stream's work first, then every rank
            try:
                if stream:
                    torch.cuda.ExternalStream(stream).synchronize()
                else:
                    torch.cuda.synchronize()
                dist.barrier(group=group)
                return 0
            except Exception as e:  # noqa: BLE001
                errors.append(e)
                return 1

        fn = _lib.COMM_A2A_FN(a2a)
        gfn = _lib.COMM_GATHER_FN(gather)
        bfn = _lib.COMM_BARRIER_FN(barrier)
        ops_ = _lib.DrCommOps(None, fn, gfn, bfn)
        h = C.c_void_p()
        check(lib().dr_comm_init(None, rank, world, C.byref(ops_), C.byref(h)))
        return cls(h, world, rank, keep=(fn, gfn, bfn, ops_, errors))

    def close(self):
        if self.h is not None and self.h.value:
            lib().dr_comm_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class NativeShardedLookup(object):
    """The row-sharded embedding_lookup_sparse through the library's own
    sharded C entries (dr_sharded_forward / dr_sharded_backward over a
    dr_comm): the same protocol and results as ShardedLookup -- index
    all-to-all, owner insert-on-miss resolve + row pack, row all-to-all back,
    ALI-order pooling; the owner's IndexedSlices in the backward -- with the
    sequence inside the C library, as a TF custom-op kernel would drive it
    (INTEGRATION.md)."""

    def __init__(self, comm, evs, device, kind="rccl", batch=0, max_ids=0):
        """kind: "rccl" (dr_sharded_create: exact-size all-to-alls, host reads
        of the split sizes), "xgmi" (peer writes over IPC-mapped buffers;
        one-hot sum over `batch` bags; no host read) or "fixed" (the
        all-to-alls at fixed capacity, `max_ids` ids per table per rank;
        no host read) -- dr_sharded_create_ex."""
        self.comm, self.evs, self.device = comm, list(evs), device
        self.T = len(self.evs)
        self.dim = self.evs[0].dim
        self.bf16 = self.evs[0].value_dtype == torch.bfloat16
        self.kind = kind
        self.batch = int(batch)
        hs = (C.c_void_p * self.T)(*[e.handle.value for e in self.evs])
        self.h = C.c_void_p()
        if kind == "rccl":
            check(lib().dr_sharded_create(comm.h, hs, self.T, C.byref(self.h)))
        else:
            k = {"xgmi": _lib.SHARDED_XGMI, "fixed": _lib.SHARDED_RCCL_FIXED}[kind]
            cfg = _lib.DrShardedConfig(k, 0, int(batch), int(max_ids))
            with torch.cuda.device(device):
                check(lib().dr_sharded_create_ex(comm.h, hs, self.T, C.byref(cfg),
                                                 C.byref(self.h)))
        self._keep = None

    def output(self, out_dtype=None):
        """XGMI kind: the engine buffer with the last forward's result (the
        EVs' value type) as a tensor view -- forward(..., copy=False)."""
        p = C.c_void_p()
        check(lib().dr_sharded_output(self.h, C.byref(p)))
        dt = torch.bfloat16 if self.bf16 else torch.float32
        v = getattr(self, "_out_view", None)
        if v is None or v[0] != p.value or v[1] != dt:   # the engine's buffer is fixed: one view
            self._out_view = (p.value, dt, _lib.device_view(p.value, (self.batch, self.T * self.dim),
                                                            dt, self.device))
        return self._out_view[2]

    def forward(self, ids, bag_offs=None, combiner="sum", need_grad=False, out_dtype=None,
                copy=True):
        """ids: [T, B] int64 (one-hot, bag_offs None) or T 1-D int64 tensors
        (table t's ids); bag_offs None or T int32 [bags + 1] offsets covering
        each table's ids.  Returns [bags, T*D] (fp32; bf16 on request for bf16
        EVs)."""
        T = self.T
        flat = None
        if torch.is_tensor(ids):
            if ids.dim() == 2 and ids.dtype == torch.int64 and ids.is_contiguous():
                flat = ids.reshape(-1)   # [T, B] table-major already: no copy
            ids = [ids[t] for t in range(ids.shape[0])]
        if len(ids) != T:
            raise ValueError("ids of %d tables expected" % T)
        lens = [int(x.numel()) for x in ids]
        koff = [0]
        for n in lens:
            koff.append(koff[-1] + n)
        if flat is None:
            flat = torch.cat([x.reshape(-1).to(torch.int64) for x in ids]).contiguous()
        if bag_offs is None:
            bags, offs = lens[0], None
        else:
            bag_offs = [o.to(torch.int32).contiguous() for o in bag_offs]
            bags = int(bag_offs[0].numel()) - 1
            offs = (C.c_void_p * T)(*[o.data_ptr() for o in bag_offs])
        bf = out_dtype == torch.bfloat16
        out = None
        if copy:
            out = torch.empty((bags, T * self.dim), dtype=torch.bfloat16 if bf else torch.float32,
                              device=self.device)
        ka = (C.c_int64 * (T + 1))(*koff)
        check(lib().dr_sharded_forward(self.h, ptr(flat), ka, offs, bags, COMBINERS[combiner],
                                       1 if need_grad else 0, _lib.SHARDED_OUT_BF16 if bf else 0,
                                       ptr(out), stream_handle(self.device)))
        if out is None:
            out = self.output()
        ops._post(self.device)
        self._keep = (flat, bag_offs) if need_grad else None
        return out

    def stats(self):
        a, b = C.c_int64(0), C.c_int64(0)
        check(lib().dr_sharded_last_stats(self.h, C.byref(a), C.byref(b)))
        return {"sent_keys": a.value, "recv_keys": b.value}

    def backward(self, grad_out):
        """grad_out [bags, T*D] -> per table the owner's (keys, grads) slice,
        also queued on evs[t].pending_grads as IndexedSlices."""
        from .kv_variable_ops import IndexedSlices
        T, D = self.T, self.dim
        g = grad_out.float().contiguous()
        if self.kind != "rccl":
            return self._backward_dev(g)
        kp, gp, cn = (C.c_void_p * T)(), (C.c_void_p * T)(), (C.c_int64 * T)()
        st = stream_handle(self.device)
        check(lib().dr_sharded_backward(self.h, ptr(g), kp, gp, cn, st))
        out = []
        for t in range(T):
            n = int(cn[t])
            k = torch.empty(n, dtype=torch.int64, device=self.device)
            v = torch.empty((n, D), dtype=torch.float32, device=self.device)
            if n:
                check(lib().dr_memcpy(k.data_ptr(), kp[t], 8 * n, 0, st))
                check(lib().dr_memcpy(v.data_ptr(), gp[t], 4 * n * D, 0, st))
            out.append((k, v))
            self.evs[t].pending_grads.append(IndexedSlices(v, k, unique=False))
        ops._post(self.device)
        self._keep = None
        return out

    def _backward_dev(self, g):
        """XGMI / fixed kinds: no host read -- each table's IndexedSlices is a
        fixed region of the engine's buffers with a DEVICE count (copied out
        here, so the slices outlive the next call)."""
        from .kv_variable_ops import IndexedSlices
        T, D = self.T, self.dim
        kp, gp, cp = (C.c_void_p * T)(), (C.c_void_p * T)(), (C.c_void_p * T)()
        region = C.c_int64(0)
        st = stream_handle(self.device)
        check(lib().dr_sharded_backward_dev(self.h, ptr(g), kp, gp, cp, C.byref(region), st))
        R = region.value
        keys = torch.empty((T, R), dtype=torch.int64, device=self.device)
        grads = torch.empty((T, R, D), dtype=torch.float32, device=self.device)
        cnt = torch.empty(T, dtype=torch.int64, device=self.device)
        for t in range(T):
            keys[t].copy_(_lib.device_view(kp[t], (R,), torch.int64, self.device))
            grads[t].copy_(_lib.device_view(gp[t], (R, D), torch.float32, self.device))
        cnt.copy_(_lib.device_view(cp[0], (T,), torch.int64, self.device))
        out = []
        for t in range(T):
            n = cnt[t:t + 1]
            out.append((keys[t], grads[t], n))
            self.evs[t].pending_grads.append(IndexedSlices(grads[t], keys[t], num_valid=n,
                                                           unique=False))
        ops._post(self.device)
        self._keep = None
        return out

    def close(self):
        self._out_view = None
        if self.h is not None and self.h.value:
            lib().dr_sharded_destroy(self.h)
        self.h = None

    def __del__(self):
        # dr_sharded_create retained every EV: an engine dropped without
        # close() must still release them.  dr_sharded_destroy synchronises
        # the device, so it goes through the EVs' capture-safe deferred path.
        h = getattr(self, "h", None)
        if h is not None and h.value:
            from .kv_variable_ops import _release_engine
            _release_engine("dr_sharded_destroy", h)
            self.h = None


def hybrid_split(cardinalities, replicate_max):
    """Features whose vocabulary is at most `replicate_max` rows are
    replicated on every rank, the others row-sharded (key % world).  On the
    real Criteo-TB cardinalities (modelzoo/SOK/DLRM/train_stand.py:242-248)
    with replicate_max = 585 935, 20 of the 26 features (1.11 M rows, 0.57 GB
    at D = 128 fp32) are replicated and 6 (1.87e8 rows) sharded."""
    rep = [t for t, c in enumerate(cardinalities) if c <= replicate_max]
    shard = [t for t, c in enumerate(cardinalities) if c > replicate_max]
    return rep, shard


class HybridShardedLookup(object):
    """Hybrid placement for row-sharded one-hot lookups (SURVEY 8e levers):
    the replicated features are looked up locally -- no link bytes at all --
    and only the sharded ones go through `engine` (XgmiShardedLookup,
    ShardedLookup or NativeShardedLookup over those features' EV shards).
    With overlap, the local lookup runs on a side stream while the exchange
    runs on the current one (the local part reads HBM, the exchange is
    link-bound).

    forward(ids_rep [T_r, B], ids_shard [T_s, B]) -> (out_rep [B, T_r*D],
    out_shard [B, T_s*D]): the replicated and the sharded features' pooled
    columns as two blocks (a model stacks them behind its dense row, as
    embedding_stack does).  Results are each feature's single-GPU lookup, bit
    for bit: the local part IS the single-GPU lookup, the sharded part is
    position-addressed by the engine.

    local_lookup(ids_rep) -> out_rep is the replicated features' lookup (the
    fused one-hot kernel over their tables on the GPU; any callable in
    tests)."""

    def __init__(self, local_lookup, engine, device=None, overlap=True):
        self.local_lookup = local_lookup
        self.engine = engine
        self.device = device
        use_side = overlap and device is not None and torch.device(device).type == "cuda"
        self.side = torch.cuda.Stream(device=device) if use_side else None

    def forward(self, ids_rep, ids_shard):
        if self.side is None:
            out_r = self.local_lookup(ids_rep)
            out_s = self.engine.forward(ids_shard)
            return out_r, out_s
        cur = torch.cuda.current_stream(self.device)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            out_r = self.local_lookup(ids_rep)
        out_s = self.engine.forward(ids_shard)
        cur.wait_stream(self.side)
        out_r.record_stream(cur)
        return out_r, out_s


def sync_replicated_grads(evs, group=None, staged=False):
    """Data-parallel gradients of REPLICATED EVs (hybrid placement's small
    features, every rank holding the whole table): each rank's pending
    gradient slices of every EV are gathered and every rank queues the same
    rank-order concatenation (Horovod's allgather of IndexedSlices, in rank
    order), so the KV optimizer -- which deduplicates a slice by key in
    position order -- applies identical updates to every replica.  staged:
    the collectives on host copies (gloo rehearsal on one GPU).  One host
    read of the slice sizes per EV (the gather is variable-sized)."""
    from .kv_variable_ops import IndexedSlices
    world = dist.get_world_size(group)
    for ev in evs:
        ks, vs = [], []
        for sl in ev.pending_grads:
            k, v = sl.indices, sl.values
            if sl.num_valid is not None:
                n = int(sl.num_valid.reshape(-1)[0].item())
                k, v = k[:n], v[:n]
            ks.append(k.reshape(-1).to(torch.int64))
            vs.append(v.reshape(-1, ev.dim).to(torch.float32))
        dev = ev.device
        k = torch.cat(ks) if ks else torch.empty(0, dtype=torch.int64, device=dev)
        v = torch.cat(vs) if vs else torch.empty((0, ev.dim), dtype=torch.float32, device=dev)
        cdev = torch.device("cpu") if staged else k.device
        n = torch.tensor([k.numel()], dtype=torch.int64, device=cdev)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n, group=group)
        sizes = [int(x.item()) for x in sizes]
        m = max(max(sizes), 1)
        kp = torch.zeros(m, dtype=torch.int64, device=cdev)
        vp = torch.zeros((m, ev.dim), dtype=torch.float32, device=cdev)
        kp[:k.numel()] = k.to(cdev)
        vp[:k.numel()] = v.to(cdev)
        kall = [torch.empty_like(kp) for _ in range(world)]
        vall = [torch.empty_like(vp) for _ in range(world)]
        dist.all_gather(kall, kp, group=group)
        dist.all_gather(vall, vp, group=group)
        kc = torch.cat([kall[r][:sizes[r]] for r in range(world)]).to(dev)
        vc = torch.cat([vall[r][:sizes[r]] for r in range(world)]).to(dev)
        ev.pending_grads.clear()
        if kc.numel():
            ev.pending_grads.append(IndexedSlices(vc, kc, unique=False))


class _ReduceScatterFn(torch.autograd.Function):
    """out[B, C] = sum over ranks of their partial[rank's bags]; backward =
    the all-gather of the gradient (every owner needs every rank's rows)."""

    @staticmethod
    def forward(ctx, partial, eng):
        ctx.eng = eng
        return eng._reduce_scatter(partial.contiguous())

    @staticmethod
    def backward(ctx, g):
        return ctx.eng._all_gather_fixed(g.contiguous()), None


class ReduceScatterShardedLookup(object):
    """SOK's owner-side pooling for multi-hot bags (the DistributedEmbedding
    of modelzoo/SOK: forward_functions.cuh:72-97 pools on the owner,
    reduce_scatter_dispatcher.cu:45-52 sums the partial bags and scatters
    the batch), over the same row sharding (owner = key % world):

      1. all-gather the per-feature id counts, the ids (uneven sizes, one
         all-to-all) and the CSR bag offsets of every rank;
      2. owner: keep the ids it owns, pool them per global bag with the
         fused lookup (combiner sum; bags without an owned id are 0) into a
         [world * B, T * D] partial;
      3. mean / sqrtn divide the partials by the global bag size, then
         reduce-scatter (sum) -> this rank's [B, T * D].

    Per bag the exchange carries T * D floats per rank pair instead of one
    row per id: cheaper than the row all-to-all once bags hold more ids than
    there are ranks.  Backward: the gradient is all-gathered and the owners'
    lookups queue IndexedSlices of their own keys.  The per-bag sum is
    associated per owner, then across owners, so results match the
    single-GPU lookup to fp32 tolerance, not bit for bit.  _all_gather_fixed
    / _all_gather_var / _reduce_scatter are torch.distributed collectives
    (RCCL); tests replace them to run several ranks in one process."""

    def __init__(self, evs, world, rank, batch, device, group=None):
        self.evs = list(evs)
        self.world, self.rank, self.batch = world, rank, batch
        self.device = device
        self.group = group
        self.T = len(self.evs)
        self.dim = self.evs[0].dim

    # -- collectives -----------------------------------------------------
    def _all_gather_fixed(self, t):
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out.reshape((self.world * t.shape[0],) + tuple(t.shape[1:]))

    def _all_gather_var(self, t, sizes):
        out = torch.empty(int(sum(sizes)), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t.repeat(self.world), list(sizes), [t.numel()] * self.world,
                               group=self.group)
        return out

    def _reduce_scatter(self, t):
        out = torch.empty((t.shape[0] // self.world,) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        dist.reduce_scatter_tensor(out, t, group=self.group)
        return out

    # -- step ------------------------------------------------------------
    def forward(self, ids, bag_offs, combiner="sum"):
        """ids[t]: [nnz_t] int64 ids of feature t; bag_offs[t]: [B + 1] int32
        CSR offsets of its bags.  Returns [B, T * D] (autograd-enabled: the
        EVs receive their IndexedSlices on backward)."""
        from .embedding_ops import SparseTensor, embedding_lookup_sparse_multi
        if combiner not in ("sum", "mean", "sqrtn"):
            raise ValueError("combiner must be one of 'sum', 'mean' or 'sqrtn'")
        T, G, B, dev = self.T, self.world, self.batch, self.device
        ids = [x.reshape(-1).to(torch.int64) for x in ids]
        offs = torch.stack([o.to(torch.int64).reshape(-1) for o in bag_offs])       # [T, B+1]
        if offs.shape != (T, B + 1):
            raise ValueError("bag_offs must be T x [B + 1]")
        nnz = torch.tensor([x.numel() for x in ids], dtype=torch.int64, device=dev)
        sizes = self._all_gather_fixed(nnz).reshape(G, T).cpu()                      # host
        per_rank = sizes.sum(1).tolist()
        all_ids = self._all_gather_var(torch.cat(ids), per_rank)
        all_offs = self._all_gather_fixed(offs).reshape(G, T, B + 1)
        rank_base = [0]
        for r in range(G):
            rank_base.append(rank_base[-1] + int(per_rank[r]))
        sps = []
        for t in range(T):
            vals, segs = [], []
            for r in range(G):
                a = rank_base[r] + int(sizes[r, :t].sum())
                v = all_ids[a:a + int(sizes[r, t])]
                o = all_offs[r, t]
                seg = torch.repeat_interleave(torch.arange(B, device=dev) + r * B, o[1:] - o[:-1],
                                              output_size=v.numel())
                vals.append(v)
                segs.append(seg)
            v = torch.cat(vals)
            seg = torch.cat(segs)
            own = torch.nonzero(v % G == self.rank).reshape(-1)        # sizes: host sync
            v, seg = v[own].contiguous(), seg[own]
            ind = torch.stack([seg, torch.zeros_like(seg)], 1)
            sps.append(SparseTensor(ind, v, (G * B, max(1, int(v.numel())))))
        partial = embedding_lookup_sparse_multi(self.evs, sps, combiner="sum")   # [G*B, T*D]
        if combiner != "sum":            # the global bag sizes are known to every owner
            cnt = (all_offs[:, :, 1:] - all_offs[:, :, :-1]).permute(0, 2, 1)
            cnt = cnt.reshape(G * B, T).to(torch.float32)
            if combiner == "sqrtn":
                cnt = torch.sqrt(cnt)
            cnt = torch.where(cnt > 0, cnt, torch.ones_like(cnt))
            partial = (partial.view(G * B, T, self.dim) / cnt[:, :, None]).reshape(G * B, -1)
        return _ReduceScatterFn.apply(partial, self)                             # [B, T*D]


class XgmiBuffers(object):
    """One rank's exchange buffers for XgmiShardedLookup (torch allocations
    shared with the peers through HIP IPC): the inbox that requesters write
    (key, slot) pairs into, the [B, T*D] output that owners write rows into,
    and the [B, T*D] gradient that owners pull rows from in backward()."""

    def __init__(self, world, T, batch, dim, device, uncached=None, value_dtype=torch.float32):
        # uncached (dr_ipc_alloc): a peer's xGMI writes can never be hidden by
        # a stale line in one of this GPU's per-XCD L2s; uncached=False keeps
        # plain torch allocations (single-process tests, all "ranks" on one
        # device and one set of L2s)
        if uncached is None:
            uncached = os.environ.get("DEEPREC_AMD_IPC_UNCACHED", "1") != "0"
        alloc = _lib.uncached_empty if uncached else \
            (lambda shape, dtype, dev: torch.zeros(shape, dtype=dtype, device=dev))
        self.cap = T * batch
        self.uncached = uncached
        self.inbox_keys = alloc((world, self.cap), torch.int64, device)
        self.inbox_slot = alloc((world, self.cap), torch.int32, device)
        self.inbox_cnt = alloc((world,), torch.int64, device)
        self.out = alloc((batch, T * dim), value_dtype, device)   # bf16 EVs: bf16 rows
        self.gin = alloc((batch, T * dim), torch.float32, device)

    def tensors(self):
        return [self.inbox_keys, self.inbox_slot, self.inbox_cnt, self.out, self.gin]


class XgmiShardedLookup(object):
    """Row-sharded one-hot embedding_lookup_sparse(sum) over xGMI peer writes.

    Same partitioning and results as ShardedLookup (owner = key % world,
    outputs bit-identical to one GPU), without staging copies: requesters
    write (key, slot) pairs straight into the owners' inboxes and owners
    write rows straight into the requesters' outputs (dr_xgmi_route /
    dr_xgmi_serve).  Two stream-ordered cross-rank barriers (a one-element
    RCCL all_reduce each) separate the phases; there is no host sync.

    forward() returns this rank's persistent output buffer: it is rewritten
    by the next forward(), so consume it (on the same stream) first.
    peer_buffers / barrier let tests run several ranks in one process.

    dedup=True: per-destination dedup before the exchange (SOK,
    all2all_input_dispatcher.cu:36-126): the requester runs the grouped
    first-occurrence Unique over its [T, B] ids, routes each table's unique
    keys only (dr_xgmi_route_ex), the owners write one row per unique key
    into the (then staging) peer buffer at slot u*T + t, and the requester
    expands them over its bags with the one-hot pooling kernel into a local
    output.  The links carry one row per distinct key instead of one per
    id -- the lever for skewed (Zipf / real-cardinality) batches; the
    Unique and the local expansion are the price.  The backward sums each
    unique key's gradient locally first (dr_pool_grad_grouped, the
    reference's per-worker IndexedSlices) and the owners pull those rows.
    Outputs are bit-identical to the non-dedup path and to one GPU.

    Multi-hot bags (forward(ids, bag_offs=...)): ids [T, nnz] with nnz up to
    the engine's per-table key capacity `batch`, bag_offs[t] int32 [bags+1]
    (the same bag count for every table), combiner sum / mean / sqrtn.  They
    always take the Unique route above (embedding_lookup_sparse's own Unique,
    embedding_ops.py:592-675): unique keys routed, one row per unique key
    served into the staging buffer, then the ALI-order segment pooling over
    the bags (SparseSegmentReduction, segment_reduction_ali_ops_util.h:193-
    318); backward: each unique key's SparseSegment*Grad sum, pulled by its
    owner.  No host read in either direction."""

    def __init__(self, evs, world, rank, batch, device, group=None, peer_buffers=None,
                 barrier=None, buffers=None, dedup=False):
        if world > _lib.MAX_PEERS:
            raise ValueError("world %d > %d" % (world, _lib.MAX_PEERS))
        for e in evs:
            if e.filter_freq != 0:
                raise ValueError("XgmiShardedLookup needs filter-free EVs")
        self.evs = evs
        self.world, self.rank, self.batch = world, rank, batch
        self.device = device
        self.group = group
        self.T = len(evs)
        self.dim = evs[0].dim
        self.handles = (C.c_void_p * self.T)(*[e.handle.value for e in evs])
        # an allocation or export failure on one rank must not leave the others
        # waiting in the handle exchange: it is carried into the all-gather
        # and every rank raises together after it
        self._setup_err = None
        try:
            self.bufs = buffers or XgmiBuffers(world, self.T, batch, self.dim, device,
                                               value_dtype=evs[0].value_dtype)
        except Exception as e:  # noqa: BLE001 -- re-raised after the exchange
            if world == 1 or peer_buffers is not None:
                raise
            self.bufs, self._setup_err = None, "rank %d: %s" % (rank, e)
        self._bases = []
        if world == 1 and peer_buffers is None:
            peer_buffers = [self.bufs]
            barrier = barrier or (lambda: None)
        if peer_buffers is None:
            peer_ptrs = self._exchange_ipc()
        else:
            peer_ptrs = [[t.data_ptr() for t in b.tensors()] for b in peer_buffers]
        p = _lib.DrXgmiPeers()
        p.world, p.rank, p.cap = world, rank, self.bufs.cap
        for q in range(world):
            p.inbox_keys[q], p.inbox_slot[q], p.inbox_cnt[q], p.out[q] = peer_ptrs[q][:4]
        self.peers = p
        self.gin_ptrs = (C.c_void_p * world)(*[peer_ptrs[q][4] for q in range(world)])
        self.cnt_ws = torch.zeros(world, dtype=torch.int64, device=device)
        self.wsb = lib().dr_xgmi_serve_workspace_size(world, self.bufs.cap)
        self.ws = workspace(self.wsb, device)
        self.flag = torch.zeros(1, dtype=torch.float32, device=device)
        self._barrier = barrier or self._rccl_barrier
        self.dedup = bool(dedup)
        self._local = HipLocal(evs, device)
        self._koff = [t * batch for t in range(self.T + 1)]
        self._tcol = torch.arange(self.T, dtype=torch.int64, device=device)[:, None]
        self._saved = None

    def _exchange_ipc(self):
        mine = []
        try:
            if self._setup_err is not None:
                raise RuntimeError(self._setup_err)
            for t in self.bufs.tensors():
                h = (C.c_char * _lib.IPC_HANDLE_BYTES)()
                off = C.c_int64(0)
                check(lib().dr_ipc_export(t.data_ptr(), h, C.byref(off)))
                mine.append((bytes(h), off.value))
        except Exception as e:  # noqa: BLE001 -- every rank raises below
            mine = "rank %d: %s" % (self.rank, e)
        everyone = [None] * self.world
        dist.all_gather_object(everyone, mine, group=self.group)
        errs = [m for m in everyone if isinstance(m, str)]
        if errs:
            raise RuntimeError("xgmi IPC setup failed: " + "; ".join(errs))
        ptrs = []
        for q in range(self.world):
            if q == self.rank:
                ptrs.append([t.data_ptr() for t in self.bufs.tensors()])
                continue
            row = []
            for hb, off in everyone[q]:
                h = (C.c_char * _lib.IPC_HANDLE_BYTES).from_buffer_copy(hb)
                pp, base = C.c_void_p(), C.c_void_p()
                check(lib().dr_ipc_import(h, off, C.byref(pp), C.byref(base)))
                self._bases.append(base.value)
                row.append(pp.value)
            ptrs.append(row)
        return ptrs

    def _rccl_barrier(self):
        dist.all_reduce(self.flag, group=self.group)

    def route(self, ids, n_dev=None):
        check(lib().dr_xgmi_route_ex(C.byref(self.peers), ptr(ids), self.T, self.batch,
                                     ptr(n_dev), ptr(self.cnt_ws), stream_handle(self.device)))
        ops._post(self.device)

    def serve(self):
        check(lib().dr_xgmi_serve(C.byref(self.peers), self.handles, self.T, self.batch,
                                  ptr(self.ws), self.wsb, stream_handle(self.device)))
        ops._post(self.device)

    def backward(self, grad_out):
        """grad_out: [B, T*D] gradient of the last forward().

        Requester: the gradient goes into this rank's shared buffer; after a
        barrier every owner pulls, over xGMI, the rows of the (key, slot)
        pairs its inbox still holds from the forward, in (table, source,
        slot) order (dr_xgmi_grad_pull_dev), and queues one IndexedSlices per
        table on its EVs -- the one-hot counterpart of
        ShardedLookup.backward, without staging copies and without a host
        read: the inbox counts stay on the device, table t's slice is the
        fixed region [t*W*B, (t+1)*W*B) with a device count.  Returns the
        per-table (keys, grads, count) -- count a DEVICE int64[1]; the first
        count rows of keys / grads are the slice."""
        from .kv_variable_ops import IndexedSlices
        g = grad_out.contiguous()
        T, D, B, W = self.T, self.dim, self.batch, self.world
        if not g.is_floating_point() or (self._saved is None and tuple(g.shape) != (B, T * D)):
            raise ValueError("grad must be a float [%d, %d]" % (B, T * D))
        if self._saved is not None:
            # per unique key: the sum of its positions' gradients (ascending
            # position, SparseSegment*Grad), laid out at the forward's slots
            # u*T + t for the owners' pulls
            idx, U, koff, bag_offs, bags, combiner = self._saved
            nnz = koff[1]
            if tuple(g.shape) != (bags, T * D):
                raise ValueError("grad must be [%d, %d]" % (bags, T * D))
            gu = self._local.pool_grad(g.float(), idx, koff, U, bag_offs, bags, combiner)
            self.bufs.gin.view(B, T, D)[:nnz].copy_(gu[:T * nnz].view(T, nnz, D).transpose(0, 1))
        elif self.dedup:
            raise RuntimeError("backward() needs a dedup forward() first")
        else:
            self.bufs.gin.copy_(g)
        self._barrier()
        tcap = W * B
        keys = torch.empty(T * tcap, dtype=torch.int64, device=self.device)
        grads = torch.empty((T * tcap, D), dtype=torch.float32, device=self.device)
        counts = torch.empty(T, dtype=torch.int64, device=self.device)
        wsb = lib().dr_xgmi_grad_pull_dev_workspace_size(W, self.bufs.cap)
        ws = workspace(wsb, self.device)
        check(lib().dr_xgmi_grad_pull_dev(C.byref(self.peers), self.gin_ptrs, T, B, D, ptr(keys),
                                          ptr(grads), ptr(counts), ptr(ws), wsb,
                                          stream_handle(self.device)))
        ops._post(self.device)
        self._barrier()          # no peer's next route() may overwrite the inbox before the pull
        out = []
        for t in range(T):
            k, v = keys[t * tcap:(t + 1) * tcap], grads[t * tcap:(t + 1) * tcap]
            n = counts[t:t + 1]
            out.append((k, v, n))
            self.evs[t].pending_grads.append(IndexedSlices(v, k, num_valid=n, unique=False))
        return out

    def forward(self, ids, out_dtype=None, bag_offs=None, combiner="sum"):
        """ids: [T, B] int64 keys (hotness 1) -> [B, T*D] pooled (sum).  bf16
        EVs travel as bf16 rows (half the link bytes); the result is widened
        to fp32 (the reference's cast) unless out_dtype=torch.bfloat16, which
        returns the peer-written bf16 buffer itself.

        Multi-hot: ids [T, nnz] (nnz <= batch), bag_offs = T int32 [bags+1]
        offset arrays -> [bags, T*D] pooled with `combiner` (a new tensor)."""
        if bag_offs is not None:
            return self._forward_bags(ids, bag_offs, combiner, out_dtype)
        if tuple(ids.shape) != (self.T, self.batch) or ids.dtype != torch.int64:
            raise ValueError("ids must be int64 [%d, %d]" % (self.T, self.batch))
        ids = ids.contiguous()
        if self.dedup:
            T, B = self.T, self.batch
            uniq, idx, _, U = ops.unique_grouped(ids.view(-1), self._koff, False)
            self.route(uniq, n_dev=U)
            self._barrier()
            self.serve()
            self._barrier()
            # expand: bag (b, t) reads the staging row of its unique key
            rowsel = (idx.view(T, B).to(torch.int64) * T + self._tcol).view(-1)
            self._saved = (idx, U, self._koff, None, B, "sum")
            return self._local.pool(self.bufs.out.view(B * T, self.dim), rowsel, None,
                                    self._koff, None, B, "sum", out_dtype)
        self._saved = None
        ph = getattr(self, "_ph", None)
        if ph is not None:   # phase timing (bench at N > 1): events between the phases
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            ev[0].record()
        self.route(ids)
        if ph is not None:
            ev[1].record()
        self._barrier()
        if ph is not None:
            ev[2].record()
        self.serve()
        if ph is not None:
            ev[3].record()
        self._barrier()
        if ph is not None:
            ev[4].record()
            ph.append(ev)
        if self.bufs.out.dtype == torch.bfloat16 and out_dtype != torch.bfloat16:
            return self.bufs.out.float()
        return self.bufs.out

    def phase_timing(self, on=True):
        """Record HIP events around each phase of the one-hot forward (route,
        barrier, serve = owner resolve + row writes over xGMI, barrier)."""
        self._ph = [] if on else None

    def phase_summary(self):
        """Mean ms per forward of each phase since phase_timing(True):
        route (requester kernel: (key, slot) pairs into the owners' inboxes),
        wait_route (barrier: the slowest peer's route + the collective's
        latency), serve (owner resolve + every row written to its requester,
        the link-bound phase), wait_serve (barrier after the serve)."""
        ph = getattr(self, "_ph", None) or []
        if not ph:
            return None
        torch.cuda.synchronize()
        names = ("route", "wait_route", "serve", "wait_serve")
        acc = [0.0] * 4
        for ev in ph:
            for i in range(4):
                acc[i] += ev[i].elapsed_time(ev[i + 1])
        n = len(ph)
        self._ph = []
        out = {k: acc[i] / n for i, k in enumerate(names)}
        out["steps"] = n
        return out

    def _forward_bags(self, ids, bag_offs, combiner, out_dtype):
        T, B = self.T, self.batch
        if ids.dim() != 2 or ids.shape[0] != T or ids.dtype != torch.int64 or ids.shape[1] > B:
            raise ValueError("multi-hot ids must be int64 [%d, nnz <= %d]" % (T, B))
        if len(bag_offs) != T or combiner not in ("sum", "mean", "sqrtn"):
            raise ValueError("bag_offs: %d offset arrays; combiner sum / mean / sqrtn" % T)
        bags = int(bag_offs[0].numel()) - 1
        if any(int(o.numel()) - 1 != bags or o.dtype != torch.int32 for o in bag_offs):
            raise ValueError("bag_offs must be int32 [bags+1] with one bag count")
        nnz = int(ids.shape[1])
        koff = [t * nnz for t in range(T + 1)]
        ids = ids.contiguous()
        uniq, idx, _, U = ops.unique_grouped(ids.view(-1), koff, False)
        if nnz == B:
            keys = uniq
        else:   # the route layout is [T, batch]: table t's unique keys at t*batch
            keys = torch.zeros((T, B), dtype=torch.int64, device=self.device)
            if nnz:
                keys[:, :nnz] = uniq.view(T, nnz)
        self.route(keys, n_dev=U)
        self._barrier()
        self.serve()
        self._barrier()
        # expand: position i of table t reads the staging row u*T + t of its
        # unique key u, pooled over its bag in the ALI order
        rowsel = (idx.view(T, nnz).to(torch.int64) * T + self._tcol).view(-1)
        self._saved = (idx, U, koff, list(bag_offs), bags, combiner)
        return self._local.pool(self.bufs.out.view(B * T, self.dim), rowsel, None, koff,
                                bag_offs, bags, combiner, out_dtype)

    def close(self):
        for b in self._bases:
            lib().dr_ipc_close(b)
        self._bases = []
