"""numpy/ctypes front-end of the CPU restatement (deeprec_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the engine under deeprec-1_amd/.
Parity pinning: see deeprec_oracle.c header (golden vectors in tests/golden/).

The composition helpers at the bottom restate DeepRec's Python graph
composition (embedding_ops.py:480-675 embedding_lookup_sparse,
:1209-1344 safe_embedding_lookup_sparse) on top of the C primitives.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdeeprec_oracle.so")
_lib = None

SUM, MEAN, SQRTN = 0, 1, 2
COMBINERS = {"sum": SUM, "mean": MEAN, "sqrtn": SQRTN}


def build():
    src = os.path.join(_HERE, "deeprec_oracle.c")
    if (not os.path.exists(_LIB_PATH)
            or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        p, i64, i32, f32 = C.c_void_p, C.c_int64, C.c_int, C.c_float
        sig = {
            "orc_unique": (i64, [p, i64, p, p, p]),
            "orc_sparse_segment_reduce": (i32, [p, i64, i64, p, p, i64, i64, i32, p, p]),
            "orc_sparse_segment_reduce_grad": (i32, [p, i64, i64, p, p, i64, i64, i32, p]),
            "orc_unsorted_segment_sum": (i32, [p, i64, i64, p, i64, p]),
            "orc_sparse_segment_sum_grad": (i32, [p, i64, i64, p, p, i64, i64, p]),
            "orc_weighted_segment_reduce": (i32, [p, i64, p, p, p, i64, i64, i32, p]),
            "orc_gather": (i32, [p, i64, i64, p, i64, p]),
            "orc_clip_rows": (None, [p, i64, i64, f32]),
            "orc_fused_local_lookup": (i32, [p, i64, i64, p, p, i64, i64, i32, f32, p, p]),
            "orc_fused_local_lookup_grad": (i32, [p, p, i64, i64, p, p, i64, i64, i32, f32, p]),
            "orc_fused_pre_lookup": (i32, [p, i64, p, i64, p, p, p]),
            "orc_fused_post_lookup": (i32, [p, p, i64, i64, i64, i64, i32, f32, p, p]),
            "orc_fused_post_lookup_grad": (i32, [p, p, p, i64, i64, i64, p, i32, f32, p]),
            "orc_weighted_segment_grad": (i32, [p, i64, i64, p, p, p, i64, i64, i32, p]),
            "orc_clip_by_norm_grad": (None, [p, p, i64, i64, f32]),
            "orc_ev_create": (p, [i64, p, i64, i64, i64, f32, i32]),
            "orc_ev_create_slot": (p, [p, i32, p]),
            "orc_ev_free": (None, [p]),
            "orc_ev_set_bf16": (None, [p]),
            "orc_bf16_round": (f32, [f32]),
            "orc_ev_gather": (i32, [p, p, i64, p, p, p]),
            "orc_ev_import": (i32, [p, p, i64, p, p, p, i64, i64, i64]),
            "orc_ev_size": (i64, [p]),
            "orc_ev_export": (i64, [p, p, p, p, p]),
            "orc_ev_freq": (i64, [p, i64]),
            "orc_ev_version": (i64, [p, i64]),
            "orc_ev_has_row": (i32, [p, i64]),
            "orc_ev_apply_sgd": (i32, [p, f32, p, p, i64, i64]),
            "orc_ev_apply_adagrad": (i32, [p, p, f32, p, p, i64, i64]),
            "orc_ev_apply_adam": (i32, [p, p, p, f32, f32, f32, f32, f32, f32, p, p, i64, i64]),
            "orc_ev_apply_adam_async": (i32, [p, p, p, f32, f32, f32, f32, f32, f32, i32, p, p,
                                              i64, i64]),
            "orc_ev_apply_adagrad_decay": (i32, [p, p, p, f32, i64, f32, f32, p, p, i64, i64]),
            "orc_ev_apply_ftrl": (i32, [p, p, p, f32, f32, f32, f32, f32, p, p, i64, i64]),
            "orc_dense_apply_sgd": (i32, [p, i64, f32, p, p, i64]),
            "orc_dense_apply_adagrad": (i32, [p, p, i64, f32, p, p, i64]),
            "orc_fm2": (None, [p, i64, i64, i64, p]),
            "orc_dot_interaction": (None, [p, i64, i64, i64, p]),
            "orc_crossnet_layer": (None, [p, p, p, p, i64, i64, p]),
            "orc_fasthash64": (C.c_uint64, [i64, C.c_uint64]),
            "orc_fingerprint64": (C.c_uint64, [p, C.c_uint64]),
            "orc_string_to_hash_bucket_fast": (None, [p, p, i64, i64, p]),
            "orc_pipeline_ev_lookup_sparse": (i32, [p, p, i64, p, i64, i32, i32, p]),
            "orc_pipeline_dense_lookup_sparse": (i32, [p, i64, p, i64, p, i64, i32, i32, p]),
            "orc_pool_create": (p, [i32]),
            "orc_pool_threads": (i32, [p]),
            "orc_pool_free": (None, [p]),
            "orc_unique_parallel": (i64, [p, p, i64, p, p]),
            "orc_pipeline_ev_lookup_sparse_pool": (i32, [p, p, p, i64, p, i64, i32, i32, p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise OracleError("%s failed with status %d" % (what, rc))


# --------------------------------------------------------------------------
# primitives
# --------------------------------------------------------------------------
def unique(x, with_counts=False):
    x = np.ascontiguousarray(x, dtype=np.int64)
    y = np.empty_like(x)
    idx = np.empty(x.shape[0], np.int32)
    cnt = np.empty(x.shape[0], np.int32)
    u = lib().orc_unique(_p(x), x.shape[0], _p(y), _p(idx), _p(cnt))
    if with_counts:
        return y[:u].copy(), idx, cnt[:u].copy()
    return y[:u].copy(), idx


class Pool(object):
    """The persistent worker pool (orc_pool_create): TF's CPU worker threads."""

    def __init__(self, threads):
        self._h = lib().orc_pool_create(int(threads))
        if not self._h:
            raise OracleError("orc_pool_create failed")
        self.threads = int(lib().orc_pool_threads(self._h))

    def close(self):
        if self._h:
            lib().orc_pool_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def unique_parallel(x, pool):
    """ParallelComputeV1 (unique_ali_op_util.h:226-445) on the pool's threads."""
    x = np.ascontiguousarray(x, dtype=np.int64)
    y = np.empty_like(x)
    idx = np.empty(x.shape[0], np.int32)
    u = lib().orc_unique_parallel(pool._h, _p(x), x.shape[0], _p(y), _p(idx))
    return y[:u].copy(), idx


def sparse_segment_reduce(data, idx, seg, combiner="sum", num_segments=-1):
    data = np.ascontiguousarray(data, np.float32)
    idx = np.ascontiguousarray(idx, np.int32)
    seg = np.ascontiguousarray(seg, np.int32)
    D = data.shape[1]
    rows = C.c_int64(0)
    _check(lib().orc_sparse_segment_reduce(_p(data), data.shape[0], D, _p(idx), _p(seg),
                                           idx.shape[0], num_segments, COMBINERS[combiner],
                                           None, C.byref(rows)), "sparse_segment_reduce")
    out = np.empty((rows.value, D), np.float32)
    _check(lib().orc_sparse_segment_reduce(_p(data), data.shape[0], D, _p(idx), _p(seg),
                                           idx.shape[0], num_segments, COMBINERS[combiner],
                                           _p(out), None), "sparse_segment_reduce")
    return out


def sparse_segment_reduce_grad(grad, idx, seg, out_rows, combiner):
    grad = np.ascontiguousarray(grad, np.float32)
    idx = np.ascontiguousarray(idx, np.int32)
    seg = np.ascontiguousarray(seg, np.int32)
    D = grad.shape[1]
    out = np.empty((out_rows, D), np.float32)
    if combiner == "sum":
        _check(lib().orc_sparse_segment_sum_grad(_p(grad), grad.shape[0], D, _p(idx), _p(seg),
                                                 idx.shape[0], out_rows, _p(out)), "segment_sum_grad")
    else:
        _check(lib().orc_sparse_segment_reduce_grad(_p(grad), grad.shape[0], D, _p(idx), _p(seg),
                                                    idx.shape[0], out_rows,
                                                    1 if combiner == "sqrtn" else 0, _p(out)),
               "sparse_segment_reduce_grad")
    return out


def unsorted_segment_sum(data, seg, num_segments):
    data = np.ascontiguousarray(data, np.float32)
    seg = np.ascontiguousarray(seg, np.int32)
    D = data.shape[1]
    out = np.empty((num_segments, D), np.float32)
    _check(lib().orc_unsorted_segment_sum(_p(data), data.shape[0], D, _p(seg), num_segments,
                                          _p(out)), "unsorted_segment_sum")
    return out


def gather(table, idx):
    table = np.ascontiguousarray(table, np.float32)
    idx = np.ascontiguousarray(idx, np.int64)
    out = np.empty((idx.shape[0], table.shape[1]), np.float32)
    _check(lib().orc_gather(_p(table), table.shape[0], table.shape[1], _p(idx), idx.shape[0],
                            _p(out)), "gather")
    return out


def clip_rows(rows, max_norm):
    rows = np.array(rows, np.float32, copy=True)
    lib().orc_clip_rows(_p(rows), rows.shape[0], rows.shape[1], max_norm)
    return rows


def fused_local_lookup(table, values, row_ids, batch, combiner, max_norm=-1.0):
    table = np.ascontiguousarray(table, np.float32)
    values = np.ascontiguousarray(values, np.int64)
    row_ids = np.ascontiguousarray(row_ids, np.int64)
    out = np.empty((batch, table.shape[1]), np.float32)
    off = np.empty(batch, np.int32)
    _check(lib().orc_fused_local_lookup(_p(table), table.shape[0], table.shape[1], _p(values),
                                        _p(row_ids), values.shape[0], batch,
                                        COMBINERS[combiner], max_norm, _p(out), _p(off)),
           "fused_local_lookup")
    return out, off


def fused_local_lookup_grad(top_grad, table, values, offsets, combiner, max_norm=-1.0):
    top_grad = np.ascontiguousarray(top_grad, np.float32)
    table = np.ascontiguousarray(table, np.float32)
    values = np.ascontiguousarray(values, np.int64)
    offsets = np.ascontiguousarray(offsets, np.int32)
    out = np.empty((values.shape[0], table.shape[1]), np.float32)
    _check(lib().orc_fused_local_lookup_grad(_p(top_grad), _p(table), table.shape[0],
                                             table.shape[1], _p(values), _p(offsets),
                                             values.shape[0], offsets.shape[0],
                                             COMBINERS[combiner], max_norm, _p(out)),
           "fused_local_lookup_grad")
    return out


def fused_pre_lookup(values, part_rows):
    values = np.ascontiguousarray(values, np.int64)
    part_rows = np.ascontiguousarray(part_rows, np.int64)
    ov = np.empty_like(values)
    op = np.empty_like(values)
    sizes = np.empty(part_rows.shape[0], np.int64)
    _check(lib().orc_fused_pre_lookup(_p(values), values.shape[0], _p(part_rows),
                                      part_rows.shape[0], _p(ov), _p(op), _p(sizes)),
           "fused_pre_lookup")
    res, k = [], 0
    for s in sizes:
        res.append((ov[k:k + s].copy(), op[k:k + s].copy()))
        k += s
    return res


def fused_post_lookup(shards, indices, batch, cols, combiner, max_norm=-1.0):
    """FusedEmbeddingSparsePostLookUp over partitions given as lists of
    [n_p, D] shards and [n_p, 2] indices -> (emb [B, D], feature_nums [B])."""
    D = np.asarray(shards[0]).shape[1]
    emb = np.ascontiguousarray(np.concatenate([np.asarray(s, np.float32).reshape(-1, D)
                                               for s in shards]), np.float32)
    ind = np.ascontiguousarray(np.concatenate([np.asarray(i, np.int64).reshape(-1, 2)
                                               for i in indices]), np.int64)
    out = np.empty((batch, D), np.float32)
    fnum = np.empty(batch, np.int32)
    _check(lib().orc_fused_post_lookup(_p(emb), _p(ind), emb.shape[0], batch, cols, D,
                                       COMBINERS[combiner], max_norm, _p(out), _p(fnum)),
           "fused_post_lookup")
    return out, fnum


def fused_post_lookup_grad(top_grad, shards, indices, feature_nums, combiner, max_norm=-1.0):
    top = np.ascontiguousarray(top_grad, np.float32)
    B, D = top.shape
    fn = np.ascontiguousarray(feature_nums, np.int32)
    outs = []
    for s, i in zip(shards, indices):
        s = np.ascontiguousarray(s, np.float32).reshape(-1, D)
        i = np.ascontiguousarray(i, np.int64).reshape(-1, 2)
        o = np.empty_like(s)
        _check(lib().orc_fused_post_lookup_grad(_p(top), _p(s), _p(i), s.shape[0], B, D, _p(fn),
                                                COMBINERS[combiner], max_norm, _p(o)),
               "fused_post_lookup_grad")
        outs.append(o)
    return outs


def weighted_segment_grad(g, idx, w, seg, num_unique, combiner):
    g = np.ascontiguousarray(g, np.float32)
    B, D = g.shape
    idx = np.ascontiguousarray(idx, np.int32)
    w = np.ascontiguousarray(w, np.float32)
    seg = np.ascontiguousarray(seg, np.int32)
    out = np.empty((num_unique, D), np.float32)
    _check(lib().orc_weighted_segment_grad(_p(g), B, D, _p(idx), _p(w), _p(seg), idx.shape[0],
                                           num_unique, COMBINERS[combiner], _p(out)),
           "weighted_segment_grad")
    return out


def clip_by_norm_grad(rows, grad, max_norm):
    rows = np.ascontiguousarray(rows, np.float32)
    g = np.array(grad, np.float32, copy=True)
    lib().orc_clip_by_norm_grad(_p(rows), _p(g), g.shape[0], g.shape[1], max_norm)
    return g


def fasthash64(key, seed):
    return lib().orc_fasthash64(int(key), int(seed))


def fingerprint64(data):
    """farmhash Fingerprint64 of a bytes object (fingerprint.h:80-88)."""
    b = np.frombuffer(bytes(data) + b"\0", np.uint8)
    return int(lib().orc_fingerprint64(_p(b), len(data)))


def strings_to_arrays(strings):
    """(offsets int64 [n+1], bytes uint8) layout of a list of str/bytes."""
    enc = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    off = np.zeros(len(enc) + 1, np.int64)
    off[1:] = np.cumsum([len(e) for e in enc])
    return off, np.frombuffer(b"".join(enc) + b"\0", np.uint8)


def string_to_hash_bucket_fast(strings, num_buckets):
    """StringToHashBucketFast (string_to_hash_bucket_ali_op.h:33-63)."""
    off, buf = strings_to_arrays(strings)
    out = np.empty(len(strings), np.int64)
    lib().orc_string_to_hash_bucket_fast(_p(buf), _p(off), len(strings), int(num_buckets),
                                         _p(out))
    return out


def dump_embedding_values(keys, values, versions, freqs):
    """DumpEmbeddingValues (kv_variable_ops.h:148-265): a snapshot's entries
    grouped into 1000 sub-partitions by key % 1000 with C++ remainder
    semantics (negative keys fall in no sub-partition and are dropped),
    snapshot order kept inside a sub-partition.  versions / freqs may be
    empty (steps_to_live == 0 / no filter).  Returns (partition_offset int32
    [1001], keys, values, versions, freqs)."""
    keys = np.asarray(keys, np.int64)
    parts = [[] for _ in range(1000)]
    for i, k in enumerate(keys.tolist()):
        if k >= 0:
            parts[k % 1000].append(i)
    order = np.array([i for p in parts for i in p], np.int64)
    offs = np.zeros(1001, np.int32)
    offs[1:] = np.cumsum([len(p) for p in parts])
    pick = lambda a: (np.asarray(a)[order] if len(a) else np.asarray(a))
    return offs, keys[order], np.asarray(values)[order], pick(versions), pick(freqs)


def fm2(emb):
    emb = np.ascontiguousarray(emb, np.float32)
    B, F, D = emb.shape
    out = np.empty((B, D), np.float32)
    lib().orc_fm2(_p(emb), B, F, D, _p(out))
    return out


def dot_interaction(x):
    x = np.ascontiguousarray(x, np.float32)
    B, F, D = x.shape
    out = np.empty((B, F * (F - 1) // 2), np.float32)
    lib().orc_dot_interaction(_p(x), B, F, D, _p(out))
    return out


def crossnet_layer(x0, xl, W, b):
    x0 = np.ascontiguousarray(x0, np.float32)
    xl = np.ascontiguousarray(xl, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    b = None if b is None else np.ascontiguousarray(b, np.float32)
    out = np.empty_like(xl)
    lib().orc_crossnet_layer(_p(x0), _p(xl), _p(W), _p(b), xl.shape[0], xl.shape[1], _p(out))
    return out


# --------------------------------------------------------------------------
# EmbeddingVariable
# --------------------------------------------------------------------------
def bf16_bits(x):
    """fp32 -> bf16 bit patterns (uint16): round to nearest even, NaN ->
    0x7FC0 -- torch's c10::BFloat16 conversion, restated."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32)
    nan = (u & np.uint32(0x7FFFFFFF)) > np.uint32(0x7F800000)
    with np.errstate(over="ignore"):
        r = ((u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16))
    return np.where(nan, np.uint32(0x7FC0), r).astype(np.uint16)


def bf16_widen(h):
    """bf16 bit patterns (uint16) -> fp32."""
    return (np.asarray(h, np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def bf16_round(x):
    """fp32 -> the nearest-even bf16 value, as fp32."""
    return bf16_widen(bf16_bits(x))


class EV(object):
    """CPU EmbeddingVariable (embedding_var.h) -- primary or slot.

    bf16=True: a bf16 EV (build-defined, the engine's value_bits 16): the
    default row is rounded to bf16, every apply computes in fp32 on the
    stored (bf16-valued) rows and rounds the updated row once; rows are kept
    as fp32 arrays holding bf16 values, so gather / export return them
    widened (bf16_bits() gives the bit patterns)."""

    def __init__(self, dim, default_row, filter_freq=0, steps_to_live=0,
                 max_element_size=0, false_positive_probability=-1.0,
                 counter_bits=64, _handle=None, _primary=None, bf16=False):
        self.dim = dim
        self._primary = _primary
        self.filter_freq = filter_freq
        self.bf16 = bool(bf16)
        if _handle is not None:
            self._h = _handle
        else:
            d = np.ascontiguousarray(np.broadcast_to(np.asarray(default_row, np.float32), (dim,)))
            self._h = lib().orc_ev_create(dim, _p(d), filter_freq, steps_to_live,
                                          max_element_size, false_positive_probability,
                                          counter_bits)
            if self.bf16:
                lib().orc_ev_set_bf16(self._h)

    def create_slot(self, slot_index, default_row):
        d = np.ascontiguousarray(np.broadcast_to(np.asarray(default_row, np.float32),
                                                 (self.dim,)))
        h = lib().orc_ev_create_slot(self._h, slot_index, _p(d))
        if not h:
            raise OracleError("bad slot index")
        return EV(self.dim, None, _handle=h, _primary=self)

    def __del__(self):
        try:
            if self._h:
                lib().orc_ev_free(self._h)
                self._h = None
        except Exception:
            pass

    def gather(self, keys, defaults=None, counts=None):
        keys = np.ascontiguousarray(keys, np.int64)
        n = keys.shape[0]
        if defaults is not None:
            defaults = np.ascontiguousarray(
                np.broadcast_to(np.asarray(defaults, np.float32), (n, self.dim)))
        if counts is not None:
            counts = np.ascontiguousarray(counts, np.int32)
        out = np.empty((n, self.dim), np.float32)
        _check(lib().orc_ev_gather(self._h, _p(keys), n, _p(defaults), _p(counts), _p(out)),
               "ev_gather")
        return out

    def insert(self, keys, values, versions=None, freqs=None, partition_id=0,
               partition_num=0, bucket_num=1000):
        keys = np.ascontiguousarray(keys, np.int64)
        values = np.ascontiguousarray(values, np.float32).reshape(keys.shape[0], self.dim)
        versions = None if versions is None else np.ascontiguousarray(versions, np.int64)
        freqs = None if freqs is None else np.ascontiguousarray(freqs, np.int64)
        _check(lib().orc_ev_import(self._h, _p(keys), keys.shape[0], _p(values), _p(versions),
                                   _p(freqs), bucket_num, partition_id, partition_num),
               "ev_import")

    def size(self):
        return lib().orc_ev_size(self._h)

    def export(self):
        n = self.size()
        keys = np.empty(n, np.int64)
        vals = np.empty((n, self.dim), np.float32)
        vers = np.empty(n, np.int64)
        frqs = np.empty(n, np.int64)
        m = lib().orc_ev_export(self._h, _p(keys), _p(vals), _p(vers), _p(frqs))
        return keys[:m], vals[:m], vers[:m], frqs[:m]

    def freq(self, key):
        return lib().orc_ev_freq(self._h, int(key))

    def version(self, key):
        return lib().orc_ev_version(self._h, int(key))

    def has_row(self, key):
        return bool(lib().orc_ev_has_row(self._h, int(key)))

    def apply_sgd(self, lr, grad, keys, gs=-1):
        grad = np.ascontiguousarray(grad, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        _check(lib().orc_ev_apply_sgd(self._h, lr, _p(grad), _p(keys), keys.shape[0], gs), "sgd")

    def apply_adagrad(self, accum, lr, grad, keys, gs=-1):
        grad = np.ascontiguousarray(grad, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        _check(lib().orc_ev_apply_adagrad(self._h, accum._h, lr, _p(grad), _p(keys),
                                          keys.shape[0], gs), "adagrad")

    def apply_adam(self, m, v, beta1_power, beta2_power, lr, beta1, beta2, eps, grad, keys,
                   gs=-1):
        grad = np.ascontiguousarray(grad, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        _check(lib().orc_ev_apply_adam(self._h, m._h, v._h, beta1_power, beta2_power, lr,
                                       beta1, beta2, eps, _p(grad), _p(keys), keys.shape[0],
                                       gs), "adam")

    def apply_adam_async(self, m, v, beta1_power, beta2_power, lr, beta1, beta2, eps, grad,
                         keys, rmsprop=False, gs=-1):
        grad = np.ascontiguousarray(grad, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        _check(lib().orc_ev_apply_adam_async(self._h, m._h, v._h, beta1_power, beta2_power, lr,
                                             beta1, beta2, eps, 1 if rmsprop else 0, _p(grad),
                                             _p(keys), keys.shape[0], gs), "adam_async")

    def apply_adagrad_decay(self, accum, power, lr, decay_step, decay_rate, decay_baseline,
                            grad, keys, gs):
        grad = np.ascontiguousarray(grad, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        _check(lib().orc_ev_apply_adagrad_decay(self._h, accum._h, power._h, lr, decay_step,
                                                decay_rate, decay_baseline, _p(grad), _p(keys),
                                                keys.shape[0], gs), "adagrad_decay")

    def apply_ftrl(self, accum, linear, lr, l1, l2, lr_power, l2_shrinkage, grad, keys, gs=-1):
        grad = np.ascontiguousarray(grad, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        _check(lib().orc_ev_apply_ftrl(self._h, accum._h, linear._h, lr, l1, l2, lr_power,
                                       l2_shrinkage, _p(grad), _p(keys), keys.shape[0], gs),
               "ftrl")


def dense_apply_sgd(table, lr, grad, idx):
    grad = np.ascontiguousarray(grad, np.float32)
    idx = np.ascontiguousarray(idx, np.int64)
    lib().orc_dense_apply_sgd(_p(table), table.shape[1], lr, _p(grad), _p(idx), idx.shape[0])


def dense_apply_adagrad(table, accum, lr, grad, idx):
    grad = np.ascontiguousarray(grad, np.float32)
    idx = np.ascontiguousarray(idx, np.int64)
    lib().orc_dense_apply_adagrad(_p(table), _p(accum), table.shape[1], lr, _p(grad), _p(idx),
                                  idx.shape[0])


# --------------------------------------------------------------------------
# Python composition (embedding_ops.py)
# --------------------------------------------------------------------------
def prune_and_fill(indices, values, dense_shape, weights=None, combiner="mean", default_id=None,
                   prune=True):
    """safe_embedding_lookup_sparse steps 1-3 (embedding_ops.py:1289-1310).

    indices [nnz,2] int64 (any order), values [nnz] int64.
    Returns (indices, values, weights, is_row_empty)."""
    indices = np.asarray(indices, np.int64).reshape(-1, 2)
    values = np.asarray(values, np.int64)
    w = None if weights is None else np.asarray(weights, np.float32)
    if prune:
        keep = values >= 0                                   # _prune_invalid_ids :1555
        if w is not None and combiner != "sum":
            keep = keep & (w > 0)                            # _prune_invalid_weights
        indices, values = indices[keep], values[keep]
        if w is not None:
            w = w[keep]
    B = int(dense_shape[0])
    indices, values, empty, rev = sparse_fill_empty_rows(indices, values, B, default_id or 0)
    if w is not None:
        w = _fill_like(rev, w, indices.shape[0], np.float32(1.0))   # fill weights with 1.0
    return indices, values, w, empty


def sparse_fill_empty_rows(indices, values, dense_rows, default_value):
    """SparseFillEmptyRows (core/kernels/sparse_fill_empty_rows_op_util.h:
    17-128), serial: entry i goes to scratch[row-1] + filled_count[row]++
    (rows ascending, input order inside a row); an empty row gets one entry
    [row, 0, ...] = default_value.  Returns (indices, values,
    empty_row_indicator, reverse_index_map)."""
    indices = np.asarray(indices, np.int64)
    rank = indices.shape[1] if indices.ndim == 2 else 2
    indices = indices.reshape(-1, rank)
    values = np.asarray(values)
    n = indices.shape[0]
    scratch = np.zeros(dense_rows, np.int64)
    for i in range(n):
        r = int(indices[i, 0])
        if not 0 <= r < dense_rows:
            raise OracleError("indices(%d, 0) is invalid: %d >= %d" % (i, r, dense_rows))
        scratch[r] += 1
    empty = scratch == 0
    scratch = np.cumsum(np.maximum(scratch, 1))
    n_full = int(scratch[-1]) if dense_rows else 0
    out_i = np.zeros((n_full, rank), np.int64)
    out_v = np.full(n_full, default_value, values.dtype if n else np.asarray(default_value).dtype)
    filled = np.zeros(dense_rows, np.int64)
    rev = np.zeros(n, np.int64)
    for i in range(n):
        r = int(indices[i, 0])
        o = (0 if r == 0 else scratch[r - 1]) + filled[r]
        filled[r] += 1
        out_i[o] = indices[i]
        out_v[o] = values[i]
        rev[i] = o
    for r in range(dense_rows):
        if filled[r] == 0:
            out_i[0 if r == 0 else scratch[r - 1], 0] = r
    return out_i, out_v, empty, rev


def _fill_like(rev, vals, n_full, default):
    out = np.full(n_full, default, np.asarray(vals).dtype)
    out[rev] = vals
    return out


def embedding_lookup_sparse(params, indices, values, batch, weights=None, combiner="mean",
                            max_norm=None):
    """embedding_lookup_sparse (embedding_ops.py:480-675) for one table.

    params: numpy [R,D] dense table, or an EV."""
    seg = np.asarray(indices, np.int64).reshape(-1, 2)[:, 0].astype(np.int32)
    if isinstance(params, EV):
        uids, idx, counts = unique(values, with_counts=True)
        emb = params.gather(uids, None, counts if _ev_filter_on(params) else None)
    else:
        uids, idx = unique(values)
        emb = gather(params, uids)
    if max_norm is not None:
        emb = clip_rows(emb, max_norm)
    if weights is None:
        # (a bf16 EV pools its widened values into fp32: the reference casts
        # bf16 embeddings to float32 first, embedding_ops.py:606-607)
        return sparse_segment_reduce(emb, idx, seg, combiner, num_segments=batch)
    D = emb.shape[1]
    out = np.empty((batch, D), np.float32)
    w = np.ascontiguousarray(weights, np.float32)
    _check(lib().orc_weighted_segment_reduce(_p(emb), D, _p(np.ascontiguousarray(idx)), _p(w),
                                             _p(np.ascontiguousarray(seg)), idx.shape[0], batch,
                                             COMBINERS[combiner], _p(out)), "weighted")
    return out


def embedding_lookup_sparse_grad(params, indices, values, batch, top_grad, weights=None,
                                 combiner="mean", max_norm=None):
    """Gradient of embedding_lookup_sparse w.r.t. the looked-up rows, as
    (unique ids in first-occurrence order, grad [U, D]): the reference's
    backward (SparseSegment*Grad, or the weighted composition's chain, then
    clip_by_norm's when max_norm is set).  Call after the forward (EV rows
    exist)."""
    seg = np.asarray(indices, np.int64).reshape(-1, 2)[:, 0].astype(np.int32)
    uids, idx = unique(values)
    U = uids.shape[0]
    g = np.ascontiguousarray(top_grad, np.float32)
    if weights is None:
        gu = sparse_segment_reduce_grad(g, idx, seg, U, combiner)
    else:
        gu = weighted_segment_grad(g, idx, weights, seg, U, combiner)
    if max_norm is not None:
        rows = params.gather(uids) if isinstance(params, EV) else gather(params, uids)
        gu = clip_by_norm_grad(rows, gu, max_norm)
    return uids, gu


def _ev_filter_on(ev):
    return getattr(ev, "filter_freq", 0) != 0


def safe_embedding_lookup_sparse(params, indices, values, dense_shape, weights=None,
                                 combiner="mean", default_id=None, max_norm=None, prune=True):
    """safe_embedding_lookup_sparse (embedding_ops.py:1209-1344), 2-D ids."""
    ind, val, w, empty = prune_and_fill(indices, values, dense_shape, weights, combiner,
                                        default_id, prune)
    res = embedding_lookup_sparse(params, ind, val, int(dense_shape[0]), w, combiner, max_norm)
    if default_id is None:
        res[empty] = 0.0
    return res


def synth_rows(seed, keys, D):
    """synth(seed, key, col) of the engine's synthetic tables (dr_common.h:
    SplitMix64 of (seed, row, col) -> uniform [-1, 1)), rows for `keys`."""
    M = np.uint64
    keys = np.asarray(keys, np.int64)
    with np.errstate(over="ignore"):
        z = (M(seed) * M(0x9E3779B97F4A7C15) + keys.astype(np.uint64)[:, None] * M(0xBF58476D1CE4E5B9)
             + np.arange(D, dtype=np.uint64)[None, :] * M(0x94D049BB133111EB))
        z ^= z >> M(30)
        z *= M(0xBF58476D1CE4E5B9)
        z ^= z >> M(27)
        z *= M(0x94D049BB133111EB)
        z ^= z >> M(31)
    hi = (z >> M(32)).astype(np.uint32).view(np.int32)
    return hi.astype(np.float32) * np.float32(1.0 / 2147483648.0)
