"""EmbeddingVariable -- the GPU-resident counterpart of DeepRec's
python/ops/kv_variable_ops.py:44-765 (class EmbeddingVariable) and
python/ops/variables.py:238-330 (EmbeddingVariableOption / CounterFilter /
CBFFilter).  Storage and the insert-on-miss lookup run in HIP kernels through
the C ABI (dr_ev_*); this module only holds the handle and the Python-level
argument semantics.
"""
import ctypes as C
import atexit
import collections
import threading

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle, workspace


# ---------------------------------------------------------------------------
# Options (variables.py:238-330)
# ---------------------------------------------------------------------------
class CounterFilter(object):
    def __init__(self, filter_freq=0):
        self.filter_freq = filter_freq


class CBFFilter(object):
    """Counting Bloom filter admission (embedding_filter.h:27-286)."""

    def __init__(self, filter_freq=0, max_element_size=0, false_positive_probability=-1.0,
                 counter_type=torch.int64):
        self.filter_freq = filter_freq
        self.max_element_size = max_element_size
        self.false_positive_probability = false_positive_probability
        bits = {torch.uint8: 8, torch.int8: 8, torch.int16: 16, torch.int32: 32,
                torch.int64: 64}
        self.counter_bits = bits.get(counter_type, 64) if not isinstance(counter_type, int) \
            else counter_type


class GlobalStepEvict(object):
    def __init__(self, steps_to_live=None):
        self.steps_to_live = steps_to_live


class EmbeddingVariableOption(object):
    def __init__(self, ht_type="", ht_partition_num=1000, evict_option=None, filter_option=None):
        self.ht_type = ht_type
        self.ht_partition_num = ht_partition_num
        self.evict_option = evict_option
        self.filter_option = filter_option


def _default_row(initializer, dim, device, dtype=torch.float32):
    """EV default_value_ (InitializeKvVariableOp input 2, a [dim] tensor)."""
    if initializer is None:
        initializer = 0.0
    if callable(initializer):
        v = initializer((dim,))
        v = torch.as_tensor(v, dtype=dtype).reshape(dim)
    else:
        v = torch.full((dim,), float(initializer), dtype=dtype)
    return v.cpu().contiguous()


# Handles whose last Python reference died.  Releasing one frees device
# memory (hipFree) and synchronises, which breaks a hipGraph capture in
# torch's default global mode if ANY stream of the process is capturing --
# and __del__ runs on whatever thread triggers the collection, whose own
# current stream says nothing about another thread's capture.  So __del__
# never releases: it queues the handle, and the queue is flushed at points
# where the library itself runs uncaptured host work (EV creation, the end
# of an optimizer's apply_gradients) and by flush_releases() -- and only when
# no capture is open anywhere in the process: torch.cuda.CUDAGraph's
# capture_begin / capture_end are counted process-wide (_CAPTURES), on every
# thread.  At interpreter exit the queue is dropped (the process's device
# memory goes with it).
# __del__ appends without the lock (deque.append is atomic): a collection
# that runs inside the locked flush below, on the same thread, must not block
# on the lock that thread holds.  The lock is reentrant for the same reason.
_DEFERRED = collections.deque()
_DEFERRED_LOCK = threading.RLock()
_CAPTURES = [0]     # torch graph captures open in this process (any thread)


def _install_capture_counter():
    G = getattr(torch.cuda, "CUDAGraph", None)
    if G is None or getattr(G, "_dr_counted", False):
        return
    begin, end = G.capture_begin, G.capture_end

    def capture_begin(self, *a, **k):
        with _DEFERRED_LOCK:
            _CAPTURES[0] += 1
        try:
            return begin(self, *a, **k)
        except BaseException:
            with _DEFERRED_LOCK:
                _CAPTURES[0] -= 1
            raise

    def capture_end(self, *a, **k):
        try:
            return end(self, *a, **k)
        finally:
            with _DEFERRED_LOCK:
                _CAPTURES[0] -= 1

    G.capture_begin, G.capture_end, G._dr_counted = capture_begin, capture_end, True


_install_capture_counter()


def _capturing():
    """A capture is open on this thread's stream or on any thread (torch)."""
    if _CAPTURES[0] > 0:
        return True
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _flush_deferred_releases():
    if not _DEFERRED:
        return
    # the lock is held across the frees: a capture_begin on another thread
    # waits for them instead of starting in between
    with _DEFERRED_LOCK:
        if _CAPTURES[0] > 0:
            return
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return
        while True:
            try:
                h = _DEFERRED.popleft()
            except IndexError:
                break
            if isinstance(h, tuple):      # (destroy entry name, handle): engines
                getattr(lib(), h[0])(h[1])
            else:
                lib().dr_ev_release(h)


def flush_releases():
    """Release the device memory of every EmbeddingVariable that has been
    garbage-collected (call outside any hipGraph capture)."""
    if _capturing():
        raise RuntimeError("flush_releases() inside a stream capture")
    _flush_deferred_releases()


def _release_handle(h):
    _DEFERRED.append(h)   # lock-free: may run from GC inside the flush


def _release_engine(destroy, h):
    """Queue an engine handle (e.g. dr_sharded_destroy, which synchronises the
    device) on the same capture-safe deferred path as EV handles."""
    _DEFERRED.append((destroy, h))


atexit.register(lambda: _DEFERRED.clear())   # dropped: the process's device memory goes too


_KEY_DTYPES = (torch.int64, torch.int32)
# bfloat16: a build-defined bf16 EV (BASELINE configs[4]; the reference
# registers float and double): bf16 value rows, fp32 optimizer slots
_VALUE_DTYPES = (torch.float32, torch.float64, torch.bfloat16)


class IndexedSlices(object):
    """values [N, D] for rows `indices` [N] (tf.IndexedSlices).

    A lookup backward may hand the values over BY ADDRESS instead
    (dr_pool_grad_rows_grouped): grad_ptr [N] int64 holds the address of
    each row (bit 0: use as 0.0f + g) and `keep` the buffers they point into.
    The EV optimizers read such rows in place (dr_ev_apply_grouped_ptr);
    `values` materialises them on first access (dr_rows_from_ptr)."""

    def __init__(self, values, indices, num_valid=None, unique=False, grad_ptr=None, dim=None,
                 keep=(), rows=None):
        self._values = values
        self.indices = indices
        # rows [N] int64: the EV row each index was resolved to by the forward
        # (a row-grouped backward); lets SGD skip the key-table probe
        self.rows = rows
        self.num_valid = num_valid  # optional device int64[1] (<= N)
        self.unique = unique        # indices known distinct (a lookup's backward)
        self.grad_ptr = grad_ptr
        self.dim = dim
        self._keep = keep

    @property
    def values(self):
        if self._values is None and self.grad_ptr is not None:
            n = self.grad_ptr.numel()
            out = torch.empty((n, self.dim), dtype=torch.float32, device=self.grad_ptr.device)
            _lib.check(_lib.lib().dr_rows_from_ptr(
                _lib.ptr(self.grad_ptr), n, _lib.ptr(self.num_valid), self.dim, _lib.ptr(out),
                _lib.stream_handle(self.grad_ptr.device)))
            self._values = out
        return self._values

    @values.setter
    def values(self, v):
        self._values = v
        self.grad_ptr = None
        self._keep = ()


class PendingRowSlices(IndexedSlices):
    """Table t's gradient of a row-grouped lookup backward, not yet formed.

    An SGD apply_gradients over every variable of the group runs the
    backward fused with the update (dr_ev_pool_grad_rows_apply_sgd: the same
    run sums and v -= lr * g roundings, no IndexedSlices in between).  Any
    other use -- indices, values, rows, num_valid, grad_ptr -- first forms the
    IndexedSlices exactly as the eager backward (dr_pool_grad_rows_grouped_ex)
    would have, and the object is an ordinary IndexedSlices from then on."""

    _LAZY = ("indices", "rows", "num_valid", "grad_ptr", "_values", "_keep")

    def __init__(self, pending, t, dim):
        self._pending = pending
        self._t = t
        self.unique = True
        self.dim = dim

    def __getattr__(self, name):
        # only reached for attributes not yet in __dict__
        if name in PendingRowSlices._LAZY:
            real = self._pending.materialize()[self._t]
            for k in PendingRowSlices._LAZY:
                self.__dict__.setdefault(k, getattr(real, k))
            return self.__dict__[name]
        raise AttributeError(name)

    def fusable(self):
        return "indices" not in self.__dict__ and self._pending.fusable()

    @property
    def values(self):
        return IndexedSlices.values.fget(self)

    @values.setter
    def values(self, v):
        self.__getattr__("indices")   # formed first: the indices stay valid
        IndexedSlices.values.fset(self, v)


class EmbeddingVariable(object):
    """Hash-keyed embedding table resident in HBM.

    initializer: float constant, or callable(shape) -> tensor (e.g.
    lambda s: torch.randn(s) * 0.01).  As in the reference, a callable
    initializer draws a fresh [N, D] default block per sparse_read call
    (kv_variable_ops.py:651-654); a constant uses the EV's own default row.
    """

    def __init__(self, name, embedding_dim, initializer=None, steps_to_live=0, ev_option=None,
                 capacity=1 << 16, device=None, _primary=None, _slot_index=0,
                 l2_weight_threshold=-1.0, key_dtype=torch.int64, value_dtype=torch.float32):
        _lib.require_gpu()
        if key_dtype not in _KEY_DTYPES or value_dtype not in _VALUE_DTYPES:
            raise TypeError("EmbeddingVariable keys are int32 / int64 and values float32 / "
                            "float64 (the reference's KvResourceGather registrations) or "
                            "bfloat16 (bf16 EV)")
        self.name = name
        self.dim = int(embedding_dim)
        self.key_dtype = key_dtype
        if _primary is None:
            self.value_dtype = value_dtype
        else:
            # optimizer slots of a bf16 EV keep fp32 state
            pv = _primary.value_dtype
            self.value_dtype = torch.float32 if pv == torch.bfloat16 else pv
        if self.value_dtype == torch.bfloat16 and self.dim % 2:
            raise _lib.DeepRecError(_lib.INVALID_ARGUMENT, "bf16 EVs need an even dim")
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        self.initializer = initializer
        self._primary = _primary
        self._slot_index = _slot_index
        self._lock = threading.Lock()
        self.pending_grads = []
        opt = ev_option or EmbeddingVariableOption()
        f = opt.filter_option
        self.filter_freq = int(getattr(f, "filter_freq", 0) or 0)
        if opt.evict_option is not None and opt.evict_option.steps_to_live:
            steps_to_live = opt.evict_option.steps_to_live
        self.steps_to_live = int(steps_to_live or 0)
        # EmbeddingConfig::l2_weight_threshold (embedding_config.h:17,28): -1 = off
        self.l2_weight_threshold = float(l2_weight_threshold)
        _flush_deferred_releases()
        bf16 = self.value_dtype == torch.bfloat16
        # the C ABI takes the default row in fp32 (a bf16 EV rounds it to
        # nearest even, as the .to(torch.bfloat16) below does)
        default = _default_row(initializer, self.dim, self.device,
                               torch.float32 if bf16 else self.value_dtype)
        self._default_host = default.to(torch.bfloat16) if bf16 else default
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            if _primary is None:
                cfg = _lib.DrEvConfig()
                cfg.dim = self.dim
                cfg.capacity = int(capacity)
                cfg.steps_to_live = self.steps_to_live
                cfg.filter_freq = self.filter_freq
                cfg.max_element_size = int(getattr(f, "max_element_size", 0) or 0)
                cfg.false_positive_probability = float(
                    getattr(f, "false_positive_probability", -1.0))
                cfg.counter_bits = int(getattr(f, "counter_bits", 64) or 64)
                cfg.layout = 1 if (self.filter_freq or self.steps_to_live) else 0
                cfg.value_bits = {torch.float64: 64, torch.bfloat16: 16}.get(self.value_dtype, 32)
                check(lib().dr_ev_create(C.byref(cfg), default.data_ptr(), C.byref(h)))
            else:
                check(lib().dr_ev_create_slot(_primary._h, _slot_index, default.data_ptr(),
                                              C.byref(h)))
        self._h = h
        self._slots = {}
        self._next_slot = 1

    # -- lifecycle ---------------------------------------------------------
    def __del__(self):
        try:
            if getattr(self, "_h", None):
                _release_handle(self._h)
                self._h = None
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def resource(self):
        """The EV as an op input (torch_ops): a host int64[1] tensor holding
        the library handle, TF's DT_RESOURCE scalar (host memory).  Ops that
        change the EV list it in mutates_args."""
        r = getattr(self, "_resource", None)
        if r is None:
            r = torch.tensor([self._h.value], dtype=torch.int64)
            self._resource = r
        return r

    def is_primary(self):
        return self._primary is None

    def slot(self, name, initializer):
        """Slot EV sharing this EV's key space (slot_creator.py:82-117)."""
        if name not in self._slots:
            idx = self._next_slot
            self._next_slot += 1
            self._slots[name] = EmbeddingVariable(self.name + "/" + name, self.dim, initializer,
                                                  device=self.device, _primary=self,
                                                  _slot_index=idx, key_dtype=self.key_dtype)
        return self._slots[name]

    def get_shape(self):
        return (None, self.dim)

    @property
    def default_value(self):
        return self._default_host.to(self.device)

    def pool(self):
        """Base pointer of this EV's value rows (device)."""
        return lib().dr_ev_pool(self._h)

    @property
    def is_bf16(self):
        return self.value_dtype == torch.bfloat16

    @property
    def row_words(self):
        """32-bit words per value row (the kernels' row stride): dim, or
        dim / 2 for a bf16 EV."""
        return self.dim // 2 if self.is_bf16 else self.dim

    # -- ops -----------------------------------------------------------------
    def _defaults_for(self, n, ev_init_value):
        if ev_init_value is not None:
            return torch.as_tensor(ev_init_value, dtype=self.value_dtype,
                                   device=self.device).expand(n, self.dim).contiguous()
        if callable(self.initializer):
            v = self.initializer((n, self.dim))
            return torch.as_tensor(v, dtype=self.value_dtype, device=self.device).reshape(
                n, self.dim).contiguous()
        return None

    def sparse_read(self, indices, counts=None, ev_init_value=None, name=None):
        """KvResourceGather / KvResourceGatherV1 (kv_variable_ops.py:644-664),
        int32 or int64 ids, float32 or float64 rows per the EV's dtypes."""
        i32 = indices.dtype == torch.int32
        ids = indices.reshape(-1).to(torch.int32 if i32 else torch.int64).contiguous()
        n = ids.numel()
        out = torch.empty((n, self.dim), dtype=self.value_dtype, device=self.device)
        if n == 0:
            return out.reshape(tuple(indices.shape) + (self.dim,))
        dflt = self._defaults_for(n, ev_init_value)
        cnt = None if counts is None else counts.reshape(-1).to(torch.int32).contiguous()
        if i32:
            wsb = lib().dr_ev_gather_i32_workspace_size(n)
            ws = workspace(wsb, self.device)
            check(lib().dr_ev_gather_i32(self._h, ptr(ids), n, ptr(dflt), ptr(cnt), ptr(out),
                                         ptr(ws), wsb, stream_handle(self.device)))
        else:
            wsb = lib().dr_ev_gather_workspace_size(n)
            ws = workspace(wsb, self.device)
            check(lib().dr_ev_gather(self._h, ptr(ids), n, ptr(dflt), ptr(cnt), ptr(out), ptr(ws),
                                     wsb, stream_handle(self.device)))
        from .ops import _post
        _post(self.device)
        return out.reshape(tuple(indices.shape) + (self.dim,))

    def resolve(self, keys, n_dev=None, counts=None, defaults=None):
        """Insert-on-miss resolve of (unique) keys to rows; -(i+1) = default row i."""
        keys = keys.reshape(-1).to(torch.int64).contiguous()
        n = keys.numel()
        rows = torch.empty(n, dtype=torch.int64, device=self.device)
        wsb = lib().dr_ev_resolve_workspace_size(n)
        ws = workspace(wsb, self.device)
        check(lib().dr_ev_resolve(self._h, ptr(keys), n, ptr(n_dev), ptr(defaults), ptr(counts),
                                  ptr(rows), ptr(ws), wsb, stream_handle(self.device)))
        return rows

    def insert(self, keys, values, versions=None, freqs=None):
        """KvResourceInsert (core/ops/kv_variable_ops.cc:478-492) with
        EmbeddingVar::Import semantics: existing rows are kept."""
        return self._import(keys, values, versions, freqs, 0, 0)

    def import_partitioned(self, keys, values, versions, freqs, partition_id, partition_num):
        """KvResourceImportV2 restore filter key % 1000 % partition_num == id."""
        return self._import(keys, values, versions, freqs, partition_id, partition_num)

    def _import(self, keys, values, versions, freqs, pid, pnum):
        i32 = keys.dtype == torch.int32
        k = keys.reshape(-1).to(device=self.device,
                                dtype=torch.int32 if i32 else torch.int64).contiguous()
        v = values.reshape(k.numel(), self.dim).to(device=self.device,
                                                   dtype=self.value_dtype).contiguous()
        ver = None if versions is None else versions.to(device=self.device,
                                                        dtype=torch.int64).contiguous()
        fr = None if freqs is None else freqs.to(device=self.device, dtype=torch.int64).contiguous()
        fn = lib().dr_ev_insert_i32 if i32 else lib().dr_ev_insert
        check(fn(self._h, ptr(k), k.numel(), ptr(v), ptr(ver), ptr(fr), pid, pnum,
                 stream_handle(self.device)))

    def insert_synthetic(self, key_begin, n, seed, key_stride=1):
        """Insert keys key_begin + i*key_stride, i < n, rows synth(seed, key, col)."""
        check(lib().dr_ev_insert_synthetic(self._h, int(key_begin), int(key_stride), int(n),
                                           int(seed), stream_handle(self.device)))

    def total_count(self):
        """KvVariableShape: [num keys, dim]."""
        n = C.c_int64(0)
        check(lib().dr_ev_size(self._h, C.byref(n), stream_handle(self.device)))
        return torch.tensor([n.value, self.dim], dtype=torch.int64)

    def export(self):
        """KvResourceExport -> (keys, values, versions, freqs), keys ascending
        (keys in the EV's key dtype, values in its value dtype)."""
        m = C.c_int64(0)
        st = stream_handle(self.device)
        check(lib().dr_ev_export(self._h, None, None, None, None, 0, C.byref(m), st))
        M = m.value
        keys = torch.empty(M, dtype=self.key_dtype, device=self.device)
        vals = torch.empty((M, self.dim), dtype=self.value_dtype, device=self.device)
        vers = torch.empty(M, dtype=torch.int64, device=self.device)
        frqs = torch.empty(M, dtype=torch.int64, device=self.device)
        fn = lib().dr_ev_export_i32 if self.key_dtype == torch.int32 else lib().dr_ev_export
        check(fn(self._h, ptr(keys), ptr(vals), ptr(vers), ptr(frqs), M, C.byref(m), st))
        n = m.value
        if self.steps_to_live == 0:
            vers = vers[:0]
        if self.filter_freq == 0:
            frqs = frqs[:0]
        return keys[:n], vals[:n], vers, frqs

    def key_meta(self, keys):
        """(freq, version, has_row) of keys, host numpy (tests/debug)."""
        import numpy as np
        k = np.ascontiguousarray(keys, dtype=np.int64)
        n = k.shape[0]
        fr = np.zeros(n, np.int64)
        ve = np.zeros(n, np.int64)
        hr = np.zeros(n, np.int32)
        check(lib().dr_ev_key_meta(self._h, k.ctypes.data, n, fr.ctypes.data, ve.ctypes.data,
                                   hr.ctypes.data, stream_handle(self.device)))
        return fr, ve, hr.astype(bool)

    def reserve(self, extra):
        check(lib().dr_ev_reserve(self._h, int(extra), stream_handle(self.device)))

    def shrink(self, global_step=0):
        """EmbeddingVar::Shrink (embedding_var.h:264-313) on the key space this
        EV shares with its slots: by L2 weight when l2_weight_threshold != -1,
        else by global step when steps_to_live > 0.  Returns keys removed."""
        p = self._primary or self
        n = C.c_int64(0)
        check(lib().dr_ev_shrink(p._h, int(global_step), p.l2_weight_threshold, C.byref(n),
                                 stream_handle(self.device)))
        return n.value


_EV_REGISTRY = {}


def get_embedding_variable(name, embedding_dim, key_dtype=torch.int64, initializer=None,
                           steps_to_live=0, ev_option=None, capacity=1 << 16, device=None,
                           partitioner=None, l2_weight_threshold=-1.0, value_dtype=torch.float32):
    """tf.get_embedding_variable (variable_scope.py:2142-2197).

    With `partitioner=n` (fixed_size_partitioner(num_shards=n)) returns a list
    of n EVs; lookups route key -> shard by key % 1000 % n
    (embedding_ops.py:207-209)."""
    if partitioner is not None and int(partitioner) > 1:
        return [get_embedding_variable("%s/part_%d" % (name, p), embedding_dim, key_dtype,
                                       initializer, steps_to_live, ev_option, capacity, device,
                                       l2_weight_threshold=l2_weight_threshold,
                                       value_dtype=value_dtype)
                for p in range(int(partitioner))]
    if name in _EV_REGISTRY:
        return _EV_REGISTRY[name]
    ev = EmbeddingVariable(name, embedding_dim, initializer, steps_to_live, ev_option, capacity,
                           device, l2_weight_threshold=l2_weight_threshold, key_dtype=key_dtype,
                           value_dtype=value_dtype)
    _EV_REGISTRY[name] = ev
    return ev


def reset_registry():
    _EV_REGISTRY.clear()
