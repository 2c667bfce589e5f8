"""EmbeddingVariable checkpoints in DeepRec's on-disk layout.

Two layers:

* `BundleWriter` / `BundleReader`: TensorFlow's TensorBundle V2 format
  (core/util/tensor_bundle/tensor_bundle.cc) -- `<prefix>.data-00000-of-00001`
  holds the tensors' raw little-endian bytes in the order they were added,
  `<prefix>.index` is an SSTable (core/lib/io/table_builder.cc, LevelDB
  format: 256 KiB blocks, restart interval 16, no compression, masked crc32c
  block trailers) mapping "" -> BundleHeaderProto and each tensor name ->
  BundleEntryProto {dtype, shape, shard_id, offset, size, masked crc32c}
  (core/protobuf/tensor_bundle.proto).  The writer reproduces the reference's
  files byte for byte (tests/golden/ckpt/, from the reference's testdata).

* `dump_embedding_values` / `restore_embedding_variable`: what DeepRec's
  saver ops do for an EV (core/kernels/kv_variable_ops.h:148-265 and
  :459-673, save_restore_v2_ops.cc:128-133).  Save writes
  `<name>-partition_offset` (int32 [1001]) and `<name>-{keys, values,
  versions, freqs}` with the keys grouped into kSavedPartitionNum = 1000
  sub-partitions by `key % 1000` (C++ remainder: negative keys match no
  sub-partition and are not saved), so a job with a different partition
  count can restore its share.  Restore follows EVRestoreDynamically: a name
  without "part_" imports everything; otherwise the new form (partition
  offsets present) reads, from every saved part, the sub-partitions
  i % partition_num == partition_id, and the old form reads whole parts;
  both import through EmbeddingVar::Import with the
  `key % 1000 % partition_num == partition_id` filter, versions default -1
  and freqs default to filter_freq (MinFreq).

The device side is the engine's: `EmbeddingVariable.export()` (dr_ev_export,
GPU), the 1000-way stable split (dr_partition_by_owner with world = 1000 +
dr_rows_pack, GPU) and `import_partitioned()` (dr_ev_insert, GPU).  Only the
file bytes pass through the host; checksums run natively (dr_crc32c_extend).
"""
import os
import struct

import numpy as np
import torch

from . import _lib

SAVED_PARTITION_NUM = 1000            # kv_variable_ops.h:39
_MAGIC = 0xdb4775248b80fb57           # table/format.h kTableMagicNumber
_BLOCK_SIZE = 262144                  # core/lib/io/table_options.h:41
_RESTART_INTERVAL = 16                # :46

_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
       np.dtype(np.uint8): 4, np.dtype(np.int16): 5, np.dtype(np.int8): 6,
       np.dtype(np.int64): 9, np.dtype(np.bool_): 10, np.dtype(np.uint16): 17,
       np.dtype(np.float16): 19, np.dtype(np.uint32): 22, np.dtype(np.uint64): 23}
_NP = {v: k for k, v in _DT.items()}


def crc32c(data, init=0):
    """crc32c::Extend (core/lib/hash/crc32c.h), native."""
    if isinstance(data, np.ndarray):
        data = np.ascontiguousarray(data)
        return _lib.lib().dr_crc32c_extend(init, data.ctypes.data, data.nbytes)
    return _lib.lib().dr_crc32c_extend(init, bytes(data), len(data))


def mask_crc(c):
    return ((((c >> 15) | (c << 17)) & 0xffffffff) + 0xa282ead8) & 0xffffffff


def unmask_crc(m):
    r = (m - 0xa282ead8) & 0xffffffff
    return ((r >> 17) | (r << 15)) & 0xffffffff


# -- protobuf wire encoding (the two messages the bundle index holds) --------
def _varint(v):
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7f
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7f) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _field(num, wire, payload):
    return _varint((num << 3) | wire) + payload


def _vfield(num, v):            # proto3 scalar: omitted when 0
    return _field(num, 0, _varint(v)) if v else b""


def _header_proto():
    # BundleHeaderProto {num_shards: 1, endianness: LITTLE (default), version {producer: 1}}
    return _vfield(1, 1) + _field(3, 2, _varint(2) + _vfield(1, 1))


def _entry_proto(dtype, shape, offset, size, crc):
    shp = b"".join(_field(2, 2, _varint(len(d)) + d)
                   for d in (_vfield(1, int(s)) for s in shape))
    return (_vfield(1, dtype) + _field(2, 2, _varint(len(shp)) + shp) + _vfield(4, offset)
            + _vfield(5, size) + _field(6, 5, struct.pack("<I", crc)))


def _parse_entry(buf):
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": 0,
         "slices": 0}
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, pos = _read_varint(buf, pos)
            name = {1: "dtype", 3: "shard_id", 4: "offset", 5: "size", 100: "is_hash_table"}
            if num in name:
                e[name[num]] = v
        elif wire == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
            if num == 6:
                e["crc32c"] = v
        elif wire == 2:
            n, pos = _read_varint(buf, pos)
            sub = buf[pos:pos + n]
            pos += n
            if num == 2:
                e["shape"] = _parse_shape(sub)
            elif num == 7:
                e["slices"] += 1
        elif wire == 1:
            pos += 8
        else:
            raise _lib.DeepRecError(_lib.INTERNAL, "bad bundle entry wire type %d" % wire)
    return e


def _parse_shape(buf):
    dims, pos = [], 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        n, pos = _read_varint(buf, pos) if key & 7 == 2 else (0, pos)
        if key >> 3 == 2:
            sub, size, p = buf[pos:pos + n], 0, 0
            while p < len(sub):
                k2, p = _read_varint(sub, p)
                v, p = _read_varint(sub, p) if k2 & 7 == 0 else (0, p)
                if k2 >> 3 == 1:
                    size = v - (1 << 64) if v >= (1 << 63) else v
            dims.append(size)
        elif key >> 3 == 3 and key & 7 == 0:       # unknown_rank
            n = 0
        pos += n
    return dims


# -- SSTable (LevelDB format) -------------------------------------------------
class _Block(object):
    def __init__(self, restart_interval):
        self.ri = restart_interval
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""

    def add(self, key, value):
        shared = 0
        if self.counter < self.ri:
            m = min(len(key), len(self.last))
            while shared < m and key[shared] == self.last[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def size_estimate(self):
        return len(self.buf) + 4 * len(self.restarts) + 4

    def finish(self):
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))

    def empty(self):
        return not self.buf


def _shortest_separator(start, limit):
    m = min(len(start), len(limit))
    i = 0
    while i < m and start[i] == limit[i]:
        i += 1
    if i < m:
        b = start[i]
        if b < 0xff and b + 1 < limit[i]:
            return start[:i] + bytes([b + 1])
    return start


def _short_successor(key):
    for i, b in enumerate(key):
        if b != 0xff:
            return key[:i] + bytes([b + 1])
    return key


class _TableWriter(object):
    def __init__(self, f, block_size=_BLOCK_SIZE):
        self.f = f
        self.block_size = block_size
        self.offset = 0
        self.data = _Block(_RESTART_INTERVAL)
        self.index = _Block(1)
        self.pending = None            # handle of the last flushed data block
        self.last = b""

    def _write_block(self, contents):
        trailer = b"\x00"
        crc = mask_crc(crc32c(contents + trailer))
        h = (self.offset, len(contents))
        self.f.write(contents + trailer + struct.pack("<I", crc))
        self.offset += len(contents) + 5
        return h

    def add(self, key, value):
        if self.pending is not None:
            self.index.add(_shortest_separator(self.last, key), _varint(self.pending[0]) +
                           _varint(self.pending[1]))
            self.pending = None
        self.data.add(key, value)
        self.last = key
        if self.data.size_estimate() >= self.block_size:
            self._flush()

    def _flush(self):
        if self.data.empty():
            return
        self.pending = self._write_block(self.data.finish())
        self.data = _Block(_RESTART_INTERVAL)

    def finish(self):
        self._flush()
        meta = self._write_block(_Block(_RESTART_INTERVAL).finish())
        if self.pending is not None:
            self.index.add(_short_successor(self.last), _varint(self.pending[0]) +
                           _varint(self.pending[1]))
        idx = self._write_block(self.index.finish())
        footer = _varint(meta[0]) + _varint(meta[1]) + _varint(idx[0]) + _varint(idx[1])
        footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", _MAGIC)
        self.f.write(footer)


def _read_block(raw, off, size, verify=True):
    contents = raw[off:off + size]
    if verify:
        want = struct.unpack_from("<I", raw, off + size + 1)[0]
        if unmask_crc(want) != crc32c(raw[off:off + size + 1]):
            raise _lib.DeepRecError(_lib.INTERNAL, "corrupted SSTable block at %d" % off)
    n = struct.unpack_from("<I", contents, len(contents) - 4)[0]
    end = len(contents) - 4 - 4 * n
    out, pos, last = [], 0, b""
    while pos < end:
        shared, pos = _read_varint(contents, pos)
        nonshared, pos = _read_varint(contents, pos)
        vlen, pos = _read_varint(contents, pos)
        key = last[:shared] + bytes(contents[pos:pos + nonshared])
        pos += nonshared
        out.append((key, bytes(contents[pos:pos + vlen])))
        pos += vlen
        last = key
    return out


def _read_table(path):
    raw = open(path, "rb").read()
    if len(raw) < 48 or struct.unpack_from("<Q", raw, len(raw) - 8)[0] != _MAGIC:
        raise _lib.DeepRecError(_lib.INTERNAL, "%s is not an SSTable" % path)
    pos = len(raw) - 48
    _, pos = _read_varint(raw, pos)
    _, pos = _read_varint(raw, pos)
    io, pos = _read_varint(raw, pos)
    isz, pos = _read_varint(raw, pos)
    entries = []
    for _, handle in _read_block(raw, io, isz):
        bo, p = _read_varint(handle, 0)
        bs, _ = _read_varint(handle, p)
        entries.extend(_read_block(raw, bo, bs))
    return entries


# -- TensorBundle --------------------------------------------------------------
def data_path(prefix):
    return prefix + ".data-00000-of-00001"


def index_path(prefix):
    return prefix + ".index"


class BundleWriter(object):
    """tensor_bundle.cc BundleWriter: add() appends a tensor's bytes to the
    data file; finish() writes the sorted index."""

    def __init__(self, prefix, block_size=_BLOCK_SIZE):
        self.prefix = prefix
        d = os.path.dirname(prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        self._data = open(data_path(prefix) + ".tmp", "wb")
        self._size = 0
        self._entries = {}
        self._block_size = block_size

    def add(self, key, array):
        key = key.encode() if isinstance(key, str) else bytes(key)
        if not key:
            raise _lib.InvalidArgumentError(_lib.INVALID_ARGUMENT, "empty tensor name")
        if key in self._entries:
            raise _lib.InvalidArgumentError(_lib.INVALID_ARGUMENT,
                                            "Adding duplicate key: %s" % key.decode())
        if torch.is_tensor(array):
            array = array.detach().cpu().numpy()
        a = np.ascontiguousarray(array)
        if a.dtype not in _DT:
            raise _lib.InvalidArgumentError(_lib.INVALID_ARGUMENT, "unsupported dtype %s" % a.dtype)
        a = a.astype(a.dtype.newbyteorder("<"), copy=False)
        crc = crc32c(a) if a.nbytes else 0
        self._data.write(memoryview(a).cast("B") if a.nbytes else b"")
        self._entries[key] = _entry_proto(_DT[a.dtype], a.shape, self._size, a.nbytes,
                                          mask_crc(crc))
        self._size += a.nbytes

    def finish(self):
        self._data.close()
        os.replace(data_path(self.prefix) + ".tmp", data_path(self.prefix))
        tmp = index_path(self.prefix) + ".tmp"
        with open(tmp, "wb") as f:
            t = _TableWriter(f, self._block_size)
            t.add(b"", _header_proto())
            for k in sorted(self._entries):
                t.add(k, self._entries[k])
            t.finish()
        os.replace(tmp, index_path(self.prefix))


class BundleReader(object):
    """tensor_bundle.cc BundleReader (single shard, little endian)."""

    def __init__(self, prefix):
        self.prefix = prefix
        ents = _read_table(index_path(prefix))
        if not ents or ents[0][0] != b"":
            raise _lib.DeepRecError(_lib.INTERNAL, "bundle index without header")
        self.entries = {k.decode(): _parse_entry(v) for k, v in ents[1:]}
        self._mm = None

    def _data(self):
        if self._mm is None:
            self._mm = np.memmap(data_path(self.prefix), np.uint8, "r") \
                if os.path.getsize(data_path(self.prefix)) else np.zeros(0, np.uint8)
        return self._mm

    def keys(self):
        return sorted(self.entries)

    def contains(self, key):
        return key in self.entries

    def dtype_and_shape(self, key):
        e = self._entry(key)
        return _NP[e["dtype"]], tuple(e["shape"])

    def _entry(self, key):
        if key not in self.entries:
            raise _lib.DeepRecError(_lib.NOT_FOUND, "Key %s not found in checkpoint" % key)
        return self.entries[key]

    def lookup(self, key, verify=True):
        e = self._entry(key)
        dt = _NP[e["dtype"]]
        raw = self._data()[e["offset"]:e["offset"] + e["size"]]
        if verify and e["size"] and unmask_crc(e["crc32c"]) != crc32c(np.asarray(raw)):
            raise _lib.DeepRecError(_lib.INTERNAL, "checksum mismatch for %s" % key)
        return np.frombuffer(raw.tobytes(), dt).reshape(e["shape"]).copy()

    def lookup_rows(self, key, begin, end):
        """Rows [begin, end) of a tensor (LookupSegmentOffset), no checksum."""
        e = self._entry(key)
        dt = _NP[e["dtype"]]
        shape = e["shape"]
        row = int(np.prod(shape[1:], dtype=np.int64)) * dt.itemsize if len(shape) > 1 \
            else dt.itemsize
        raw = self._data()[e["offset"] + begin * row:e["offset"] + end * row]
        return np.frombuffer(raw.tobytes(), dt).reshape((end - begin,) + tuple(shape[1:])).copy()


# -- EmbeddingVariable save / restore ------------------------------------------
def partition_snapshot(keys, values, versions, freqs):
    """DumpEmbeddingValues' layout on the device: keys grouped by key % 1000
    (stable), negative keys dropped.  Returns (offsets int32 [1001], keys,
    values, versions, freqs) as device tensors."""
    from . import ops
    keep = keys >= 0
    if not bool(keep.all()):
        keys, values = keys[keep], values[keep]
        versions = versions[keep] if versions.numel() else versions
        freqs = freqs[keep] if freqs.numel() else freqs
    n = keys.numel()
    offs = torch.zeros(SAVED_PARTITION_NUM + 1, dtype=torch.int32, device=keys.device)
    if n == 0:
        return offs, keys, values, versions, freqs
    ks, perm, counts = ops.partition_by_owner(keys.contiguous(), SAVED_PARTITION_NUM)
    vals = torch.empty_like(values)
    ops.rows_pack(values.contiguous(), perm, vals)
    p64 = perm.to(torch.int64)
    versions = versions[p64] if versions.numel() else versions
    freqs = freqs[p64] if freqs.numel() else freqs
    offs[1:] = torch.cumsum(counts[:SAVED_PARTITION_NUM], 0).to(torch.int32)
    return offs, ks, vals, versions, freqs


def dump_embedding_values(ev, tensor_key, writer):
    """DumpEmbeddingValues (kv_variable_ops.h:148-265) of one EV (primary or
    slot) under `tensor_key` (e.g. "emb/part_0")."""
    keys, vals, vers, frqs = ev.export()
    offs, keys, vals, vers, frqs = partition_snapshot(keys, vals, vers, frqs)
    write_ev_tensors(writer, tensor_key, offs, keys, vals.reshape(-1, ev.dim), vers, frqs)


def write_ev_tensors(writer, tensor_key, offs, keys, vals, vers, frqs):
    """The five tensors of one EV, in DumpEmbeddingValues' write order
    (partition_offset first, then keys, values, versions, freqs)."""
    writer.add(tensor_key + "-partition_offset", offs)
    writer.add(tensor_key + "-keys", keys)
    writer.add(tensor_key + "-values", vals)
    writer.add(tensor_key + "-versions", vers)
    writer.add(tensor_key + "-freqs", frqs)


def save(prefix, variables, global_step=None):
    """Saver.save for EVs: {tensor_key: EmbeddingVariable} -> one bundle.

    Like DumpEv (save_restore_v2_ops.cc:117-133), each variable's key space
    is shrunk first (EmbeddingVar::Shrink: by L2 weight when the EV has an
    l2_weight_threshold, else by global step when steps_to_live > 0), so
    evicted keys are not written; global_step None skips the step eviction."""
    w = BundleWriter(prefix)
    for name in variables:
        ev = variables[name]
        p = ev._primary or ev
        if p.l2_weight_threshold != -1.0 or (global_step is not None and p.steps_to_live > 0):
            ev.shrink(0 if global_step is None else global_step)
        dump_embedding_values(ev, name, w)
    w.finish()
    return prefix


def _part_name(name, part, partition_id):
    i = name.find("part_")
    post = name[i + len("part_") + len(str(partition_id)):]
    return name[:i] + "part_" + str(part) + post


def _import(ev, reader, tname, begin, end, filtered, partition_id, partition_num):
    keys = reader.lookup_rows(tname + "-keys", begin, end)
    n = keys.shape[0]
    if n == 0:
        return
    vals = reader.lookup_rows(tname + "-values", begin, end)
    vshape = reader.entries[tname + "-versions"]["shape"]
    vers = (reader.lookup_rows(tname + "-versions", begin, end) if vshape and vshape[0] > 0
            else np.full(n, -1, np.int64))
    fkey = tname + "-freqs"
    if reader.contains(fkey) and reader.entries[fkey]["shape"] and \
            reader.entries[fkey]["shape"][0] > 0:
        frqs = reader.lookup_rows(fkey, begin, end)
    else:
        frqs = np.full(n, ev.filter_freq, np.int64)          # MinFreq
    dev = ev.device
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    if filtered:
        ev.import_partitioned(t(keys), t(vals), t(vers), t(frqs), partition_id, partition_num)
    else:
        ev.import_partitioned(t(keys), t(vals), t(vers), t(frqs), 0, 0)


def restore_embedding_variable(ev, reader, name, partition_id=0, partition_num=1):
    """EVRestoreDynamically (kv_variable_ops.h:459-673)."""
    if isinstance(reader, str):
        reader = BundleReader(reader)
    if "part_" not in name:                                 # RestoreValue, no filter
        n = reader.dtype_and_shape(name + "-keys")[1][0]
        _import(ev, reader, name, 0, n, False, 0, 1)
        return
    new_form = reader.contains(_part_name(name, 0, partition_id) + "-partition_offset")
    part = 0
    while True:
        tname = _part_name(name, part, partition_id)
        if not reader.contains(tname + "-keys"):
            break
        if new_form:
            for key in ("-values", "-versions"):
                # LookupHeader / LookupTensorShape fail on a missing tensor and
                # EVRestoreDynamically treats that as fatal: raise, do not
                # leave the EV half restored
                if not reader.contains(tname + key):
                    raise _lib.DeepRecError(_lib.NOT_FOUND, "Key %s%s not found in checkpoint"
                                       % (tname, key))
            offs = reader.lookup(tname + "-partition_offset")
            for sub in range(partition_id % SAVED_PARTITION_NUM, SAVED_PARTITION_NUM,
                             partition_num):
                if offs[sub + 1] > offs[sub]:
                    _import(ev, reader, tname, int(offs[sub]), int(offs[sub + 1]), True,
                            partition_id, partition_num)
        else:                                               # DynamicRestoreValue
            n = reader.dtype_and_shape(tname + "-keys")[1][0]
            _import(ev, reader, tname, 0, n, True, partition_id, partition_num)
        part += 1


def restore(prefix, variables, partition_id=0, partition_num=1):
    """Restore {tensor_key: EmbeddingVariable} from a bundle."""
    r = BundleReader(prefix)
    for name in variables:
        restore_embedding_variable(variables[name], r, name, partition_id, partition_num)
