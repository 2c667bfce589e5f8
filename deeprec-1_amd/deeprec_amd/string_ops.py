"""String -> id ops on the GPU (the step before the lookup).

Mirrors tf.strings.to_hash_bucket_fast / string_to_hash_bucket_fast
(python/ops/string_ops.py, op StringToHashBucketFast core/ops/string_ops.cc:77,
CPU kernel core/kernels/string_to_hash_bucket_ali_op.h:33-63) and the hashing
of EV string columns (python/feature_column/feature_column_v2.py:5954-5957:
num_buckets = INT64_MAX).  The hash is farmhash Fingerprint64, computed by
dr_fingerprint64 / dr_string_to_hash_bucket_fast (csrc/strings.hip).

Strings live on the device as a `StringTensor`: one uint8 byte buffer plus
int64 offsets [n+1] (Arrow's binary layout).  Python lists of str/bytes are
packed once on the host and copied over.
"""
import numpy as np
import torch

from . import ops
from ._lib import INVALID_ARGUMENT, DeepRecError, check, lib, ptr, require_gpu, stream_handle

INT64_MAX = np.iinfo(np.int64).max


class StringTensor(object):
    """n strings on a device: bytes (uint8) + offsets (int64 [n+1])."""

    def __init__(self, data, offsets):
        if data.dtype != torch.uint8 or offsets.dtype != torch.int64:
            raise DeepRecError(INVALID_ARGUMENT, "StringTensor needs uint8 data, int64 offsets")
        self.data = data.contiguous()
        self.offsets = offsets.contiguous()

    @classmethod
    def from_list(cls, strings, device="cuda"):
        require_gpu()
        enc = [s.encode("utf-8") if isinstance(s, str) else bytes(s) for s in strings]
        off = np.zeros(len(enc) + 1, np.int64)
        if enc:
            off[1:] = np.cumsum([len(e) for e in enc])
        buf = np.frombuffer(b"".join(enc) or b"\0", np.uint8)
        return cls(torch.as_tensor(buf.copy(), device=device),
                   torch.as_tensor(off, device=device))

    def __len__(self):
        return self.offsets.numel() - 1

    @property
    def device(self):
        return self.offsets.device


def _as_strings(x, device=None):
    if isinstance(x, StringTensor):
        return x
    return StringTensor.from_list(list(x), device or "cuda")


def fingerprint64(strings, device=None):
    """uint64 farmhash Fingerprint64 per string, returned as int64 bits."""
    s = _as_strings(strings, device)
    dev = ops._dev(s.offsets)
    out = torch.empty(len(s), dtype=torch.int64, device=dev)
    check(lib().dr_fingerprint64(ptr(s.data), ptr(s.offsets), len(s), ptr(out),
                                 stream_handle(dev)))
    ops._post(dev)
    return out


def string_to_hash_bucket_fast(input, num_buckets, name=None):
    """StringToHashBucketFast: Fingerprint64(s) % num_buckets (int64)."""
    num_buckets = int(num_buckets)
    if num_buckets <= 0:
        raise DeepRecError(INVALID_ARGUMENT, "num_buckets must be positive")
    s = _as_strings(input)
    dev = ops._dev(s.offsets)
    out = torch.empty(len(s), dtype=torch.int64, device=dev)
    check(lib().dr_string_to_hash_bucket_fast(ptr(s.data), ptr(s.offsets), len(s), num_buckets,
                                              ptr(out), stream_handle(dev)))
    ops._post(dev)
    return out


to_hash_bucket_fast = string_to_hash_bucket_fast


def ev_string_ids(input):
    """Keys of an EV string column (feature_column_v2.py:5954-5957)."""
    return string_to_hash_bucket_fast(input, INT64_MAX)
