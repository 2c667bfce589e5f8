"""deeprec_amd -- MI355X-native engine for DeepRec's EmbeddingVariable /
embedding_lookup_sparse hot path.

The compute is HIP (gfx950) behind the C ABI in include/deeprec_amd.h; this
package mirrors the reference's Python op surface (tf.get_embedding_variable,
EmbeddingVariable.sparse_read, tf.nn.embedding_lookup_sparse,
safe_embedding_lookup_sparse, fused_embedding_lookup_sparse, the EV sparse
optimizers) on torch device tensors.
"""
from . import _lib
from . import torch_ops  # noqa: F401  (registers torch.ops.deeprec.*)
from ._lib import DeepRecError, InvalidArgumentError, load
from .embedding_ops import (DenseTable, SparseTensor, embedding_lookup, embedding_lookup_sparse,
                            embedding_lookup_sparse_multi, fused_embedding_lookup_sparse,
                            safe_embedding_lookup_sparse)
from .kv_variable_ops import (CBFFilter, CounterFilter, EmbeddingVariable, EmbeddingVariableOption,
                              GlobalStepEvict, IndexedSlices, flush_releases,
                              get_embedding_variable)
from .ops import set_validate, status_check
from .string_ops import StringTensor, string_to_hash_bucket_fast
from .training import (AdagradDecayOptimizer, AdagradOptimizer, AdamAsyncOptimizer, AdamOptimizer,
                       FtrlOptimizer, GradientDescentOptimizer)

__all__ = [
    "DeepRecError", "InvalidArgumentError", "load", "DenseTable", "SparseTensor",
    "embedding_lookup", "embedding_lookup_sparse", "embedding_lookup_sparse_multi",
    "fused_embedding_lookup_sparse", "safe_embedding_lookup_sparse", "CBFFilter",
    "CounterFilter", "EmbeddingVariable", "EmbeddingVariableOption", "GlobalStepEvict",
    "IndexedSlices", "get_embedding_variable", "set_validate", "status_check",
    "AdagradOptimizer", "AdagradDecayOptimizer", "AdamAsyncOptimizer", "AdamOptimizer",
    "FtrlOptimizer", "GradientDescentOptimizer", "StringTensor",
    "string_to_hash_bucket_fast",
]
