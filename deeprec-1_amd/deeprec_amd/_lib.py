"""ctypes binding of the engine's C ABI (include/deeprec_amd.h).

The shared library is built in-tree by `make -C deeprec-1_amd` (or
__graft_entry__.build()).  There is deliberately no CPU fallback: if the
library is missing, or no GPU is visible, every op raises.
"""
import ctypes as C
import os

# hipGraph replays and the ROCm runtime's graph packet capture
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE, on by default in this ROCm): with it on,
# a captured graph is right on its first replay and can be wrong from the
# second on once other kernels and allocations ran in the process between
# replays -- reproduced with plain torch ops, no engine code involved
# (tools/torch_graph_churn_probe.py: a.sum() + b.sum() in a graph, replayed
# after allocator churn, changes value; profiles/r06_graph_replay_bisect.log).
# The runtime reads the flag once, when HIP initialises: it is set here, before
# this module touches the GPU, unless the caller set it.  GRAPH_REPLAY_SAFE
# says whether that happened before HIP was up (a process that initialised the
# GPU before importing deeprec_amd must export the variable itself).
GRAPH_PACKET_CAPTURE_ENV = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
os.environ.setdefault(GRAPH_PACKET_CAPTURE_ENV, "0")

import torch  # noqa: E402

GRAPH_REPLAY_SAFE = (os.environ.get(GRAPH_PACKET_CAPTURE_ENV) == "0"
                     and not torch.cuda.is_initialized())

_HERE = os.path.dirname(os.path.abspath(__file__))
# DEEPREC_AMD_LIB: an A/B build of the same library (measurement only)
LIB_PATH = os.environ.get("DEEPREC_AMD_LIB") or os.path.join(_HERE, "libdeeprec_amd.so")

# TF error::Code values (include/deeprec_amd.h)
OK, INVALID_ARGUMENT, NOT_FOUND, ALREADY_EXISTS, RESOURCE_EXHAUSTED, INTERNAL = 0, 3, 5, 6, 8, 13
_CODE_NAMES = {3: "InvalidArgument", 5: "NotFound", 6: "AlreadyExists", 8: "ResourceExhausted",
               13: "Internal"}

COMBINERS = {"sum": 0, "mean": 1, "sqrtn": 2}
ORDER_ALI, ORDER_SEQ = 0, 1
MAX_GROUP = 32
MAX_PARTITIONS = 64
POOL_ONEHOT = 1
POOL_BF16 = 2
POOL_OUT_BF16 = 4
LOOKUP_OUT_BF16 = 1
LOOKUP_TABLE_ORDER = 2
LOOKUP_ROWS_RECORD = 4


class DeepRecError(RuntimeError):
    """Raised for a non-OK status (mirrors tf.errors.*Error by code)."""

    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (_CODE_NAMES.get(code, "Error"), code, msg))
        self.code = code


class InvalidArgumentError(DeepRecError, ValueError):
    pass


class DrPoolDesc(C.Structure):
    _fields_ = [
        ("pool", C.c_void_p), ("pool_rows", C.c_int64), ("ids", C.c_void_p), ("idx", C.c_void_p),
        ("rows", C.c_void_p), ("default_rows", C.c_void_p), ("default_stride", C.c_int64),
        ("bag_off", C.c_void_p),
        ("weights", C.c_void_p), ("out", C.c_void_p), ("out_stride", C.c_int64),
        ("combiner", C.c_int32), ("max_norm", C.c_float),
    ]


class DrPoolGradDesc(C.Structure):
    _fields_ = [
        ("top_grad", C.c_void_p), ("top_stride", C.c_int64), ("bag_off", C.c_void_p),
        ("seg", C.c_void_p), ("seg_stride", C.c_int64), ("idx", C.c_void_p), ("nnz", C.c_int64),
        ("num_unique", C.c_void_p), ("combiner", C.c_int32),
        ("weights", C.c_void_p), ("bag_scale", C.c_void_p),
    ]


class DrEvConfig(C.Structure):
    _fields_ = [
        ("dim", C.c_int64), ("capacity", C.c_int64), ("steps_to_live", C.c_int64),
        ("filter_freq", C.c_int64), ("max_element_size", C.c_int64),
        ("false_positive_probability", C.c_float), ("counter_bits", C.c_int32),
        ("layout", C.c_int32), ("value_bits", C.c_int32),
    ]


MAX_PEERS = 16
IPC_HANDLE_BYTES = 64


class DrXgmiPeers(C.Structure):
    _fields_ = [
        ("world", C.c_int32), ("rank", C.c_int32), ("cap", C.c_int64),
        ("inbox_keys", C.c_void_p * MAX_PEERS), ("inbox_slot", C.c_void_p * MAX_PEERS),
        ("inbox_cnt", C.c_void_p * MAX_PEERS), ("out", C.c_void_p * MAX_PEERS),
    ]


_P, _I64, _I32, _F32, _SZ, _U64 = C.c_void_p, C.c_int64, C.c_int, C.c_float, C.c_size_t, C.c_uint64

# dr_comm_ops.all_to_all_v (include/deeprec_amd.h)
COMM_A2A_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.c_void_p,
                          C.POINTER(C.c_int64), C.c_int64, C.c_void_p)


# dr_comm_ops.all_gather / .barrier
COMM_GATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)
COMM_BARRIER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)


class DrCommOps(C.Structure):
    _fields_ = [("user", C.c_void_p), ("all_to_all_v", COMM_A2A_FN),
                ("all_gather", COMM_GATHER_FN), ("barrier", COMM_BARRIER_FN)]


# dr_sharded_create_ex kinds and config (include/deeprec_amd.h)
SHARDED_RCCL, SHARDED_XGMI, SHARDED_RCCL_FIXED = 0, 1, 2


class DrShardedConfig(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("batch", C.c_int64),
                ("max_ids", C.c_int64)]


class DrDinMlpBuf(C.Structure):
    """dr_din_mlp_buf (include/deeprec_amd.h): the fused DIN attention MLP's
    caller-owned buffers."""
    _fields_ = [(n, C.c_void_p) for n in ("pos", "cnt", "off", "w1p", "w2t", "cq", "h1t", "h2t",
                                          "da1t", "da2t", "xt", "dsc", "dqp", "s1", "dq2")]


RCCL_UNIQUE_ID_BYTES = 128
SHARDED_OUT_BF16 = 1

# name -> (restype, argtypes); must match include/deeprec_amd.h
SIGNATURES = {
    "dr_abi_version": (_I32, []),
    "dr_last_error": (C.c_char_p, []),
    "dr_status_check": (_I32, [_P]),
    "dr_unique_workspace_size": (_SZ, [_I64]),
    "dr_unique": (_I32, [_P, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_unique_grouped_workspace_size": (_SZ, [_P, _I32]),
    "dr_unique_grouped": (_I32, [_P, _P, _I32, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_unique_set_lds_probes": (_I32, [_I32]),
    "dr_kernel_timing": (_I32, [_I32]),
    "dr_kernel_timing_result": (_I32, [_P, _P]),
    "dr_route_workspace_size": (_SZ, [_I64, _I32, _I32]),
    "dr_route_by_owner": (_I32, [_P, _P, _I32, _P, _I32, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_sort_pairs_workspace_size": (_SZ, [_I64]),
    "dr_sort_pairs": (_I32, [_P, _P, _P, _P, _I64, _I32, _I32, _P, _SZ, _P]),
    "dr_gather": (_I32, [_P, _I64, _I64, _P, _I64, _P, _P]),
    "dr_segment_workspace_size": (_SZ, [_I64]),
    "dr_sparse_segment_reduce": (_I32, [_P, _I64, _I64, _P, _P, _I64, _I64, _I32, _P, _P, _SZ, _P]),
    "dr_segment_grad_workspace_size": (_SZ, [_I64, _I64, _I64]),
    "dr_sparse_segment_reduce_grad": (_I32, [_P, _I64, _I64, _P, _P, _I64, _I64, _I32, _P, _P, _SZ,
                                             _P]),
    "dr_unsorted_segment_sum_workspace_size": (_SZ, [_I64, _I64]),
    "dr_unsorted_segment_sum": (_I32, [_P, _I64, _I64, _P, _I64, _P, _P, _SZ, _P]),
    "dr_pool_grouped": (_I32, [_P, _I32, _I64, _I32, _I32, _P]),
    "dr_pool_grouped_ex": (_I32, [_P, _I32, _I64, _I32, _I32, _I32, _P]),
    "dr_bag_offsets": (_I32, [_P, _I64, _I64, _P, _P]),
    "dr_bag_offsets_i32": (_I32, [_P, _I64, _I64, _P, _P]),
    "dr_bag_offsets_strided": (_I32, [_P, _I64, _I64, _I64, _P, _P]),
    "dr_bag_offsets_strided_dev": (_I32, [_P, _I64, _I64, _P, _I64, _P, _P]),
    "dr_bag_offsets_grouped": (_I32, [_P, _P, _P, _I32, _I64, _P, _P]),
    "dr_rows_per_nnz": (_I32, [_P, _P, _P, _I32, _P, _P]),
    "dr_pool_grad_workspace_size": (_SZ, [_I64]),
    "dr_pool_grad_grouped_workspace_size": (_SZ, [_I64]),
    "dr_pool_grad_grouped": (_I32, [_P, _I32, _I64, _I32, _P, _P, _SZ, _P]),
    "dr_pool_grad_rows_workspace_size": (_SZ, [_I64]),
    "dr_pool_grad_rows_grouped": (_I32, [_P, _I32, _I64, _I32, _P, _I64, _P, _I32, _P, _P, _P, _P,
                                         _P, _SZ, _P]),
    "dr_pool_grad_rows_grouped_ex": (_I32, [_P, _I32, _I64, _I32, _P, _I64, _P, _I32, _P, _P, _P,
                                            _P, _P, _P, _SZ, _P]),
    "dr_pool_grad_rows_grouped_ex2": (_I32, [_P, _I32, _I64, _I32, _P, _I32, _I64, _P, _I32, _P,
                                             _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_rows_from_ptr": (_I32, [_P, _I64, _P, _I32, _P, _P]),
    "dr_pool_grad": (_I32, [_P, _I64, _I64, _I32, _P, _P, _P, _I64, _P, _I32, _P, _P, _SZ, _P]),
    "dr_ev_create": (_I32, [_P, _P, _P]),
    "dr_ev_create_slot": (_I32, [_P, _I32, _P, _P]),
    "dr_ev_retain": (_I32, [_P]),
    "dr_ev_release": (_I32, [_P]),
    "dr_ev_size": (_I32, [_P, _P, _P]),
    "dr_ev_dim": (_I64, [_P]),
    "dr_ev_filter_freq": (_I64, [_P]),
    "dr_embedding_lookup_sparse_workspace_size": (_SZ, [_I64, _I64]),
    "dr_embedding_lookup_sparse": (_I32, [_P, _P, _I64, _I32, _P, _P, _P, _I64, _I64, _I32, _F32,
                                          _I32, _I64, _I32, _P, _I64, _P, _SZ, _P]),
    "dr_ev_row_capacity": (_I64, [_P]),
    "dr_ev_value_bits": (_I32, [_P]),
    "dr_ev_lock_updates": (_I32, [_P, _I32, _P]),
    "dr_ev_unlock_updates": (_I32, [_P, _I32, _P]),
    "dr_ev_gather_i32_workspace_size": (_SZ, [_I64]),
    "dr_ev_gather_i32": (_I32, [_P, _P, _I64, _P, _P, _P, _P, _SZ, _P]),
    "dr_ev_insert_i32": (_I32, [_P, _P, _I64, _P, _P, _P, _I64, _I64, _P]),
    "dr_ev_export_i32": (_I32, [_P, _P, _P, _P, _P, _I64, _P, _P]),
    "dr_unique_i32_workspace_size": (_SZ, [_I64]),
    "dr_unique_i32": (_I32, [_P, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_ev_shrink": (_I32, [_P, _I64, _F32, _P, _P]),
    "dr_ev_reserve": (_I32, [_P, _I64, _P]),
    "dr_ev_resolve_workspace_size": (_SZ, [_I64]),
    "dr_ev_resolve": (_I32, [_P, _P, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_ev_resolve_grouped": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_ev_lookup_onehot_workspace_size": (_SZ, [_I32, _I64]),
    "dr_ev_lookup_onehot": (_I32, [_P, _I32, _P, _I64, _P, _I64, _I32, _P, _SZ, _P]),
    "dr_ev_lookup_onehot_rows": (_I32, [_P, _I32, _P, _I64, _P, _I64, _I32, _P, _P, _SZ, _P]),
    "dr_ev_lookup_onehot_ex": (_I32, [_P, _I32, _P, _I64, _I64, _I64, _P, _I64, _I32, _I32, _P,
                                      _P, _SZ, _P]),
    "dr_ev_lookup_onehot_strided": (_I32, [_P, _I32, _P, _I64, _I64, _I64, _P, _I64, _I32, _P, _P,
                                           _SZ, _P]),
    "dr_ev_resolve_tagged": (_I32, [_P, _I32, _P, _P, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "dr_ev_gather_tagged": (_I32, [_P, _I32, _P, _P, _I64, _P, _P, _P]),
    "dr_ev_pool": (_P, [_P]),
    "dr_ev_default_row": (_P, [_P]),
    "dr_ev_gather_workspace_size": (_SZ, [_I64]),
    "dr_ev_gather": (_I32, [_P, _P, _I64, _P, _P, _P, _P, _SZ, _P]),
    "dr_ev_insert": (_I32, [_P, _P, _I64, _P, _P, _P, _I64, _I64, _P]),
    "dr_ev_insert_synthetic": (_I32, [_P, _I64, _I64, _I64, _U64, _P]),
    "dr_ev_export": (_I32, [_P, _P, _P, _P, _P, _I64, _P, _P]),
    "dr_ev_key_meta": (_I32, [_P, _P, _I64, _P, _P, _P, _P]),
    "dr_ev_apply_sgd": (_I32, [_P, _F32, _P, _P, _I64, _P, _I64, _P]),
    "dr_ev_apply_adagrad": (_I32, [_P, _P, _F32, _P, _P, _I64, _P, _I64, _P]),
    "dr_ev_apply_adam": (_I32, [_P, _P, _P, _F32, _F32, _F32, _F32, _F32, _F32, _P, _P, _I64, _P,
                                _I64, _P]),
    "dr_ev_apply_grouped": (_I32, [_I32, _P, _P, _P, _I32, _P, _P, _P, _P, _F32, _F32, _F32,
                                   _F32, _F32, _F32, _I64, _P]),
    "dr_ev_apply_grouped_ptr": (_I32, [_I32, _P, _P, _P, _I32, _P, _P, _P, _P, _F32, _F32, _F32,
                                       _F32, _F32, _F32, _I64, _P]),
    "dr_ev_apply_grouped_ptr_rows": (_I32, [_I32, _P, _I32, _P, _P, _P, _P, _P, _F32, _I64, _P]),
    "dr_ev_pool_grad_rows_sgd_workspace_size": (_SZ, [_I64, _I32]),
    "dr_ev_pool_grad_rows_apply_sgd": (_I32, [_P, _P, _I32, _I64, _I32, _P, _F32, _I64, _P, _SZ,
                                              _P]),
    "dr_ev_pool_grad_rows_apply_sgd_ex": (_I32, [_P, _P, _I32, _I64, _I32, _P, _I32, _F32, _I64,
                                                 _P, _SZ, _P]),
    "dr_ev_apply_adam_async_grouped": (_I32, [_I32, _I32, _P, _P, _P, _I32, _P, _P, _P, _P, _P,
                                              _F32, _F32, _F32, _F32, _I64, _P]),
    "dr_ev_apply_adam_grouped_dev": (_I32, [_I32, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _F32,
                                            _F32, _F32, _F32, _I64, _P]),
    "dr_ev_apply_adagrad_decay_grouped": (_I32, [_P, _P, _P, _I32, _P, _I32, _P, _P, _P, _F32,
                                                 _I64, _F32, _F32, _I64, _P]),
    "dr_ev_apply_ftrl_grouped_ptr": (_I32, [_P, _P, _P, _I32, _P, _P, _P, _P, _F32, _F32, _F32,
                                            _F32, _F32, _I64, _P]),
    "dr_ev_apply_ftrl": (_I32, [_P, _P, _P, _F32, _F32, _F32, _F32, _F32, _P, _P, _I64, _P, _I64,
                                _P]),
    "dr_ev_apply_ftrl_grouped": (_I32, [_P, _P, _P, _I32, _P, _P, _P, _P, _F32, _F32, _F32, _F32,
                                        _F32, _I64, _P]),
    "dr_fused_local_workspace_size": (_SZ, [_I64]),
    "dr_fused_local_lookup": (_I32, [_P, _I64, _I32, _P, _P, _I64, _I64, _I32, _F32, _P, _P, _P,
                                     _SZ, _P]),
    "dr_fused_local_lookup_grad": (_I32, [_P, _P, _I64, _I32, _P, _P, _I64, _I64, _I32, _F32, _P,
                                          _P]),
    "dr_bag_weight_scale": (_I32, [_P, _P, _I64, _I32, _P, _P]),
    "dr_clip_by_norm_grad": (_I32, [_P, _I64, _P, _P, _I64, _P, _I64, _I32, _F32, _P, _P]),
    "dr_fused_pre_lookup_workspace_size": (_SZ, [_I64]),
    "dr_fused_pre_lookup": (_I32, [_P, _P, _I64, _P, _I32, _P, _P, _P, _P, _SZ, _P]),
    "dr_fused_post_lookup_workspace_size": (_SZ, [_I64, _I64]),
    "dr_fused_post_lookup": (_I32, [_P, _P, _P, _I32, _I64, _I64, _I32, _I32, _F32, _P, _P, _P,
                                    _SZ, _P]),
    "dr_fused_post_lookup_grad": (_I32, [_P, _P, _P, _P, _I32, _I64, _I32, _P, _I32, _F32, _P,
                                         _P]),
    "dr_partition_by_owner_mod": (_I32, [_P, _I64, _P, _I32, _I64, _P, _P, _P, _P, _SZ, _P]),
    "dr_partition_workspace_size": (_SZ, [_I64]),
    "dr_partition_by_owner": (_I32, [_P, _I64, _P, _I32, _P, _P, _P, _P, _SZ, _P]),
    "dr_rows_scatter": (_I32, [_P, _P, _I64, _P, _I32, _P, _P]),
    "dr_rows_pack": (_I32, [_P, _P, _I64, _P, _I32, _P, _P]),
    "dr_ipc_export": (_I32, [_P, _P, _P]),
    "dr_ipc_import": (_I32, [_P, _I64, _P, _P]),
    "dr_ipc_close": (_I32, [_P]),
    "dr_ipc_alloc": (_I32, [_SZ, _P]),
    "dr_ipc_free": (_I32, [_P]),
    "dr_ipc_alloc_dlpack": (_I32, [_I32, _P, _I32, _I32, _I32, _P]),
    "dr_xgmi_route": (_I32, [_P, _P, _I32, _I64, _P, _P]),
    "dr_xgmi_route_ex": (_I32, [_P, _P, _I32, _I64, _P, _P, _P]),
    "dr_xgmi_serve_workspace_size": (_SZ, [_I32, _I64]),
    "dr_xgmi_serve": (_I32, [_P, _P, _I32, _I64, _P, _SZ, _P]),
    "dr_xgmi_grad_pull_workspace_size": (_SZ, [_I32, _I64]),
    "dr_xgmi_grad_pull": (_I32, [_P, _P, _P, _I32, _I64, _I32, _P, _P, _P, _P, _SZ, _P]),
    "dr_xgmi_grad_pull_dev_workspace_size": (_SZ, [_I32, _I64]),
    "dr_xgmi_grad_pull_dev": (_I32, [_P, _P, _I32, _I64, _I32, _P, _P, _P, _P, _SZ, _P]),
    "dr_comm_rccl_unique_id": (_I32, [_P, _I64]),
    "dr_comm_init": (_I32, [_P, _I32, _I32, _P, _P]),
    "dr_comm_destroy": (_I32, [_P]),
    "dr_comm_rank": (_I32, [_P]),
    "dr_comm_world": (_I32, [_P]),
    "dr_comm_all_to_all_v": (_I32, [_P, _P, _P, _P, _P, _I64, _P]),
    "dr_sharded_create": (_I32, [_P, _P, _I32, _P]),
    "dr_sharded_destroy": (_I32, [_P]),
    "dr_sharded_forward": (_I32, [_P, _P, _P, _P, _I64, _I32, _I32, _I32, _P, _P]),
    "dr_sharded_backward": (_I32, [_P, _P, _P, _P, _P, _P]),
    "dr_sharded_last_stats": (_I32, [_P, _P, _P]),
    "dr_sharded_create_ex": (_I32, [_P, _P, _I32, _P, _P]),
    "dr_dlpack_view": (_I32, [_P, _I32, _P, _I32, _I32, _I32, _P]),
    "dr_sharded_output": (_I32, [_P, _P]),
    "dr_sharded_backward_dev": (_I32, [_P, _P, _P, _P, _P, _P, _P]),
    "dr_memcpy": (_I32, [_P, _P, _I64, _I32, _P]),
    "dr_fm2": (_I32, [_P, _I64, _I32, _I32, _P, _P]),
    "dr_fm2_grad": (_I32, [_P, _P, _I64, _I32, _I32, _P, _P]),
    "dr_fm2_bf16_copy": (_I32, [_P, _I64, _I32, _I32, _P, _P, _P]),
    "dr_fm2_grad_add_bf16": (_I32, [_P, _P, _P, _I64, _I64, _I32, _I32, _P, _P]),
    "dr_dot_interaction": (_I32, [_P, _I64, _I32, _I32, _P, _P]),
    "dr_dot_interaction_grad": (_I32, [_P, _P, _I64, _I32, _I32, _P, _P]),
    "dr_dot_interaction_concat_bf16": (_I32, [_P, _I64, _I32, _I32, _P, _I64, _P]),
    "dr_dot_interaction_concat_grad_bf16": (_I32, [_P, _P, _I64, _I64, _I32, _I32, _P, _P]),
    "dr_crossnet_layer_bf16": (_I32, [_P, _P, _P, _P, _I64, _I32, _P, _P]),
    "dr_crossnet_forward_bf16": (_I32, [_P, _P, _P, _P, _I64, _I32, _P, _P, _P]),
    "dr_crossnet_backward_workspace_size": (_SZ, [_I64, _I32]),
    "dr_crossnet_dx_bf16": (_I32, [_P, _P, _P, _I64, _I32, _P, _P]),
    "dr_gemm_nt_workspace_size": (_SZ, [_I64, _I64, _I32]),
    "dr_gemm_nt_bf16": (_I32, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I32, _P, _I64, _I32,
                               _I32, _P, _SZ, _P]),
    "dr_gemm_nt_bf16_ex": (_I32, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I32, _P, _I64, _P,
                                  _I64, _I32, _I32, _P, _SZ, _P]),
    "dr_transpose_bf16": (_I32, [_P, _I64, _I64, _I64, _P, _I64, _P]),
    "dr_transpose_bf16_colsum": (_I32, [_P, _I64, _I64, _I64, _P, _I64, _P, _P]),
    "dr_mlp_head_forward_bf16": (_I32, [_P, _I64, _I64, _I32, _P, _I32, _P, _P, _P]),
    "dr_mlp_head_grad_partials": (_SZ, [_I64]),
    "dr_gemm_tn_workspace_size": (_SZ, [_I64, _I64, _I32, _I32]),
    "dr_gemm_tn_bf16": (_I32, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I32, _P, _SZ,
                               _P]),
    "dr_relu_grad_bf16": (_I32, [_P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P]),
    "dr_mlp_head_backward_bf16": (_I32, [_P, _I64, _I64, _I32, _P, _I32, _P, _P, _I64, _P, _P,
                                         _P]),
    "dr_crossnet_backward_elem_bf16": (_I32, [_P, _P, _P, _P, _P, _P, _P, _I64, _I32, _P, _SZ,
                                              _P]),
    "dr_din_attention_input": (_I32, [_P, _P, _I64, _I64, _I32, _P, _P]),
    "dr_din_attention_input_grad": (_I32, [_P, _P, _P, _I64, _I64, _I32, _P, _P, _I32, _P]),
    "dr_din_attention_pool": (_I32, [_P, _P, _P, _I64, _I64, _I32, _P, _P, _P, _P]),
    "dr_din_dice_forward": (_I32, [_P, _P, _I64, _I32, _F32, _P, _P, _P]),
    "dr_din_fcn_input_forward": (_I32, [_P, _P, _P, _P, _P, _P, _I64, _I32, _I32, _F32, _P, _P]),
    "dr_din_fcn_input_backward": (_I32, [_P, _P, _P, _P, _P, _P, _I64, _I32, _I32, _F32, _P, _P,
                                         _P, _P, _P, _P, _P]),
    "dr_din_dice_backward": (_I32, [_P, _P, _P, _P, _I64, _I32, _F32, _P, _P, _P]),
    "dr_din_attention_pool_grad": (_I32, [_P, _P, _P, _P, _P, _I64, _I64, _I32, _P, _P, _P]),
    "dr_crossnet_dw_workspace_size": (_SZ, [_I64, _I32]),
    "dr_crossnet_dw_bf16": (_I32, [_P, _P, _I64, _I32, _P, _P, _SZ, _P]),
    "dr_din_mlp_forward": (_I32, [_P, _P, _P, _I64, _I64, _I32, _P, _P, _I32, _P, _P, _I32, _P,
                                  _P, _P, _P, _P]),
    "dr_din_mlp_backward": (_I32, [_P, _P, _I64, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "dr_din_mlp_backward_tail": (_I32, [_P, _P, _I64, _I64, _I32, _I32, _I32, _P, _P, _P, _P,
                                        _I32, _P]),
    "dr_din_mlp_wgrad_workspace_size": (_SZ, [_I32, _I32, _I32]),
    "dr_din_mlp_wgrad": (_I32, [_P, _P, _P, _P, _P, _P, _I64, _I32, _I32, _I32, _P, _P, _SZ, _P]),
    "dr_din_mlp_wgrad_valid": (_I32, [_P, _P, _P, _P, _P, _P, _I64, _P, _I32, _I32, _I32, _P, _P,
                                      _SZ, _P]),
    "dr_fingerprint64": (_I32, [_P, _P, _I64, _P, _P]),
    "dr_string_to_hash_bucket_fast": (_I32, [_P, _P, _I64, _I64, _P, _P]),
    "dr_crc32c_extend": (C.c_uint32, [C.c_uint32, _P, _SZ]),
    "dr_sparse_fill_workspace_size": (_SZ, [_I64, _I64]),
    "dr_sparse_prune_fill": (_I32, [_P, _I32, _P, _P, _I64, _I64, _I32, _I64, _F32, _P, _P, _P,
                                    _P, _P, _P, _P, _SZ, _P]),
    "dr_fill_synthetic": (_I32, [_P, _I64, _I32, _U64, _P]),
    "dr_synth_value": (_F32, [_U64, _I64, _I64]),
}

_lib = None


def load():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DeepRecError(INTERNAL, "HIP extension %s not built; run "
                                         "`make -C deeprec-1_amd` or __graft_entry__.build()"
                               % LIB_PATH)
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def lib():
    return _lib if _lib is not None else load()


def check(rc):
    if rc != OK:
        msg = lib().dr_last_error()
        msg = msg.decode() if msg else ""
        if rc == INVALID_ARGUMENT:
            raise InvalidArgumentError(rc, msg)
        raise DeepRecError(rc, msg)


def require_gpu():
    if not torch.cuda.is_available():
        raise DeepRecError(INTERNAL, "deeprec_amd ops need an MI355X (no GPU visible); "
                                     "there is no CPU fallback")


def ptr(t):
    """Device pointer of a tensor (None passes through as NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


_DL_CODES = {torch.int64: (0, 64), torch.int32: (0, 32), torch.float32: (2, 32),
             torch.bfloat16: (4, 16)}


def uncached_empty(shape, dtype, device):
    """A zero-filled torch tensor in UNCACHED device memory (dr_ipc_alloc):
    for buffers that peer GPUs write or read over xGMI.  Owned by torch
    through DLPack; freed by the library's deleter."""
    from torch.utils import dlpack
    code, bits = _DL_CODES[dtype]
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    shp = (C.c_int64 * len(shape))(*[int(x) for x in shape])
    m = C.c_void_p()
    with torch.cuda.device(idx):
        check(lib().dr_ipc_alloc_dlpack(len(shape), shp, code, bits, idx, C.byref(m)))
    new = C.pythonapi.PyCapsule_New
    new.restype = C.py_object
    new.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p]
    return dlpack.from_dlpack(new(m, b"dltensor", None))


def device_view(address, shape, dtype, device):
    """A torch tensor viewing library-owned device memory (dr_dlpack_view; it
    owns nothing: keep the owner alive while the view is used)."""
    from torch.utils import dlpack
    code, bits = _DL_CODES[dtype]
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    shp = (C.c_int64 * len(shape))(*[int(x) for x in shape])
    m = C.c_void_p()
    check(lib().dr_dlpack_view(C.c_void_p(address), len(shape), shp, code, bits, idx,
                               C.byref(m)))
    new = C.pythonapi.PyCapsule_New
    new.restype = C.py_object
    new.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p]
    return dlpack.from_dlpack(new(m, b"dltensor", None))


def status_check(device=None):
    """Synchronise and raise if a kernel latched an error (OP_REQUIRES)."""
    check(lib().dr_status_check(stream_handle(device)))
