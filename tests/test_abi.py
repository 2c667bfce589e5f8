"""CPU-side checks of the drop-in boundary: the C-ABI library is built for
gfx950, loads, and exports every entry point include/deeprec_amd.h declares;
the Python mirror imports and refuses to run without a GPU (no CPU fallback).
No compute calls are made here (there is no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "deeprec_amd.h")
LIB = os.path.join(ROOT, "deeprec-1_amd", "deeprec_amd", "libdeeprec_amd.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dr_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def built_lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "deeprec-1_amd")])
    return LIB


def test_header_declares_core_entry_points():
    names = declared_functions()
    for required in ("dr_unique", "dr_ev_gather", "dr_ev_insert", "dr_ev_export",
                     "dr_sparse_segment_reduce", "dr_sparse_segment_reduce_grad",
                     "dr_unsorted_segment_sum", "dr_pool_grouped", "dr_ev_apply_adam",
                     "dr_fused_local_lookup", "dr_partition_by_owner", "dr_fm2",
                     "dr_crossnet_layer_bf16"):
        assert required in names


def test_library_exports_every_declared_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_is_gfx950_code_object(built_lib):
    # the fat binary embeds an amdgcn-amd-amdhsa--gfx950 code object
    data = open(built_lib, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_python_mirror_signatures_match_header():
    import deeprec_amd._lib as L
    declared = set(declared_functions())
    assert set(L.SIGNATURES) <= declared
    # every declared compute entry point is bound
    unbound = declared - set(L.SIGNATURES)
    assert not unbound, unbound


def test_ops_refuse_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import deeprec_amd
    with pytest.raises(deeprec_amd.DeepRecError):
        deeprec_amd.EmbeddingVariable("x", 4, 0.0)
    from deeprec_amd import ops
    with pytest.raises(deeprec_amd.DeepRecError):
        ops.unique(torch.arange(4))


def test_abi_version_without_device(built_lib):
    lib = ctypes.CDLL(built_lib)
    lib.dr_abi_version.restype = ctypes.c_int
    assert lib.dr_abi_version() == 2


def test_synth_rows_restatement_matches_library(built_lib):
    """The numpy synth(seed, key, col) used by the headline-size parity checks
    (oracle.synth_rows, bench.synth_rows) equals the library's host synth."""
    import sys
    import numpy as np
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "deeprec-1_amd"))
    import bench
    from oracle import oracle as orc
    L = ctypes.CDLL(built_lib)
    L.dr_synth_value.restype = ctypes.c_float
    L.dr_synth_value.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64]
    keys = np.array([0, 1, 7, 12_499_999, 99_999_999_999, 2 ** 40 + 3], np.int64)
    for seed in (1000, 1025):
        want = np.array([[L.dr_synth_value(seed, int(k), c) for c in range(128)] for k in keys],
                        np.float32)
        np.testing.assert_array_equal(orc.synth_rows(seed, keys, 128), want)
        np.testing.assert_array_equal(bench.synth_rows(seed, keys, 128), want)
